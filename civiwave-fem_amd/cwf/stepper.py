"""Mirror of ``cwf::gpu::newmark::Stepper`` (include/cwf/gpu/newmark_stepper.hpp:92-190).

Node state (u, v, a), predictor, external force and Dirichlet values live in HBM; ``step()``
runs predictor -> effective RHS (+ beta_R K d) -> Dirichlet clamp -> PCG -> corrector ->
adaptive dt on the GPU (src/gpu/newmark_stepper.cpp:1094-1160, CPU-branch arithmetic).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib
from .pcg import Expected, MatrixFreeSystem, PcgTelemetry
from .physics import RayleighCoefficients, SolverSettings, TimeSettings


@dataclass
class AdaptivePolicy:
    low_iteration_ratio: float = 0.3
    increase_factor: float = 1.1
    decrease_factor: float = 0.5


@dataclass
class StepError:
    message: str
    context: list


@dataclass
class StepTelemetry:
    simulation_time: float
    time_step: float
    applied_tolerance: float
    paused_mode: bool
    dt_increased: bool
    dt_decreased: bool
    dt_clamped_min: bool
    dt_clamped_max: bool
    pcg: PcgTelemetry


class Stepper:
    """Stepper(packing, materials, rayleigh, solver_settings, time_settings, adaptive_policy)."""

    DISPLACEMENT, VELOCITY, ACCELERATION, SOLUTION, EXTERNAL_FORCE = 0, 1, 2, 3, 4

    def __init__(self, packing, materials, rayleigh: RayleighCoefficients, solver_settings: SolverSettings,
                 time_settings: TimeSettings, adaptive_policy: AdaptivePolicy | None = None,
                 mode: int = _lib.MODE_PARITY, device: int = 0, system: MatrixFreeSystem | None = None):
        pol = adaptive_policy or AdaptivePolicy()
        self.packing = packing
        self.system = system or MatrixFreeSystem.from_packing(packing, materials, 1.0, 0.0, mode, device)
        h = self.system.handle()
        self._f = np.ascontiguousarray(packing.external_force, np.float32)
        self._bcv = np.ascontiguousarray(packing.bc_value, np.float32)
        d = _lib.StepperDescC(rayleigh.alpha, rayleigh.beta, solver_settings.runtime_tolerance,
                              solver_settings.pause_tolerance, int(solver_settings.max_iterations),
                              time_settings.initial_dt, int(time_settings.adaptive), 1, time_settings.min_dt,
                              time_settings.max_dt, pol.low_iteration_ratio, pol.increase_factor,
                              pol.decrease_factor, _lib.ptr(self._f), _lib.ptr(self._bcv))
        st = C.c_void_p()
        rc = _lib.load().cwf_hip_stepper_create(h, C.byref(d), C.byref(st))
        if rc:
            msg, ctx = _lib.last_error(h)
            raise RuntimeError(f"stepper create failed: {msg} {ctx}")
        self._st = st
        self.dof_count = packing.dof_count
        self.node_count = packing.node_count

    def step(self, simulation_time_seconds: float, paused_mode: bool = False) -> Expected:
        t = _lib.StepTelemetryC()
        rc = _lib.load().cwf_hip_stepper_step(self._st, simulation_time_seconds, int(paused_mode), C.byref(t))
        if rc:
            msg, ctx = _lib.last_error(self.system._h)
            return Expected(error=StepError(msg, ctx))
        return Expected(StepTelemetry(t.simulation_time, t.time_step, t.applied_tolerance, bool(t.paused_mode),
                                      bool(t.dt_increased), bool(t.dt_decreased), bool(t.dt_clamped_min),
                                      bool(t.dt_clamped_max), PcgTelemetry.from_c(t.pcg)))

    def _times(self):
        ct, dt = C.c_double(), C.c_double()
        _lib.load().cwf_hip_stepper_time(self._st, C.byref(ct), C.byref(dt))
        return ct.value, dt.value

    def current_time(self) -> float:
        return self._times()[0]

    def time_step(self) -> float:
        return self._times()[1]

    def set_warm_start(self, enabled: bool):
        _lib.load().cwf_hip_stepper_set_warm_start(self._st, int(enabled))

    def get_state(self, which: int, out=None):
        if out is None:
            out = np.zeros(self.dof_count, np.float32)
        kind = _lib.PTR_HOST if isinstance(out, np.ndarray) else _lib.PTR_DEVICE
        rc = _lib.load().cwf_hip_stepper_get_state(self._st, which, _lib.ptr(out), self.dof_count, kind)
        if rc:
            raise RuntimeError(_lib.last_error(self.system._h))
        return out

    def set_state(self, which: int, values):
        kind = _lib.PTR_HOST if isinstance(values, np.ndarray) else _lib.PTR_DEVICE
        if isinstance(values, np.ndarray):
            values = np.ascontiguousarray(values, np.float32)
        rc = _lib.load().cwf_hip_stepper_set_state(self._st, which, _lib.ptr(values), self.dof_count, kind)
        if rc:
            raise RuntimeError(_lib.last_error(self.system._h))

    def set_external_force(self, force):
        """Rewrite nodes.external_force between steps (the viewer does this, viewer.cpp:262-266)."""
        kind = _lib.PTR_HOST if isinstance(force, np.ndarray) else _lib.PTR_DEVICE
        if isinstance(force, np.ndarray):
            force = np.ascontiguousarray(force, np.float32)
        rc = _lib.load().cwf_hip_stepper_set_external_force(self._st, _lib.ptr(force), self.dof_count, kind)
        if rc:
            raise RuntimeError(_lib.last_error(self.system._h))

    def set_load_pattern(self, base: np.ndarray, pattern: np.ndarray):
        """Device-side time-varying load (cwf_hip_stepper_set_load_pattern): f64 [3N] loads no curve scales and
        the point-load values one curve scales; set_load_scale(c) then packs f32(base + c * pattern)."""
        self._lbase = np.ascontiguousarray(base, np.float64)
        self._lpat = np.ascontiguousarray(pattern, np.float64)
        rc = _lib.load().cwf_hip_stepper_set_load_pattern(self._st, _lib.ptr(self._lbase), _lib.ptr(self._lpat),
                                                          self.dof_count)
        if rc:
            raise RuntimeError(_lib.last_error(self.system._h))

    def set_load_scale(self, scale: float):
        rc = _lib.load().cwf_hip_stepper_set_load_scale(self._st, float(scale))
        if rc:
            raise RuntimeError(_lib.last_error(self.system._h))

    def close(self):
        if getattr(self, "_st", None) is not None:
            _lib.load().cwf_hip_stepper_destroy(self._st)
            self._st = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
