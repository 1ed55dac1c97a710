"""Post stack mirror: ``cwf::post`` (include/cwf/post/*.hpp) over the C-ABI.

* ``compute_derived_fields`` -- derived_fields.cpp:139-211, computed on the GPU by the handle's
  ``cwf_hip_derived_fields`` kernels (bit-exact with the reference's fp64 arithmetic);
* ``write_vtu`` -- vtu_writer.cpp:171-297, the reference's binary-appended VTU byte for byte;
* ``ProbeLogger`` -- probe_logger.cpp:60-124, CSV rows with ``%.9f`` fields;
* ``OutputManager`` -- output_manager.cpp:36-87: derived fields every frame, ``vtu/frame_%05u.vtu``
  every ``vtu_stride`` frames, ``probes/probes.csv``; errors are wrapped as ``"vtu: ..."`` /
  ``"probes: ..."`` like the reference.

Per-element / per-node fields are f32 [count, 13] arrays {strain[6], stress[6], von_mises}, the
memory layout of ``ElementField`` / ``NodeField`` (derived_fields.hpp:37-55).
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass, field

import numpy as np

from . import _lib
from .pcg import Expected, MatrixFreeSystem


@dataclass
class PostError:
    message: str
    context: list = field(default_factory=list)


@dataclass
class DerivedFieldSet:
    elements: np.ndarray  # f32 [E, 13]
    nodes: np.ndarray  # f32 [N, 13]

    @staticmethod
    def strain(a):
        return a[:, 0:6]

    @staticmethod
    def stress(a):
        return a[:, 6:12]

    @staticmethod
    def von_mises(a):
        return a[:, 12]


def compute_derived_fields(packing, materials=None, system: MatrixFreeSystem | None = None,
                           displacement=None) -> DerivedFieldSet:
    """derived_fields.cpp:139 compute_derived_fields(packing, materials) on the device.

    ``system`` is the handle whose element tables are used (one is created from ``packing`` /
    ``materials`` when omitted); ``displacement`` defaults to ``packing.displacement`` and may be a
    device tensor (e.g. the Stepper's state)."""
    own = system is None
    if own:
        hex8 = packing.element_count and int(packing.connectivity[4]) != 0xFFFFFFFF  # native hex8: FAST only
        system = MatrixFreeSystem.from_packing(packing, materials, 1.0, 0.0,
                                               _lib.MODE_FAST if hex8 else _lib.MODE_PARITY)
    try:
        u = packing.displacement if displacement is None else displacement
        ukind = _lib.PTR_HOST if isinstance(u, np.ndarray) else _lib.PTR_DEVICE
        if isinstance(u, np.ndarray):
            u = np.ascontiguousarray(u, np.float32)
        el = np.zeros((packing.element_count, 13), np.float32)
        nd = np.zeros((packing.node_count, 13), np.float32)
        h = system.handle()
        rc = _lib.load().cwf_hip_derived_fields(h, _lib.ptr(u), 3 * packing.node_count, ukind, _lib.ptr(el),
                                                 _lib.ptr(nd), _lib.PTR_HOST)
        if rc:
            msg, ctx = _lib.last_error(h)
            raise RuntimeError(f"derived fields failed: {msg} {ctx}")
        return DerivedFieldSet(el, nd)
    finally:
        if own:
            system.close()


def _frame(packing, derived: DerivedFieldSet, keep: list) -> _lib.FrameViewC:
    arrs = [np.ascontiguousarray(np.asarray(packing.position0, np.float32).reshape(-1)),
            np.ascontiguousarray(packing.displacement, np.float32).reshape(-1),
            np.ascontiguousarray(packing.velocity, np.float32).reshape(-1),
            np.ascontiguousarray(packing.acceleration, np.float32).reshape(-1),
            np.ascontiguousarray(derived.elements, np.float32),
            np.ascontiguousarray(derived.nodes, np.float32),
            np.ascontiguousarray(packing.connectivity, np.uint32)]
    keep.extend(arrs)
    p = _lib.ptr
    return _lib.FrameViewC(packing.node_count, packing.element_count, *(p(a) for a in arrs))


def write_vtu(path, packing, derived: DerivedFieldSet, simulation_time: float, frame_index: int) -> Expected:
    """vtu_writer.cpp:171 write_vtu(path, mesh, packing, derived, time, frame); the cells are the packed
    connectivity (the mesh's tet4 elements in mesh order)."""
    keep: list = []
    f = _frame(packing, derived, keep)
    rc = _lib.load().cwf_write_vtu(os.fsencode(str(path)), C.byref(f), float(simulation_time), int(frame_index))
    if rc:
        msg, ctx = _lib.last_error(None)
        return Expected(error=PostError(msg, ctx))
    return Expected(True)


class ProbeLogger:
    """probe_logger.hpp:29-45 ProbeLogger(path, probes).log_frame(time, frame, packing, derived)."""

    def __init__(self, path, probes):
        self.path = str(path)
        self.probes = np.ascontiguousarray(list(probes), np.uint32)
        self._header = C.c_int(0)

    def log_frame(self, simulation_time: float, frame_index: int, packing, derived: DerivedFieldSet) -> Expected:
        keep: list = []
        f = _frame(packing, derived, keep)
        rc = _lib.load().cwf_probe_log_frame(os.fsencode(self.path), C.byref(self._header), _lib.ptr(self.probes),
                                              len(self.probes), C.byref(f), float(simulation_time),
                                              int(frame_index))
        if rc:
            msg, ctx = _lib.last_error(None)
            return Expected(error=PostError(msg, ctx))
        return Expected(True)


class OutputManager:
    """output_manager.hpp:29-52 OutputManager(root, mesh, packing, materials, settings).

    ``system`` (optional) is the solver handle whose HBM-resident element tables compute the derived
    fields; ``stepper`` (optional) makes ``handle_frame`` pull u/v/a from the device state first (the
    viewer copies the stepper state into the packing before exporting, viewer.cpp:262-277)."""

    def __init__(self, root, mesh, packing, materials, settings, system: MatrixFreeSystem | None = None,
                 stepper=None):
        self.root = str(root)
        self.mesh = mesh
        self.packing = packing
        self.materials = materials
        self.settings = settings
        self.stepper = stepper
        self.system = system if system is not None else (stepper.system if stepper is not None else None)
        self._own = self.system is None
        if self._own:
            self.system = MatrixFreeSystem.from_packing(packing, materials, 1.0, 0.0, _lib.MODE_PARITY)
        self.probe_logger = ProbeLogger(os.path.join(self.root, "probes", "probes.csv"), settings.probes)

    def _write_vtu_frame(self, derived, simulation_time, frame_index) -> Expected:
        stride = int(self.settings.vtu_stride)
        if stride == 0 or frame_index % stride != 0:
            return Expected(True)
        path = os.path.join(self.root, "vtu", f"frame_{frame_index:05d}.vtu")
        r = write_vtu(path, self.packing, derived, simulation_time, frame_index)
        if not r.has_value():
            return Expected(error=PostError("vtu: " + r.error().message, r.error().context))
        return r

    def handle_frame(self, simulation_time: float, frame_index: int) -> Expected:
        if self.stepper is not None:
            from .stepper import Stepper
            self.packing.displacement = self.stepper.get_state(Stepper.DISPLACEMENT)
            self.packing.velocity = self.stepper.get_state(Stepper.VELOCITY)
            self.packing.acceleration = self.stepper.get_state(Stepper.ACCELERATION)
        derived = compute_derived_fields(self.packing, self.materials, system=self.system)
        r = self._write_vtu_frame(derived, simulation_time, frame_index)
        if not r.has_value():
            return r
        p = self.probe_logger.log_frame(simulation_time, frame_index, self.packing, derived)
        if not p.has_value():
            return Expected(error=PostError("probes: " + p.error().message, p.error().context))
        return Expected(True)

    def close(self):
        if self._own and self.system is not None:
            self.system.close()
            self.system = None
