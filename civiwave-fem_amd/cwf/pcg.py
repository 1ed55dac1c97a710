"""Mirror of ``cwf::gpu::pcg`` (include/cwf/gpu/pcg.hpp) over the HIP C-ABI.

Same names, argument meaning and error behaviour as the reference:
``apply_keff(system, input, output, workspace)``, ``solve_pcg(system, rhs, settings, vectors,
workspace)`` and ``build_block_jacobi_inverse(system, workspace, out_inverse)`` return an
``Expected`` (std::expected analogue) whose error is a ``PcgError{message, context}`` with the
reference's texts. All arithmetic runs in libcwf_hip.so on the GPU; there is no CPU path.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from typing import Any

import numpy as np

from . import _lib


@dataclass
class PcgError:
    message: str
    context: list = field(default_factory=list)


class Expected:
    """std::expected<T, E> analogue: has_value()/value()/error(), truthy on success."""

    def __init__(self, value: Any = None, error: Any = None):
        self._value, self._error = value, error

    def has_value(self) -> bool:
        return self._error is None

    __bool__ = has_value

    def value(self):
        if self._error is not None:
            raise RuntimeError(f"bad expected access: {self._error}")
        return self._value

    def error(self):
        return self._error

    def __repr__(self):
        return f"Expected(value={self._value!r})" if self.has_value() else f"Unexpected({self._error!r})"


@dataclass
class PcgSettings:
    max_iterations: int = 128
    relative_tolerance: float = 3.0e-4
    warm_start: bool = False


@dataclass
class PcgTelemetry:
    iterations: int = 0
    residual_norm: float = 0.0
    rhs_norm: float = 0.0
    alpha_last: float = 0.0
    beta_last: float = 0.0
    converged: bool = False

    @classmethod
    def from_c(cls, t) -> "PcgTelemetry":
        return cls(int(t.iterations), t.residual_norm, t.rhs_norm, t.alpha_last, t.beta_last, bool(t.converged))


@dataclass
class PcgVectors:
    solution: np.ndarray
    residual: np.ndarray
    search_direction: np.ndarray | None = None
    preconditioned: np.ndarray | None = None
    matvec: np.ndarray | None = None
    partials: np.ndarray | None = None


@dataclass
class MatrixFreeWorkspace:
    """Device scratch lives in the HIP handle; kept for signature parity (pcg.hpp:91-97)."""

    block_inverse: np.ndarray | None = None


class MatrixFreeSystem:
    """cwf::gpu::pcg::MatrixFreeSystem (pcg.hpp:67-86) bound to one HIP handle (one device,
    one stream). Arrays are copied to HBM on first use; stiffness_scale / mass_factor may be
    changed freely between calls (they are pushed to the handle before every call)."""

    def __init__(self, element_connectivity, element_gradients, element_volume, element_material_index, materials,
                 lumped_mass, bc_mask, node_count, element_count, dof_count, stiffness_scale=1.0, mass_factor=0.0,
                 reduction_block=256, reduction_partials=None, adjacency=None, mode: int = _lib.MODE_PARITY,
                 device: int = 0, node_coords=None, keep_node_order: bool = False):
        # node_coords (optional, [N,3]) orders the FAST-mode element tiles and (FAST, unless keep_node_order)
        # the handle's internal node numbering (cwf_hip.h CWF_DESC_KEEP_NODE_ORDER); shards keep their order
        self.flags = _lib.DESC_KEEP_NODE_ORDER if keep_node_order else 0
        self.node_coords = (None if node_coords is None else
                            np.ascontiguousarray(np.asarray(node_coords, np.float64).reshape(-1)))
        self.element_connectivity = np.ascontiguousarray(element_connectivity, np.uint32)
        self.element_gradients = np.ascontiguousarray(element_gradients, np.float32)
        self.element_volume = np.ascontiguousarray(element_volume, np.float32)
        self.element_material_index = np.ascontiguousarray(element_material_index, np.uint32)
        stiff = [m.stiffness if hasattr(m, "stiffness") else m for m in materials]
        self.material_stiffness = np.ascontiguousarray(np.asarray(stiff, np.float64).reshape(-1))
        self.lumped_mass = np.ascontiguousarray(lumped_mass, np.float32)
        self.bc_mask = np.ascontiguousarray(bc_mask, np.uint32)
        self.node_count, self.element_count, self.dof_count = int(node_count), int(element_count), int(dof_count)
        self.stiffness_scale, self.mass_factor = float(stiffness_scale), float(mass_factor)
        self.reduction_block = int(reduction_block)
        self.reduction_partials = (int(reduction_partials) if reduction_partials is not None else
                                   max(1, (self.dof_count + max(1, self.reduction_block) - 1) //
                                       max(1, self.reduction_block)))
        self.adjacency = adjacency  # (offsets, element_indices, local_indices) or None
        self.mode = mode
        self.device = device
        self._h = None

    @classmethod
    def from_packing(cls, packing, materials, stiffness_scale=1.0, mass_factor=0.0, mode=_lib.MODE_PARITY,
                     device=0):
        return cls(packing.connectivity, packing.gradients, packing.volume, packing.material_index, materials,
                   packing.lumped_mass, packing.bc_mask, packing.node_count, packing.element_count,
                   packing.dof_count, stiffness_scale, mass_factor, packing.reduction_block,
                   packing.reduction_partials, (packing.offsets, packing.element_indices, packing.local_indices),
                   mode, device, packing.position64 if getattr(packing, "position64", None) is not None
                   else packing.position0)

    def desc(self) -> "_lib.SystemDesc":
        """The C descriptor over this object's host arrays (kept alive by the object)."""
        p = _lib.ptr
        adj = self.adjacency
        if adj is not None:
            adj = (np.ascontiguousarray(adj[0], np.uint32), np.ascontiguousarray(adj[1], np.uint32),
                   np.ascontiguousarray(adj[2], np.uint8))
        self._keep = adj  # keep the buffers alive across the C calls
        return _lib.SystemDesc(
            self.node_count, self.element_count, self.dof_count, p(self.element_connectivity),
            p(self.element_gradients), p(self.element_volume), p(self.element_material_index),
            p(self.material_stiffness), self.material_stiffness.size // 36, p(self.lumped_mass), p(self.bc_mask),
            p(adj[0]) if adj is not None else None,
            p(adj[1]) if adj is not None else None,
            p(adj[2]) if adj is not None else None,
            self.stiffness_scale, self.mass_factor, self.reduction_block, self.reduction_partials, self.mode,
            self.flags,
            p(self.node_coords) if self.node_coords is not None else None)

    # -- handle management --------------------------------------------------------------
    def handle(self):
        if self._h is None:
            L = _lib.load()
            desc = self.desc()
            h = C.c_void_p()
            st = L.cwf_hip_system_create(C.byref(desc), self.device, C.byref(h))
            if st:
                msg, ctx = _lib.last_error(None)
                raise PcgException(PcgError(msg, ctx), st)
            self._h = h
        L = _lib.load()
        L.cwf_hip_system_set_scalars(self._h, self.stiffness_scale, self.mass_factor)
        st = L.cwf_hip_system_set_mode(self._h, self.mode)
        if st:  # a mode the handle cannot take (hex8 or a renumbered handle asked for PARITY): loud, not FAST
            raise PcgException(self._err(), st)
        return self._h

    def close(self):
        if self._h is not None:
            _lib.load().cwf_hip_system_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _err(self) -> PcgError:
        msg, ctx = _lib.last_error(self._h)
        return PcgError(msg, ctx)


class PcgException(RuntimeError):
    def __init__(self, err: PcgError, code: int):
        super().__init__(f"{err.message} {err.context}")
        self.error, self.code = err, code


def _kind(a) -> int:
    return _lib.PTR_HOST if isinstance(a, np.ndarray) else _lib.PTR_DEVICE


def _size(a) -> int:
    return a.size if isinstance(a, np.ndarray) else a.numel()


def apply_keff(system: MatrixFreeSystem, input, output, workspace: MatrixFreeWorkspace | None = None) -> Expected:
    """pcg.hpp:161-163. input/output: f32 numpy arrays (host) or device tensors."""
    if _size(input) != system.dof_count or _size(output) != system.dof_count:
        return Expected(error=PcgError("input/output span size mismatch",
                                       [f"input={_size(input)}", f"output={_size(output)}",
                                        f"dofs={system.dof_count}"]))
    h = system.handle()
    st = _lib.load().cwf_hip_apply_keff(h, _lib.ptr(input), _lib.ptr(output), system.dof_count, _kind(input))
    return Expected(None) if st == 0 else Expected(error=system._err())


def build_block_jacobi_inverse(system: MatrixFreeSystem, workspace: MatrixFreeWorkspace | None,
                               out_inverse) -> Expected:
    """pcg.hpp:226-227"""
    required = system.node_count * 9
    if _size(out_inverse) < required:
        return Expected(error=PcgError("block inverse span too small",
                                       [f"required={required}", f"available={_size(out_inverse)}"]))
    h = system.handle()
    st = _lib.load().cwf_hip_build_block_jacobi_inverse(h, _lib.ptr(out_inverse), _size(out_inverse),
                                                        _kind(out_inverse))
    return Expected(None) if st == 0 else Expected(error=system._err())


def fast_block_inverse(system: MatrixFreeSystem, out_inverse, packed=None) -> Expected:
    """The preconditioner a FAST solve applies (no reference counterpart; cwf_hip_fast_block_inverse):
    build_block_jacobi_inverse symmetrised, restricted to the free axes and dequantised from the
    update pass's 16-B record. `packed` (optional host u32[4 N]) receives the records. The value is the
    number of nodes applied from their fp32 block (the packing's fallback)."""
    required = system.node_count * 9
    if _size(out_inverse) < required:
        return Expected(error=PcgError("block inverse span too small",
                                       [f"required={required}", f"available={_size(out_inverse)}"]))
    h = system.handle()
    nf = C.c_uint64()
    st = _lib.load().cwf_hip_fast_block_inverse(h, _lib.ptr(out_inverse), _size(out_inverse), _kind(out_inverse),
                                                _lib.ptr(packed) if packed is not None else None, C.byref(nf))
    return Expected(int(nf.value)) if st == 0 else Expected(error=system._err())


def pack_block_inverse(upper, mask: int):
    """Host packing of one node's block (blockinv_pack.hpp, the code the device runs): upper =
    {a00 a01 a02 a11 a12 a22} f32, mask bit k = axis k constrained. Returns (packed, record u32[4],
    applied upper triangle f32[6])."""
    v = np.ascontiguousarray(upper, np.float32)
    w = np.zeros(4, np.uint32)
    d = np.zeros(6, np.float32)
    ok = _lib.load().cwf_pack_block_inverse(_lib.ptr(v), int(mask), _lib.ptr(w), _lib.ptr(d))
    return bool(ok), w, d


def dot(system: MatrixFreeSystem, a, b, partials=None) -> Expected:
    """dot_accumulate (pcg.cpp:170-207)."""
    h = system.handle()
    out = C.c_double()
    st = _lib.load().cwf_hip_dot(h, _lib.ptr(a), _lib.ptr(b), _size(a), _kind(a), C.byref(out),
                                 _lib.ptr(partials) if partials is not None else None)
    return Expected(out.value) if st == 0 else Expected(error=system._err())


def solve_pcg(system: MatrixFreeSystem, rhs, settings: PcgSettings, vectors: PcgVectors,
              workspace: MatrixFreeWorkspace | None = None, check_interval: int = 0) -> Expected:
    """pcg.hpp:210-212. vectors.solution is the warm start / output; vectors.residual receives r."""
    if _size(rhs) != system.dof_count:
        return Expected(error=PcgError("rhs span size mismatch", [f"rhs={_size(rhs)}", f"dofs={system.dof_count}"]))
    if settings.max_iterations == 0:
        return Expected(error=PcgError("max_iterations must be >= 1", ["max_iterations=0"]))
    h = system.handle()
    s = _lib.PcgSettingsC(settings.max_iterations, settings.relative_tolerance, int(settings.warm_start),
                          check_interval)
    tel = _lib.PcgTelemetryC()
    st = _lib.load().cwf_hip_solve_pcg(h, _lib.ptr(rhs), C.byref(s), _lib.ptr(vectors.solution),
                                       _lib.ptr(vectors.residual) if vectors.residual is not None else None,
                                       system.dof_count, _kind(rhs), C.byref(tel))
    if st:
        return Expected(error=system._err())
    return Expected(PcgTelemetry.from_c(tel))


def residual_history(system: MatrixFreeSystem) -> np.ndarray:
    h = system.handle()
    cap = 1 << 16
    out = np.zeros(cap, np.float64)
    n = C.c_uint64()
    _lib.load().cwf_hip_residual_history(h, _lib.ptr(out), cap, C.byref(n))
    return out[: n.value].copy()
