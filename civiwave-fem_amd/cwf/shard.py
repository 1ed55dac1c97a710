"""Multi-GPU decomposition over the C-ABI (include/cwf_hip.h).

``build_shard`` cuts a mesh (the global packing, or a sub-mesh holding every element that touches
the rank's nodes) into the rank-local system: owned nodes first, ghost nodes grouped by owner rank,
plus the halo plan. ``Comm.local`` runs every rank of a decomposition in this process on one device;
``Comm.rccl`` is one rank per process over RCCL (the unique id travels over torch.distributed or any
other channel the caller has). The reference is single-device, so there is no reference interface
to mirror here; the solver calls on a shard keep the ``cwf::gpu::pcg`` semantics on local vectors.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib
from .pcg import Expected, MatrixFreeSystem, PcgError, PcgSettings, PcgTelemetry


def slab_ranges(node_count: int, nranks: int, align: int = 1) -> np.ndarray:
    """Contiguous node ranges [begin_r, begin_{r+1}) of near-equal size, boundaries multiples of
    `align` (256 nodes = 768 DOF = three 256-DOF reduction chunks keeps chunk partials rank-local)."""
    b = [0]
    for r in range(1, nranks):
        cut = (node_count * r) // nranks
        cut = min(node_count, ((cut + align // 2) // align) * align) if align > 1 else cut
        b.append(max(b[-1], cut))
    b.append(node_count)
    return np.asarray(b, np.uint64)


def _morton_keys(c: np.ndarray) -> np.ndarray:
    lo, hi = c.min(0), c.max(0)
    q = np.floor((c - lo) / max(float((hi - lo).max()), 1e-300) * ((1 << 20) - 1)).astype(np.uint64)

    def spread(v):
        v = v & np.uint64(0x1FFFFF)
        v = (v | v << np.uint64(32)) & np.uint64(0x1F00000000FFFF)
        v = (v | v << np.uint64(16)) & np.uint64(0x1F0000FF0000FF)
        v = (v | v << np.uint64(8)) & np.uint64(0x100F00F00F00F00F)
        v = (v | v << np.uint64(4)) & np.uint64(0x10C30C30C30C30C3)
        v = (v | v << np.uint64(2)) & np.uint64(0x1249249249249249)
        return v

    return spread(q[:, 0]) | spread(q[:, 1]) << np.uint64(1) | spread(q[:, 2]) << np.uint64(2)


def rcb_node_ranges(coords: np.ndarray, nranks: int):
    """Recursive coordinate bisection of the nodes into `nranks` parts of near-equal size (the
    C4 mesh is randomly numbered, so contiguous ranges of its own ids would make every shard's halo most of the
    mesh). A range of parts is split along its longest extent at the node count proportional to its two halves'
    part counts (ties broken by node id, so every rank computes the same partition). Nodes are then numbered
    part after part, along a Morton curve inside a part (the locality the shard's tiles gather with).
    Returns (global id per input node u64 [N], rank_node_begin u64 [nranks + 1]) for cwf_shard_build."""
    c = np.asarray(coords, np.float64).reshape(-1, 3)
    N = c.shape[0]
    part = np.empty(N, np.int64)
    stack = [(np.arange(N, dtype=np.int64), 0, nranks)]
    while stack:
        idx, p0, n = stack.pop()
        if n == 1 or idx.size == 0:
            part[idx] = p0
            continue
        sub = c[idx]
        axis = int(np.argmax(sub.max(0) - sub.min(0)))
        nl = n // 2
        cut = (idx.size * nl) // n
        order = np.lexsort((idx, sub[:, axis]))  # by coordinate, then node id
        stack.append((idx[order[:cut]], p0, nl))
        stack.append((idx[order[cut:]], p0 + nl, n - nl))
    key = _morton_keys(c)
    order = np.lexsort((np.arange(N), key, part))  # part, then Morton, then id
    gid = np.empty(N, np.uint64)
    gid[order] = np.arange(N, dtype=np.uint64)
    counts = np.bincount(part, minlength=nranks)
    begin = np.concatenate([[0], np.cumsum(counts)]).astype(np.uint64)
    return gid, begin


@dataclass
class Shard:
    rank: int
    nranks: int
    owned_nodes: int
    local_nodes: int
    local_elements: int
    neighbor_ranks: np.ndarray  # i32 [K]
    send_offsets: np.ndarray  # u64 [K+1]
    send_nodes: np.ndarray  # u32 owned local ids
    recv_offsets: np.ndarray  # u64 [K+1] ghost ranges (relative to owned_nodes)
    node_global: np.ndarray  # u64 [local_nodes]
    node_source: np.ndarray  # u64 [local_nodes] node index in the input
    element_source: np.ndarray  # u64 [local_elements] element index in the input
    # local system arrays
    connectivity: np.ndarray
    gradients: np.ndarray
    volume: np.ndarray
    material_index: np.ndarray
    lumped_mass: np.ndarray
    bc_mask: np.ndarray
    node_coords: np.ndarray | None
    _c: object = None  # cwf_shard* (owns the arrays the info points into)

    def info(self) -> _lib.ShardInfoC:
        i = _lib.ShardInfoC()
        _lib.load().cwf_shard_get(self._c, None, C.byref(i))
        return i

    def local_dofs(self, global_vec: np.ndarray) -> np.ndarray:
        """Gather a node-interleaved input vector (indexed like the input mesh) into local order."""
        v = np.asarray(global_vec).reshape(-1, 3)
        return np.ascontiguousarray(v[self.node_source.astype(np.int64)].reshape(-1))

    def system(self, materials, stiffness_scale=1.0, mass_factor=0.0, device=0, mode=_lib.MODE_FAST) -> MatrixFreeSystem:
        """The shard's local handle (its node order is the halo plan's). mode=MODE_PARITY gives the bit-exact
        sharded solve; it needs slab_ranges(..., align=256) ranges (cwf_hip.h cwf_hip_system_attach)."""
        return MatrixFreeSystem(self.connectivity, self.gradients, self.volume, self.material_index, materials,
                                self.lumped_mass, self.bc_mask, self.local_nodes, self.local_elements,
                                3 * self.local_nodes, stiffness_scale, mass_factor, 256, None, None,
                                mode, device, self.node_coords, keep_node_order=True)

    def close(self):
        if self._c is not None:
            _lib.load().cwf_shard_destroy(self._c)
            self._c = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def build_shard(system: MatrixFreeSystem, rank_node_begin, rank: int, node_global=None) -> Shard:
    """cwf_shard_build over `system`'s host arrays (global mesh or a covering sub-mesh)."""
    L = _lib.load()
    begin = np.ascontiguousarray(rank_node_begin, np.uint64)
    ng = None if node_global is None else np.ascontiguousarray(node_global, np.uint64)
    desc = system.desc()
    h = C.c_void_p()
    st = L.cwf_shard_build(C.byref(desc), _lib.ptr(ng), _lib.ptr(begin), begin.size - 1, rank, C.byref(h))
    if st:
        msg, ctx = _lib.last_error(None)
        raise RuntimeError(f"shard build failed: {msg} {ctx}")
    d, i = _lib.SystemDesc(), _lib.ShardInfoC()
    L.cwf_shard_get(h, C.byref(d), C.byref(i))

    def arr(p, n, dt):
        if n == 0 or not p:
            return np.zeros(0, dt)
        return np.ctypeslib.as_array(C.cast(p, C.POINTER(np.ctypeslib.as_ctypes_type(dt))), (n,)).copy()

    NL, EL, K = i.local_nodes, i.local_elements, i.neighbor_count
    return Shard(rank, begin.size - 1, int(i.owned_nodes), int(NL), int(EL), arr(i.neighbor_ranks, K, np.int32),
                 arr(i.send_offsets, K + 1, np.uint64), arr(i.send_nodes, int(arr(i.send_offsets, K + 1,
                                                                                   np.uint64)[-1]), np.uint32),
                 arr(i.recv_offsets, K + 1, np.uint64), arr(i.node_global, NL, np.uint64),
                 arr(i.node_source, NL, np.uint64), arr(i.element_source, EL, np.uint64),
                 arr(d.element_connectivity, EL * 8, np.uint32), arr(d.element_gradients, EL * 24, np.float32),
                 arr(d.element_volume, EL, np.float32), arr(d.element_material_index, EL, np.uint32),
                 arr(d.lumped_mass, NL, np.float32), arr(d.bc_mask, NL, np.uint32),
                 arr(d.node_coords, NL * 3, np.float64) if d.node_coords else None, h)


class Comm:
    """cwf_hip_comm: LOCAL (all ranks in this process, one device) or RCCL (one rank per process)."""

    def __init__(self, handle, nranks: int, kind: str):
        self._h, self.nranks, self.kind = handle, nranks, kind
        self._members = {}

    @staticmethod
    def unique_id() -> bytes:
        buf = (C.c_uint8 * _lib.COMM_ID_BYTES)()
        if _lib.load().cwf_hip_comm_unique_id(buf):
            raise RuntimeError(f"rccl unique id: {_lib.last_error(None)}")
        return bytes(buf)

    @classmethod
    def rccl(cls, nranks: int, rank: int, uid: bytes, device: int = 0) -> "Comm":
        buf = (C.c_uint8 * _lib.COMM_ID_BYTES).from_buffer_copy(uid)
        h = C.c_void_p()
        if _lib.load().cwf_hip_comm_create_rccl(nranks, rank, buf, device, C.byref(h)):
            raise RuntimeError(f"rccl communicator: {_lib.last_error(None)}")
        return cls(h, nranks, "rccl")

    @classmethod
    def peer(cls, nranks: int, rank: int, device: int = 0) -> "Comm":
        """PEER (peer.hip): one process per rank; after attach, exchange `handle()` between the processes and
        `connect(handles)` with all of them in rank order."""
        h = C.c_void_p()
        if _lib.load().cwf_hip_comm_create_peer(nranks, rank, device, C.byref(h)):
            raise RuntimeError(f"peer communicator: {_lib.last_error(None)}")
        return cls(h, nranks, "peer")

    def handle(self) -> bytes:
        buf = (C.c_uint8 * _lib.IPC_HANDLE_BYTES)()
        if _lib.load().cwf_hip_comm_peer_handle(self._h, buf):
            raise RuntimeError(f"peer handle: {_lib.last_error(None)}")
        return bytes(buf)

    def mailbox_kind(self) -> int:
        """_lib.PEER_MAILBOX_{DEVICE,FINEGRAINED,UNCACHED}: the memory this rank's mailbox was allocated in"""
        k = C.c_int(-1)
        if _lib.load().cwf_hip_comm_peer_mailbox_kind(self._h, C.byref(k)):
            raise RuntimeError(f"peer mailbox kind: {_lib.last_error(None)}")
        return k.value

    def connect(self, handles: list):
        blob = b"".join(handles)
        buf = (C.c_uint8 * len(blob)).from_buffer_copy(blob)
        if _lib.load().cwf_hip_comm_peer_connect(self._h, buf):
            raise RuntimeError(f"peer connect: {_lib.last_error(None)}")

    @staticmethod
    def time_exchange(system: MatrixFreeSystem, steps: int = 200) -> float:
        """microseconds per exchange step of the single-launch iteration's shape (collective)"""
        us = C.c_double()
        h = system.handle()
        if _lib.load().cwf_hip_comm_time_exchange(h, steps, C.byref(us)):
            raise RuntimeError(f"time exchange: {_lib.last_error(h)}")
        return us.value

    @classmethod
    def local(cls, nranks: int, device: int = 0) -> "Comm":
        h = C.c_void_p()
        if _lib.load().cwf_hip_comm_create_local(nranks, device, C.byref(h)):
            raise RuntimeError(f"local communicator: {_lib.last_error(None)}")
        return cls(h, nranks, "local")

    def attach(self, system: MatrixFreeSystem, shard: Shard):
        info = shard.info()
        h = system.handle()
        if _lib.load().cwf_hip_system_attach(h, self._h, shard.rank, C.byref(info)):
            raise RuntimeError(f"attach: {_lib.last_error(h)}")
        self._members[shard.rank] = system

    def close(self):
        if self._h is not None:
            for s in self._members.values():
                s.close()
            self._members = {}
            _lib.load().cwf_hip_comm_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def solve_pcg_group(systems: list, rhs: list, settings: PcgSettings, solutions: list,
                    check_interval: int = 0, residuals: list | None = None) -> Expected:
    """solve_pcg over every rank of a LOCAL communicator (systems in rank order); `residuals` (optional)
    receives each rank's local r."""
    n = len(systems)
    hs = (C.c_void_p * n)(*[s.handle().value for s in systems])
    rp = (C.c_void_p * n)(*[_lib.ptr(r).value for r in rhs])
    xp = (C.c_void_p * n)(*[_lib.ptr(x).value for x in solutions])
    resp = (C.c_void_p * n)(*[_lib.ptr(r).value for r in residuals]) if residuals is not None else None
    kind = _lib.PTR_HOST if isinstance(rhs[0], np.ndarray) else _lib.PTR_DEVICE
    s = _lib.PcgSettingsC(settings.max_iterations, settings.relative_tolerance, int(settings.warm_start),
                          check_interval)
    tel = _lib.PcgTelemetryC()
    st = _lib.load().cwf_hip_solve_pcg_group(hs, n, rp, C.byref(s), xp, resp, kind, C.byref(tel))
    if st:
        msg, ctx = _lib.last_error(systems[0]._h)
        return Expected(error=PcgError(msg, ctx))
    return Expected(PcgTelemetry.from_c(tel))
