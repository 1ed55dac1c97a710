"""Packed SoA buffers for the hot path: mesh::pre::run + pack::build_packed_buffers
(src/mesh/preprocess.cpp:284-405, src/mesh/pack.cpp:61-235) + the load and Dirichlet builders
they call (src/physics/loads.cpp:87-174, src/physics/solver.cpp:312-352).

The fp64 geometry (gradients, volumes, lumped masses, CSR) is computed by the native host
routine ``cwf_preprocess_tets`` of libcwf_hip.so; loads and masks are vectorised numpy in the
reference's accumulation order (gravity first, then tractions, then point loads).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field

import numpy as np

from . import _lib
from .physics import Config, evaluate_curve


@dataclass
class Mesh:
    """Subset of cwf::mesh::Mesh (include/cwf/mesh/mesh.hpp:120-150) for tet4 (or native hex8) meshes."""

    coords: np.ndarray  # f64 [N,3]
    tets: np.ndarray  # u32 [E,4] (tet4) or [E,8] (hex8, Gmsh corner order; FAST mode only)
    element_group: np.ndarray | None = None  # u32 [E] physical group id per element
    group_names: dict = field(default_factory=dict)  # name -> id
    node_groups: dict = field(default_factory=dict)  # id -> u32 node indices
    surfaces: list = field(default_factory=list)  # [(group_id, (n0, n1, n2[, n3]))]

    @property
    def node_count(self):
        return self.coords.shape[0]

    @property
    def element_count(self):
        return self.tets.shape[0]


def from_tetmesh(tm, solid_group: str = "SOLID") -> Mesh:
    """Wrap a meshgen.TetMesh: one SOLID volume group (id 1) + its node groups (ids 2..)."""
    names = {solid_group: 1}
    groups = {}
    for i, (name, nodes) in enumerate(tm.node_groups.items()):
        names[name] = i + 2
        groups[i + 2] = np.asarray(nodes, np.uint32)
    return Mesh(np.ascontiguousarray(tm.coords, np.float64), np.ascontiguousarray(tm.tets, np.uint32),
                np.ones(tm.tets.shape[0], np.uint32), names, groups, [])


@dataclass
class PackError(Exception):
    message: str
    context: list

    def __str__(self):
        return f"{self.message} {self.context}"


@dataclass
class PackingResult:
    node_count: int
    element_count: int
    dof_count: int
    reduction_block: int
    reduction_partials: int
    position0: np.ndarray  # f32 [N,3]
    external_force: np.ndarray  # f32 [3N] (dof = 3n+k)
    bc_mask: np.ndarray  # u32 [N]
    bc_value: np.ndarray  # f32 [3N]
    lumped_mass: np.ndarray  # f32 [N]
    lumped_mass64: np.ndarray  # f64 [N] (pre::Outputs::lumped_mass)
    connectivity: np.ndarray  # u32 [E*8]
    gradients: np.ndarray  # f32 [E*24]
    volume: np.ndarray  # f32 [E]
    material_index: np.ndarray  # u32 [E]
    offsets: np.ndarray  # u32 [N+1]
    element_indices: np.ndarray  # u32 [4E]
    local_indices: np.ndarray  # u8 [4E]
    position64: np.ndarray | None = None  # f64 [N,3] the preprocess input (FAST tiles: order + geometry)
    # nodes.displacement / velocity / acceleration (pack.hpp:95-105), f32 [3N]; the post stack reads them
    displacement: np.ndarray | None = None
    velocity: np.ndarray | None = None
    acceleration: np.ndarray | None = None

    def __post_init__(self):
        for name in ("displacement", "velocity", "acceleration"):
            if getattr(self, name) is None:
                setattr(self, name, np.zeros(3 * self.node_count, np.float32))


def _group_nodes(mesh: Mesh, gid: int) -> np.ndarray:
    """solver.cpp:90-125 gather_group_nodes: surface nodes + tagged nodes (a set)."""
    parts = [np.asarray(mesh.node_groups.get(gid, []), np.int64)]
    for sg, nodes in mesh.surfaces:
        if sg == gid:
            parts.append(np.asarray(nodes, np.int64))
    return np.unique(np.concatenate(parts)) if parts else np.zeros(0, np.int64)


def preprocess(mesh: Mesh, cfg: Config):
    """Native geometry pass (preprocess.cpp:284-405) -> dict of arrays."""
    L = _lib.load()
    N, E = mesh.node_count, mesh.element_count
    # bind_materials (preprocess.cpp:48-84)
    density = np.array([m.density for m in cfg.materials] or [0.0], np.float64)
    group_to_mat = {}
    for i, a in enumerate(cfg.assignments):
        if a.group not in mesh.group_names:
            raise PackError(f"assignment references missing physical group '{a.group}'",
                            ["assignments", f"[{i}]"])
        names = [m.name for m in cfg.materials]
        if a.material not in names:
            raise PackError(f"assignment references missing material '{a.material}'", ["assignments", f"[{i}]"])
        group_to_mat.setdefault(mesh.group_names[a.group], names.index(a.material))
    eg = mesh.element_group if mesh.element_group is not None else np.ones(E, np.uint32)
    mat = np.full(E, 0xFFFFFFFF, np.uint32)
    for gid, mi in group_to_mat.items():
        mat[eg == gid] = mi
    bad = np.nonzero(mat == 0xFFFFFFFF)[0]
    if bad.size:
        raise PackError("element physical group missing assignment", ["elements", f"[{int(bad[0])}]"])
    coords = np.ascontiguousarray(mesh.coords, np.float64)
    tets = np.ascontiguousarray(mesh.tets, np.uint32)
    K = tets.shape[1] if tets.ndim == 2 else 4  # 4: tet4 (the reference path), 8: native hex8
    out = dict(grads=np.zeros(E * 24, np.float32), volume=np.zeros(E, np.float32), mass64=np.zeros(N, np.float64),
               mass32=np.zeros(N, np.float32), offsets=np.zeros(N + 1, np.uint32),
               adj_elem=np.zeros(E * K, np.uint32), adj_local=np.zeros(E * K, np.uint8),
               conn8=np.zeros(E * 8, np.uint32), material_index=mat)
    p = _lib.ptr
    fn = L.cwf_preprocess_hex8 if K == 8 else L.cwf_preprocess_tets
    st = fn(N, E, p(coords), p(tets), p(mat), p(density), len(cfg.materials), p(out["grads"]),
            p(out["volume"]), p(out["mass64"]), p(out["mass32"]), p(out["offsets"]),
            p(out["adj_elem"]), p(out["adj_local"]), p(out["conn8"]))
    if st:
        msg, ctx = _lib.last_error(None)
        raise PackError(msg, ctx)
    return out


def assemble_load_vector(mesh: Mesh, cfg: Config, mass64: np.ndarray, time: float = 0.0) -> np.ndarray:
    """loads.cpp:87-174 (f64 [3N])."""
    N = mesh.node_count
    loads = np.zeros((N, 3), np.float64)
    g = np.asarray(cfg.loads.gravity, np.float64)
    loads += mass64[:, None] * g[None, :]
    for tr in cfg.loads.tractions:
        gid = mesh.group_names.get(tr.group)
        if gid is None:
            continue
        scale = evaluate_curve(cfg.curves[tr.scale_curve], time) if tr.scale_curve in cfg.curves else 1.0
        for sg, nodes in mesh.surfaces:
            if sg != gid:
                continue
            P = mesh.coords
            area = _tri_area(P, nodes[0], nodes[1], nodes[2])
            if len(nodes) == 4:
                area = area + _tri_area(P, nodes[0], nodes[2], nodes[3])
            share = (area * scale) / float(len(nodes))
            for n in nodes:
                for k in range(3):
                    loads[n, k] += share * tr.value[k]
    for pl in cfg.loads.points:
        gid = mesh.group_names.get(pl.group)
        if gid is None or gid not in mesh.node_groups:
            continue
        scale = evaluate_curve(cfg.curves[pl.scale_curve], time) if pl.scale_curve in cfg.curves else 1.0
        nodes = np.asarray(mesh.node_groups[gid], np.int64)
        for k in range(3):
            np.add.at(loads[:, k], nodes, scale * pl.value[k])
    return loads.reshape(-1)


def _tri_area(P, i0, i1, i2) -> float:
    import math

    p0, p1, p2 = P[i0], P[i1], P[i2]
    v1 = [p1[0] - p0[0], p1[1] - p0[1], p1[2] - p0[2]]
    v2 = [p2[0] - p0[0], p2[1] - p0[1], p2[2] - p0[2]]
    cr = [(v1[1] * v2[2]) - (v1[2] * v2[1]), (v1[2] * v2[0]) - (v1[0] * v2[2]), (v1[0] * v2[1]) - (v1[1] * v2[0])]
    return 0.5 * math.sqrt((cr[0] * cr[0]) + (cr[1] * cr[1]) + (cr[2] * cr[2]))


def build_dirichlet(mesh: Mesh, cfg: Config):
    """solver.cpp:312-352 -> (mask bool [3N], targets f64 [3N])."""
    N = mesh.node_count
    mask = np.zeros(3 * N, bool)
    targets = np.zeros(3 * N, np.float64)
    for fix in cfg.dirichlet:
        gid = mesh.group_names.get(fix.group)
        if gid is None:
            continue
        nodes = _group_nodes(mesh, gid)
        for k in range(3):
            if not fix.constrain_axis[k]:
                continue
            v = fix.value[k] if fix.value[k] is not None else 0.0
            mask[3 * nodes + k] = True
            targets[3 * nodes + k] = v
    return mask, targets


def build_packed_buffers(mesh: Mesh, cfg: Config, load_time_seconds: float = 0.0,
                         reduction_block_size: int = 256) -> PackingResult:
    if reduction_block_size == 0:
        raise PackError("reduction block size must be >= 1", ["PackingParameters", "reduction_block_size"])
    pre = preprocess(mesh, cfg)
    N, E = mesh.node_count, mesh.element_count
    D = 3 * N
    mask, targets = build_dirichlet(mesh, cfg)
    loads = assemble_load_vector(mesh, cfg, pre["mass64"], load_time_seconds)
    bc_mask = (mask.reshape(N, 3).astype(np.uint32) * np.array([1, 2, 4], np.uint32)).sum(1).astype(np.uint32)
    bc_value = np.where(mask, targets, 0.0).astype(np.float32)
    rb = max(1, reduction_block_size)
    return PackingResult(N, E, D, rb, max(1, (D + rb - 1) // rb), mesh.coords.astype(np.float32),
                         _safe_f32(loads), bc_mask, bc_value, pre["mass32"], pre["mass64"], pre["conn8"],
                         pre["grads"], pre["volume"], pre["material_index"], pre["offsets"], pre["adj_elem"],
                         pre["adj_local"], np.ascontiguousarray(mesh.coords, np.float64))


def _safe_f32(v: np.ndarray) -> np.ndarray:
    """pack.cpp:41-57 safe_cast_double_to_float (finite values clamp to +-FLT_MAX)."""
    fmax = float(np.finfo(np.float32).max)
    with np.errstate(over="ignore"):
        out = np.where(np.isfinite(v), np.clip(v, -fmax, fmax), v).astype(np.float32)
    return out
