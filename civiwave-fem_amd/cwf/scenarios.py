"""Synthetic scenarios of BASELINE.json's configs: structured Kuhn-tet
blocks, x=0 face fixed, gravity + a -500 N point load per node of the x=max face, steel-like
material (E=30 GPa, nu=0.2, rho=2500), Newmark dt=0.01."""
from __future__ import annotations

import os
from dataclasses import dataclass

import numpy as np

from . import meshgen, pack
from .physics import (Assignment, Config, Curve, Damping, DirichletFix, Loads, Material, PointLoad, SolverSettings,
                      TimeSettings, compute_rayleigh, effective_scalars, evaluate_curve, make_coefficients,
                      make_properties)

HARMONIC_POINTS = 64  # samples of one period of the C4 harmonic tip load


def harmonic_curve(freq: float, points: int = HARMONIC_POINTS) -> Curve:
    """F(t) / F0 = sin(2 pi f t) sampled at `points` equally spaced times over one period [0, 1/f] as a
    piecewise-linear load curve (config::Curve, evaluated by loads.cpp:63-85)."""
    T = 1.0 / freq
    return Curve([(k * T / (points - 1), float(np.sin(2.0 * np.pi * freq * (k * T / (points - 1)))))
                  for k in range(points)])


@dataclass
class Case:
    name: str
    mesh: pack.Mesh
    cfg: Config
    packing: pack.PackingResult

    @property
    def materials(self):
        return [make_properties(m) for m in self.cfg.materials]

    @property
    def rayleigh(self):
        return compute_rayleigh(self.cfg.damping)

    def scalars(self, dt: float | None = None):
        c = make_coefficients(dt if dt is not None else self.cfg.time.initial_dt)
        return effective_scalars(c, self.rayleigh)

    @property
    def load_curve(self):
        """(name, Curve) of the curve-scaled point load, or None (static loads)."""
        for pl in self.cfg.loads.points:
            if pl.scale_curve in self.cfg.curves:
                return pl.scale_curve, self.cfg.curves[pl.scale_curve]
        return None

    def load_scale(self, t: float) -> float:
        """The load curve at time t, periodically extended past its last sample (the harmonic load repeats)."""
        _, c = self.load_curve
        period = c.points[-1][0] - c.points[0][0]
        return evaluate_curve(c, t % period if period > 0 else t)

    def external_force_at(self, t: float) -> np.ndarray:
        """nodes.external_force at time t: loads.cpp:87-174 at the curve's periodic time, cast as pack.cpp:41-57
        (the vector the viewer's host rewrite would upload before each step, viewer.cpp:262-266)."""
        _, c = self.load_curve
        period = c.points[-1][0] - c.points[0][0]
        f = pack.assemble_load_vector(self.mesh, self.cfg, self.packing.lumped_mass64, t % period)
        return pack._safe_f32(f)

    def load_pattern(self):
        """(base, pattern) f64 [3N] for Stepper.set_load_pattern: the loads no curve scales, and the values of
        the curve-scaled point loads (external_force(t) = f32(base + curve(t) * pattern))."""
        from dataclasses import replace

        name, _ = self.load_curve
        scaled = [pl for pl in self.cfg.loads.points if pl.scale_curve == name]
        rest = replace(self.cfg, loads=replace(self.cfg.loads,
                                                points=[pl for pl in self.cfg.loads.points if pl.scale_curve != name]))
        base = pack.assemble_load_vector(self.mesh, rest, self.packing.lumped_mass64)
        pattern = np.zeros((self.mesh.node_count, 3), np.float64)
        for pl in scaled:
            gid = self.mesh.group_names.get(pl.group)
            if gid is None or gid not in self.mesh.node_groups:
                continue
            nodes = np.asarray(self.mesh.node_groups[gid], np.int64)
            for k in range(3):
                np.add.at(pattern[:, k], nodes, pl.value[k])
        return base, pattern.reshape(-1)

    def static_rhs(self) -> np.ndarray:
        """external force with the constrained rows zeroed (the survey drivers' solve_pcg RHS)."""
        rhs = self.packing.external_force.copy()
        mask = np.repeat(self.packing.bc_mask, 3) & np.tile(np.array([1, 2, 4], np.uint32), self.packing.node_count)
        rhs[mask != 0] = 0.0
        return rhs


def make_config(xi=0.02, w=(5.0, 50.0), tol=3e-4, max_iterations=2000, dt=0.01, gravity=(0.0, 0.0, -9.81),
                point=(0.0, 0.0, -500.0), point_group="TIP", dirichlet=None, harmonic=None) -> Config:
    """harmonic=f (Hz): the point load is F0 sin(2 pi f t) with F0 = `point`, a 64-point curve (C4)."""
    fixes = dirichlet if dirichlet is not None else [DirichletFix("FIXED", (True, True, True), (0.0, 0.0, 0.0))]
    curves = {"harmonic": harmonic_curve(harmonic)} if harmonic else {}
    return Config(materials=[Material("steel", 30.0e9, 0.2, 2500.0)], assignments=[Assignment("SOLID", "steel")],
                  damping=Damping(xi, w[0], w[1]), time=TimeSettings(dt, False, 0.0, 0.0),
                  solver=SolverSettings("pcg", "block_jacobi", tol, 1.0e-5, max_iterations),
                  loads=Loads(tuple(gravity), [], [PointLoad(point_group, tuple(point),
                                                             "harmonic" if harmonic else "")]),
                  curves=curves, dirichlet=fixes)


def block_case(nx, ny, nz, h=0.1, jitter=False, element="tet4", **cfg_kw) -> Case:
    """element="tet4": the Kuhn expansion (the reference's path); "hex8": native hexes (SURVEY 8f4,
    FAST mode only)."""
    tm = meshgen.hex_block(nx, ny, nz, h) if element == "hex8" else meshgen.kuhn_block(nx, ny, nz, h)
    if jitter:
        tm = meshgen.jitter_and_permute(tm, h)
    if os.environ.get("CWF_MORTON_NODES") == "1":  # diagnostic: node-order locality experiment
        tm = meshgen.morton_renumber(tm)
    mesh = pack.from_tetmesh(tm)
    cfg = make_config(**cfg_kw)
    tag = "hex" if element == "hex8" else "kuhn"
    return Case(f"{tag}{nx}x{ny}x{nz}", mesh, cfg, pack.build_packed_buffers(mesh, cfg))


def config_case(key: str, max_iterations: int = 2000, element: str = "tet4") -> Case:
    c = meshgen.CONFIGS[key]
    case = block_case(*c["shape"], h=c["h"], jitter=c.get("jitter", False), xi=c["xi"], w=c["w"], tol=c["tol"],
                      max_iterations=max_iterations, element=element, harmonic=c.get("harmonic"))
    name = c["name"].replace("(Kuhn tets)", "(native hex8)") if element == "hex8" else c["name"]
    case.name = f"{key}: {name}"
    return case


def slab_case_shape(shape, nranks: int, rank: int, h: float = 0.1, max_iterations: int = 2000, stack: bool = True,
                    element: str = "tet4", **cfg_kw):
    """Slab decomposition of an nx*ny*nz block. stack=True (weak scaling): the global block stacks `nranks`
    copies along z (nz * nranks cells); stack=False (strong scaling): the global block is the nx*ny*nz block
    itself. Rank r owns a contiguous range of node planes and gets the sub-mesh of every cell touching them
    (its ghost layer). Returns (case over the sub-mesh, global node id per sub-mesh node, rank_node_begin
    [nranks + 1] in global node ids)."""
    nx, ny, nz1 = shape
    nz = nz1 * nranks if stack else nz1
    A, B = nx + 1, ny + 1
    planes = [(nz + 1) * r // nranks for r in range(nranks + 1)]
    kc0, kc1 = max(planes[rank] - 1, 0), min(planes[rank + 1], nz)
    tm, node_global = meshgen.kuhn_slab(nx, ny, nz, kc0, kc1, h, element)
    mesh = pack.from_tetmesh(tm)
    cfg = make_config(max_iterations=max_iterations, **cfg_kw)
    tag = "hex" if element == "hex8" else "kuhn"
    case = Case(f"{tag}{nx}x{ny}x{nz}/slab{rank}of{nranks}", mesh, cfg, pack.build_packed_buffers(mesh, cfg))
    begin = np.asarray([p * A * B for p in planes], np.uint64)
    return case, node_global, begin


def slab_case(key: str, nranks: int, rank: int, max_iterations: int = 2000, strong: bool = False,
              element: str = "tet4"):
    """slab_case_shape for BASELINE config `key`: weak scaling (`key`'s block per rank) or strong scaling
    (`key`'s block split into `nranks` slabs, e.g. C3's fixed 10.1M DOF on 1/2/4/8 GPUs)."""
    c = meshgen.CONFIGS[key]
    case, node_global, begin = slab_case_shape(c["shape"], nranks, rank, h=c["h"], max_iterations=max_iterations,
                                               stack=not strong, element=element, xi=c["xi"], w=c["w"],
                                               tol=c["tol"], harmonic=c.get("harmonic"))
    name = c["name"].replace("(Kuhn tets)", "(native hex8)") if element == "hex8" else c["name"]
    case.name = f"{key}: {name}, " + (f"slab {rank} of {nranks} (strong)" if strong
                                      else f"x{nranks} stacked, slab {rank} (weak)")
    return case, node_global, begin


def rcb_case(key: str, nranks: int, max_iterations: int = 2000):
    """Strong-scaling decomposition of an unstructured BASELINE config (C4): the whole mesh on every rank,
    nodes partitioned by recursive coordinate bisection and renumbered part after part (shard.rcb_node_ranges).
    Returns (global case, global id per node, rank_node_begin) for shard.build_shard."""
    from .shard import rcb_node_ranges

    case = config_case(key, max_iterations=max_iterations)
    gid, begin = rcb_node_ranges(case.mesh.coords, nranks)
    case.name = f"{case.name}, RCB x{nranks} (strong)"
    return case, gid, begin


def roller_case(nx, ny, nz, h=0.1, element="tet4", **cfg_kw) -> Case:
    """Partial Dirichlet masks (config.hpp:208 constrain_axis): rollers on three faces -- x=0 fixed in x
    only (FIXED), y=0 in y only (SIDE), z=0 in z only (BOTTOM) -- which remove the rigid modes while most
    constrained nodes keep two free axes (edges one, the origin none). Loads as block_case."""
    tm = meshgen.hex_block(nx, ny, nz, h) if element == "hex8" else meshgen.kuhn_block(nx, ny, nz, h)
    A, B = nx + 1, ny + 1
    n = np.arange(tm.coords.shape[0], dtype=np.int64)
    i, j, k = n % A, (n // A) % B, n // (A * B)
    tm.node_groups["SIDE"] = n[j == 0].astype(np.uint32)
    tm.node_groups["BOTTOM"] = n[k == 0].astype(np.uint32)
    assert np.array_equal(tm.node_groups["FIXED"], n[i == 0].astype(np.uint32))
    mesh = pack.from_tetmesh(tm)
    fixes = [DirichletFix("FIXED", (True, False, False), (0.0, None, None)),
             DirichletFix("SIDE", (False, True, False), (None, 0.0, None)),
             DirichletFix("BOTTOM", (False, False, True), (None, None, 0.0))]
    cfg = make_config(dirichlet=fixes, **cfg_kw)
    tag = "hex" if element == "hex8" else "kuhn"
    return Case(f"{tag}{nx}x{ny}x{nz}-rollers", mesh, cfg, pack.build_packed_buffers(mesh, cfg))
