"""Host side of the structured-block FAST operator (lattice.cpp) on the CPU: the detection and the stencil blocks
it derives, through the C-ABI introspection entry cwf_lattice_describe (no device needed).

The blocks are applied here in numpy (fp64 over the f32 blocks), with the kernel's algorithm (lattice.inc): the 14
off-centre interior stencil blocks on the differences u_(n+d) - u_n for the nodes inside the block, and for the
nodes on its surface each existing cell's blocks on the differences to the node's own value. That must reproduce the pinned oracle's apply_keff (the reference's element loop) to the f32 rounding of
the blocks: 1e-6 of the operator scale (max |row|)."""
import ctypes as C

import numpy as np
import pytest

from cwf import _lib, meshgen, pack, pcg, scenarios, shard
from helpers import oracle_system

OFF = np.array([[0, 0, 0], [1, 0, 0], [-1, 0, 0], [0, 1, 0], [0, -1, 0], [0, 0, 1], [0, 0, -1], [1, 1, 0],
                [-1, -1, 0], [1, 0, 1], [-1, 0, -1], [0, 1, 1], [0, -1, -1], [1, 1, 1], [-1, -1, -1]])
KUHN = [[0, 1, 3, 7], [0, 1, 5, 7], [0, 2, 3, 7], [0, 2, 6, 7], [0, 4, 5, 7], [0, 4, 6, 7]]
PAIRS = [(c, c2) for c in range(8) for c2 in range(8) if c == c2 or any(c in t and c2 in t for t in KUHN)]


def describe(system, renumber=True):
    L = _lib.load()
    desc = system.desc()
    dims = (C.c_uint32 * 3)()
    coef = np.zeros(549, np.float32)
    plane = np.zeros(1 << 16, np.uint32)
    st = L.cwf_lattice_describe(C.byref(desc), int(renumber), dims, coef.ctypes.data, plane.ctypes.data)
    assert st in (0, 1), st
    if st != 1:
        return None
    sym = bool(dims[0] >> 31)
    d = (dims[0] & 0x7FFFFFFF, dims[1], dims[2])
    return d, coef, plane[: d[2]].copy(), sym


def fast_system(case):
    sK, sM = case.scalars()
    return pcg.MatrixFreeSystem.from_packing(case.packing, case.materials, sK, sM, mode=_lib.MODE_FAST)


def lattice_apply(dims, coef, x3, sK):
    """K x (no mass, no Dirichlet) on an nx*ny*nz lattice in lexicographic order, the kernel's algorithm
    (lattice.inc): interior nodes by the difference-form stencil sum_(d != 0) S_d (u_(n+d) - u_n), surface nodes by
    the cell form (each existing cell's blocks on the differences to the node's own value)."""
    nx, ny, nz = dims
    u = np.pad(x3.reshape(nz, ny, nx, 3), ((1, 1), (1, 1), (1, 1), (0, 0)), mode="edge")
    S = coef[:135].astype(np.float64).reshape(15, 3, 3)
    Kp = coef[135:549].astype(np.float64).reshape(46, 3, 3)
    u0 = u[1:nz + 1, 1:ny + 1, 1:nx + 1]

    def nb(d):
        dx, dy, dz = d
        return u[1 + dz:nz + 1 + dz, 1 + dy:ny + 1 + dy, 1 + dx:nx + 1 + dx] - u0

    y = np.zeros((nz, ny, nx, 3))
    for o in range(1, 15):
        y += nb(OFF[o]) @ S[o].T
    k, j, i = np.meshgrid(np.arange(nz), np.arange(ny), np.arange(nx), indexing="ij")
    surface = (i == 0) | (i == nx - 1) | (j == 0) | (j == ny - 1) | (k == 0) | (k == nz - 1)
    ys = np.zeros_like(y)
    for c in range(8):
        cx, cy, cz = c & 1, (c >> 1) & 1, (c >> 2) & 1
        has = ((i >= 1) if cx else (i + 1 < nx)) & ((j >= 1) if cy else (j + 1 < ny)) & \
              ((k >= 1) if cz else (k + 1 < nz))
        t = np.zeros_like(y)
        for p, (a, b) in enumerate(PAIRS):
            if a == c and b != c:
                d = ((b & 1) - cx, ((b >> 1) & 1) - cy, ((b >> 2) & 1) - cz)
                t += nb(d) @ Kp[p].T
        ys += np.where(has[..., None], t, 0.0)
    y = np.where(surface[..., None], ys, y)
    return sK * y.reshape(-1, 3)


@pytest.mark.parametrize("name", ["8x3x4", "rayleigh", "rollers", "c1"])
def test_stencil_reproduces_the_oracle_operator(name):
    case = {"8x3x4": lambda: scenarios.block_case(8, 3, 4, h=0.1),
            "rayleigh": lambda: scenarios.block_case(6, 4, 3, h=0.1, xi=0.05, w=(10.0, 100.0)),
            "rollers": lambda: scenarios.roller_case(7, 5, 4),
            "c1": lambda: scenarios.config_case("c1")}[name]()
    P = case.packing
    out = describe(fast_system(case))
    assert out is not None
    dims, coef, plane, sym = out
    assert sym  # isotropic: S_(-d) == S_d
    assert dims == tuple(int(v) + 1 for v in meshgen_shape(case))
    assert np.array_equal(plane, np.arange(dims[2]) * dims[0] * dims[1])
    sK, sM = case.scalars()
    rng = np.random.Generator(np.random.PCG64(1))
    x = rng.uniform(-1, 1, P.dof_count).astype(np.float32)
    mask = (np.repeat(P.bc_mask, 3) & np.tile(np.array([1, 2, 4], np.uint32), P.node_count)) != 0
    xs = np.where(mask, 0.0, x.astype(np.float64))
    y = lattice_apply(dims, coef, xs, sK).reshape(-1) + sM * np.repeat(P.lumped_mass.astype(np.float64), 3) * xs
    y = np.where(mask, x, y)
    ref = oracle_system(P, case.materials, sK, sM).apply_keff(x).astype(np.float64)
    assert np.max(np.abs(y - ref)) <= 1e-6 * np.max(np.abs(ref))


def meshgen_shape(case):
    c = case.mesh.coords
    h = 0.1
    return np.round((c.max(0) - c.min(0)) / h).astype(int)


def test_jittered_mesh_is_refused():
    assert describe(fast_system(scenarios.block_case(6, 5, 4, h=0.1, jitter=True))) is None


def test_permuted_lattice_needs_renumbering():
    tm = meshgen.jitter_and_permute(meshgen.kuhn_block(5, 4, 3, 0.1), 0.1, jitter=0.0)
    mesh = pack.from_tetmesh(tm)
    cfg = scenarios.make_config()
    case = scenarios.Case("perm", mesh, cfg, pack.build_packed_buffers(mesh, cfg))
    s = fast_system(case)
    assert describe(s, renumber=False) is None
    dims, _, plane, _ = describe(s, renumber=True)
    assert dims == (6, 5, 4) and np.array_equal(plane, np.arange(4) * 30)


def test_slab_shard_local_order_is_a_lattice():
    """A slab shard's local order (owned planes, then the ghost planes of the rank below and above) is
    lexicographic within planes, so the shard keeps the lattice without renumbering (it cannot renumber)."""
    shape, nranks, r = (6, 5, 3), 3, 1
    case, node_global, begin = scenarios.slab_case_shape(shape, nranks, r)
    sK, sM = case.scalars()
    src = fast_system(case)
    sh = shard.build_shard(src, begin, r, node_global)
    s = sh.system(case.materials, sK, sM)
    dims, _, plane, _ = describe(s, renumber=False)
    A = (shape[0] + 1) * (shape[1] + 1)
    nplanes = dims[2]
    assert dims[:2] == (shape[0] + 1, shape[1] + 1) and nplanes * A == sh.local_nodes
    own = sh.owned_nodes // A
    # local planes in k order: the ghost plane below (stored after the owned planes), the owned planes, the ghost
    # plane above
    assert plane[0] == own * A and np.array_equal(plane[1:own + 1], np.arange(own) * A)
    assert plane[own + 1] == (own + 1) * A
