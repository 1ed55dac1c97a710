"""Native hex8. PARITY UNPINNED: the reference rejects hex8 elements
(src/mesh/preprocess.cpp:326-330), so there is no reference output to match. The checks are:
  * the native host preprocess equals the fp64 oracle restatement (oracle/hex8_oracle.c) bit for bit;
  * the oracle operator has the physics of the isoparametric element (rigid modes in the kernel,
    constant-strain patch test on distorted hexes, symmetry, diagonal blocks);
  * hex8 and the pinned Kuhn-tet discretisation converge towards each other under refinement;
  * GPU (FAST mode, fp32 sum-factorised kernel) against the oracle with the tolerances written below.
"""
import numpy as np
import pytest

import oracle as O
from cwf import _lib, meshgen, pack, pcg, scenarios
from cwf.stepper import Stepper
from cwf.physics import SolverSettings, TimeSettings
from helpers import oracle_system


def jittered_hex(nx, ny, nz, h=0.1, amp=0.2, seed=7):
    tm = meshgen.hex_block(nx, ny, nz, h)
    c = tm.coords.copy()
    lo, hi = c.min(0), c.max(0)
    inner = np.all((c > lo + 1e-9) & (c < hi - 1e-9), 1)
    rng = np.random.Generator(np.random.PCG64(seed))
    c[inner] += rng.uniform(-amp * h, amp * h, (int(inner.sum()), 3))
    tm.coords = c
    return tm, inner


def hex_case(nx, ny, nz, jitter=0.0, **kw):
    case = scenarios.block_case(nx, ny, nz, element="hex8", **kw)
    if jitter:
        tm, _ = jittered_hex(nx, ny, nz, amp=jitter)
        mesh = pack.from_tetmesh(tm)
        case = scenarios.Case(case.name + "-jitter", mesh, case.cfg, pack.build_packed_buffers(mesh, case.cfg))
    return case


D_STEEL = O.make_stiffness(30.0e9, 0.2)


# ------------------------------------------------------------------------------------ CPU ----
def test_hex8_preprocess_native_equals_oracle():
    case = hex_case(5, 3, 4, jitter=0.2)
    P = case.packing
    vol, m64, gr = O.hex8_preprocess(case.mesh.coords, case.mesh.tets, P.material_index, [2500.0])
    assert np.array_equal(vol.astype(np.float32), P.volume)
    assert np.array_equal(m64, P.lumped_mass64)
    assert np.array_equal(gr, P.gradients)
    assert P.element_indices.size == 8 * P.element_count and P.local_indices.max() == 7
    assert abs(P.volume.astype(np.float64).sum() - 0.5 * 0.3 * 0.4) < 1e-7


def test_hex8_preprocess_rejects_inverted_element():
    tm = meshgen.hex_block(2, 1, 1, 0.1)
    tm.tets[1] = tm.tets[1][[4, 5, 6, 7, 0, 1, 2, 3]]  # mirrored: det J < 0
    mesh = pack.from_tetmesh(tm)
    with pytest.raises(pack.PackError) as e:
        pack.build_packed_buffers(mesh, scenarios.make_config())
    assert e.value.message == "hexahedron Jacobian non-positive (inverted or degenerate)"
    assert e.value.context == ["elements [1]"]


def test_hex8_oracle_rigid_modes_and_patch_test():
    tm, inner = jittered_hex(4, 3, 3, amp=0.2)
    c, hexes = tm.coords, tm.tets
    N, E = c.shape[0], hexes.shape[0]
    mat = np.zeros(E, np.uint32)
    _, m64, _ = O.hex8_preprocess(c, hexes, mat, [2500.0])
    mask = np.zeros(N, np.uint32)
    mass = m64.astype(np.float32)
    scale = 30.0e9 * 0.1  # E h: the magnitude of a stiffness entry
    # rigid translation and (linearised) rotation -> no forces
    for u in (np.tile([1.0, -2.0, 0.5], N),
              np.cross(np.array([0.3, -0.2, 0.5]), c - c.mean(0)).reshape(-1)):
        y = O.hex8_apply(c, hexes, mat, D_STEEL, 1.0, 0.0, mass, mask, u.astype(np.float32))
        assert np.abs(y).max() <= 1e-6 * scale * np.abs(u).max()
    # constant-strain patch test on distorted hexes: interior nodes carry no force
    A = np.array([[1.0, 2.0, -3.0], [0.5, -1.0, 2.0], [3.0, 1.0, 0.25]]) * 1e-3
    u = (c @ A.T).astype(np.float32).reshape(-1)
    y = O.hex8_apply(c, hexes, mat, D_STEEL, 1.0, 0.0, mass, mask, u).reshape(-1, 3)
    assert np.abs(y[inner]).max() <= 1e-6 * np.abs(y[~inner]).max()


def test_hex8_oracle_symmetric_positive_and_diag_blocks():
    tm, _ = jittered_hex(3, 3, 2, amp=0.2)
    c, hexes = tm.coords, tm.tets
    N, E = c.shape[0], hexes.shape[0]
    mat = np.zeros(E, np.uint32)
    mask = np.zeros(N, np.uint32)
    mass = np.zeros(N, np.float32)
    rng = np.random.Generator(np.random.PCG64(5))
    a, b = rng.standard_normal((2, 3 * N)).astype(np.float32)
    Ka = O.hex8_apply(c, hexes, mat, D_STEEL, 1.0, 0.0, mass, mask, a).astype(np.float64)
    Kb = O.hex8_apply(c, hexes, mat, D_STEEL, 1.0, 0.0, mass, mask, b).astype(np.float64)
    assert abs(b @ Ka - a @ Kb) <= 1e-6 * abs(a @ Ka)
    assert a @ Ka > 0 and b @ Kb > 0
    blk = O.hex8_diag_blocks(c, hexes, mat, D_STEEL, 1.0)
    for n in (0, N // 2, N - 1):
        col = np.zeros((3, 3))
        for k in range(3):
            e = np.zeros(3 * N, np.float32)
            e[3 * n + k] = 1.0
            col[:, k] = O.hex8_apply(c, hexes, mat, D_STEEL, 1.0, 0.0, mass, mask, e)[3 * n:3 * n + 3]
        assert np.abs(col - blk[n]).max() <= 1e-6 * np.abs(blk[n]).max()


def _dense_tip_deflection(n, element):
    """static cantilever (x=0 fixed, -z load on the tip face), dense solve of the oracle operator"""
    case = scenarios.block_case(4 * n, n, n, h=0.4 / (4 * n), element=element, gravity=(0.0, 0.0, 0.0))
    P = case.packing
    D = P.dof_count
    if element == "hex8":
        apply = lambda x: O.hex8_apply(case.mesh.coords, case.mesh.tets, P.material_index, D_STEEL, 1.0, 0.0,
                                       P.lumped_mass, P.bc_mask, x)
    else:
        o = oracle_system(P, case.materials, 1.0, 0.0)
        apply = o.apply_keff
    K = np.zeros((D, D))
    for j in range(D):
        e = np.zeros(D, np.float32)
        e[j] = 1.0
        K[:, j] = apply(e)
    u = np.linalg.solve(K, case.static_rhs().astype(np.float64))
    tip = case.mesh.node_groups[case.mesh.group_names["TIP"]]
    return u.reshape(-1, 3)[tip.astype(np.int64), 2].mean() / P.external_force.reshape(-1, 3)[tip, 2].sum()


def test_hex8_and_kuhn_tets_converge_together():
    gaps = []
    for n in (1, 2, 3):
        h8, t4 = _dense_tip_deflection(n, "hex8"), _dense_tip_deflection(n, "tet4")
        assert h8 > 0 and t4 > 0  # compliance per unit load, both meshes deflect with the load
        gaps.append(abs(h8 - t4) / abs(t4))
    # linear tets are the stiffer (locking) discretisation; the gap closes under refinement
    assert gaps[2] < gaps[1] < gaps[0]


# ------------------------------------------------------------------------------------ GPU ----
def gpu_hex_system(case, sK=None, sM=None, mode=_lib.MODE_FAST):
    s0, m0 = case.scalars()
    return pcg.MatrixFreeSystem.from_packing(case.packing, case.materials, s0 if sK is None else sK,
                                             m0 if sM is None else sM, mode=mode)


GPU_CASES = {
    "block": lambda: hex_case(9, 5, 6, tol=1e-6, max_iterations=800),
    "jitter": lambda: hex_case(8, 6, 5, jitter=0.2, tol=1e-6, max_iterations=800),
    "tiles": lambda: hex_case(24, 12, 10, tol=1e-6, max_iterations=2000),  # many tiles, partial last tile
}


@pytest.fixture(scope="module", params=sorted(GPU_CASES))
def hcase(request):
    return GPU_CASES[request.param]()


@pytest.mark.gpu
def test_gpu_hex8_apply_keff_matches_oracle(hcase):
    s = gpu_hex_system(hcase)
    P = hcase.packing
    sK, sM = hcase.scalars()
    rng = np.random.Generator(np.random.PCG64(11))
    x = rng.uniform(-1, 1, P.dof_count).astype(np.float32)
    y = np.zeros_like(x)
    pcg.apply_keff(s, x, y).value()
    ref = O.hex8_apply(hcase.mesh.coords, hcase.mesh.tets, P.material_index, D_STEEL, sK, sM, P.lumped_mass,
                       P.bc_mask, x).astype(np.float64)
    # fp32 sum-factorised element math vs the fp64 oracle, relative to the operator scale (max |row|)
    assert np.max(np.abs(y - ref)) <= 2e-5 * np.max(np.abs(ref))
    mask = np.repeat(P.bc_mask, 3) & np.tile(np.array([1, 2, 4], np.uint32), P.node_count)
    assert np.array_equal(y[mask != 0], x[mask != 0])  # Dirichlet rows pass x through


def _keff_kernel(s):
    return (_lib.load().cwf_hip_system_keff_kernel(s.handle()) or b"").decode()


@pytest.mark.gpu
def test_gpu_hex8_structured_blocks_run_the_lattice_stencil(hcase):
    """A structured hex block (every hex a cell of one box lattice) runs the 27-point stencil of the shared
    trilinear cell stiffness (lattice.cpp); a jittered one the hex tiles. Either way the apply test above holds."""
    kern = _keff_kernel(gpu_hex_system(hcase))
    # an isotropic block's stencil is point-symmetric (S_-d = S_d): the paired-direction instantiation
    want = (("k_keff_hex_tiles",) if hcase.name.endswith("-jitter") else
            ("k_keff_lattice<1, false, true, LatHex,", "k_pcg_lattice<true, LatHex,", "k_pcg_resident<true, LatHex,"))
    assert kern.startswith(want), kern


@pytest.mark.gpu
def test_gpu_hex8_lattice_z_from_r_solve(monkeypatch):
    """The hex8 lattice with z formed from r in the K_eff pass (CWF_LAT_ZR=1, the default from 2M nodes) solves to
    the stored-z solution (the same p bit for bit; the iteration count equal up to the initial z's source)."""
    case = GPU_CASES["tiles"]()
    rhs = case.static_rhs()
    xs = {}
    monkeypatch.setenv("CWF_FUSED", "0")  # the two-kernel iteration's z source (the fused one always forms z from r)
    for zr in ("0", "1"):
        monkeypatch.setenv("CWF_LAT_ZR", zr)
        s = gpu_hex_system(case)
        assert _keff_kernel(s).rstrip(">").split(", ")[-3:-1] == ["true", "true" if zr == "1" else "false"]
        xs[zr] = np.zeros_like(rhs)
        t = pcg.solve_pcg(s, rhs, pcg.PcgSettings(2000, 1e-6), pcg.PcgVectors(xs[zr], np.zeros_like(rhs))).value()
        assert t.converged
    assert np.linalg.norm(xs["1"] - xs["0"]) <= 1e-4 * np.linalg.norm(xs["0"])


@pytest.mark.gpu
def test_gpu_hex8_256_lane_tiles_apply_and_solve(hcase, monkeypatch):
    """The 256-lane hex tiles (the default from 1M hexes; CWF_HEX_NT=256 forces them here, with the structured-block
    stencil off) keep the apply tolerance and the PCG solution of the 128-lane tiles, and the lattice stencil's."""
    rhs = hcase.static_rhs()
    xl = np.zeros_like(rhs)
    pcg.solve_pcg(gpu_hex_system(hcase), rhs, pcg.PcgSettings(2000, 1e-6),
                  pcg.PcgVectors(xl, np.zeros_like(rhs))).value()
    monkeypatch.setenv("CWF_LATTICE", "0")
    monkeypatch.setenv("CWF_HEX_NT", "256")
    s = gpu_hex_system(hcase)
    P = hcase.packing
    sK, sM = hcase.scalars()
    rng = np.random.Generator(np.random.PCG64(12))
    x = rng.uniform(-1, 1, P.dof_count).astype(np.float32)
    y = np.zeros_like(x)
    pcg.apply_keff(s, x, y).value()
    ref = O.hex8_apply(hcase.mesh.coords, hcase.mesh.tets, P.material_index, D_STEEL, sK, sM, P.lumped_mass,
                       P.bc_mask, x).astype(np.float64)
    assert np.max(np.abs(y - ref)) <= 2e-5 * np.max(np.abs(ref))
    rhs = hcase.static_rhs()
    x256 = np.zeros_like(rhs)
    t = pcg.solve_pcg(s, rhs, pcg.PcgSettings(2000, 1e-6), pcg.PcgVectors(x256, np.zeros_like(rhs))).value()
    assert t.converged
    monkeypatch.setenv("CWF_HEX_NT", "128")
    x128 = np.zeros_like(rhs)
    s128 = gpu_hex_system(hcase)
    assert _keff_kernel(s128).startswith("k_keff_hex_tiles")
    pcg.solve_pcg(s128, rhs, pcg.PcgSettings(2000, 1e-6), pcg.PcgVectors(x128, np.zeros_like(rhs))).value()
    assert np.linalg.norm(x256 - x128) <= 1e-4 * np.linalg.norm(x128)
    assert np.linalg.norm(xl - x128) <= 1e-4 * np.linalg.norm(x128)


@pytest.mark.gpu
def test_gpu_hex8_block_jacobi_matches_oracle(hcase):
    s = gpu_hex_system(hcase)
    P = hcase.packing
    sK, sM = hcase.scalars()
    inv = np.zeros(9 * P.node_count, np.float32)
    pcg.build_block_jacobi_inverse(s, None, inv).value()
    blk = O.hex8_diag_blocks(hcase.mesh.coords, hcase.mesh.tets, P.material_index, D_STEEL, sK)
    blk += (P.lumped_mass.astype(np.float64) * sM)[:, None, None] * np.eye(3)[None]
    ref = np.linalg.inv(blk)
    for k in range(3):
        c = (P.bc_mask & (1 << k)) != 0
        ref[c, k, :] = 0.0
        ref[c, k, k] = 1.0
    got = inv.reshape(-1, 3, 3).astype(np.float64)
    # constrained rows are identity (1.0) while free entries are ~1/K ~ 1e-10: compare each entry against
    # its own row/column scale sqrt(B_ii B_jj) of the fp64 block, so the free entries are really checked
    free = ((P.bc_mask[:, None] >> np.arange(3)[None]) & 1) == 0
    d = np.abs(np.einsum("nii->ni", ref))
    scale = np.sqrt(d[:, :, None] * d[:, None, :])
    rows = np.repeat(free[:, :, None], 3, 2)
    assert np.all(np.abs(got - ref)[rows] <= 1e-5 * scale[rows])
    assert np.array_equal(got[~free], ref[~free])  # identity rows


@pytest.mark.gpu
def test_gpu_hex8_pcg_solution_satisfies_oracle_operator(hcase):
    s = gpu_hex_system(hcase)
    P = hcase.packing
    sK, sM = hcase.scalars()
    rhs = hcase.static_rhs()
    x = np.zeros_like(rhs)
    t = pcg.solve_pcg(s, rhs, pcg.PcgSettings(2000, 1e-6), pcg.PcgVectors(x, np.zeros_like(rhs))).value()
    assert t.converged and t.iterations > 1
    ref = O.hex8_solve64(hcase.mesh.coords, hcase.mesh.tets, P.material_index, D_STEEL, sK, sM, P.lumped_mass,
                         P.bc_mask, rhs)
    # |r| <= 1e-6 |rhs| in the device's fp32 operator; against the fp64 solution (fp64 PCG to 1e-11)
    # the solutions agree to 1e-4 relative (fp32 operator rounding x the problem's conditioning)
    assert np.linalg.norm(x - ref) <= 1e-4 * np.linalg.norm(ref)


@pytest.mark.gpu
def test_gpu_hex8_pcg_with_partial_masks():
    """rollers on three faces (partial masks, physical units): the packed FAST preconditioner keeps the
    free entries of the partly constrained nodes, so the solve converges to the fp64 solution"""
    case = scenarios.roller_case(10, 5, 5, element="hex8", tol=1e-6, max_iterations=2000)
    s = gpu_hex_system(case)
    P = case.packing
    sK, sM = case.scalars()
    rhs = case.static_rhs()
    x = np.zeros_like(rhs)
    t = pcg.solve_pcg(s, rhs, pcg.PcgSettings(2000, 1e-6), pcg.PcgVectors(x, np.zeros_like(rhs))).value()
    assert t.converged and t.iterations < 1000
    applied = np.zeros(9 * P.node_count, np.float32)
    assert pcg.fast_block_inverse(s, applied).value() == 0  # no fp32 fallback block
    ref = O.hex8_solve64(case.mesh.coords, case.mesh.tets, P.material_index, D_STEEL, sK, sM, P.lumped_mass,
                         P.bc_mask, rhs)
    assert np.linalg.norm(x - ref) <= 1e-4 * np.linalg.norm(ref)


@pytest.mark.gpu
def test_gpu_hex8_stepper_runs_and_deflects():
    case = hex_case(12, 4, 4, tol=1e-6, max_iterations=1500)
    P = case.packing
    st = Stepper(P, case.materials, case.rayleigh, SolverSettings("pcg", "block_jacobi", 1e-6, 1e-5, 1500),
                 TimeSettings(0.01, False, 0.0, 0.0), mode=_lib.MODE_FAST)
    for i in range(3):
        tel = st.step(0.01 * i).value()
        assert tel.pcg.converged
    u = st.get_state(Stepper.DISPLACEMENT).reshape(-1, 3)
    tip = case.mesh.node_groups[case.mesh.group_names["TIP"]].astype(np.int64)
    fixed = case.mesh.node_groups[case.mesh.group_names["FIXED"]].astype(np.int64)
    assert np.all(np.isfinite(u)) and np.all(u[fixed] == 0.0)
    assert u[tip, 2].mean() < 0.0  # gravity + the -z tip load push the free end down


@pytest.mark.gpu
def test_gpu_hex8_parity_mode_is_rejected():
    case = hex_case(2, 2, 2)
    s = gpu_hex_system(case, mode=_lib.MODE_PARITY)
    with pytest.raises(pcg.PcgException) as e:
        s.handle()
    assert "hex8 elements run in CWF_MODE_FAST only" in str(e.value)


@pytest.mark.gpu
def test_gpu_hex8_derived_fields_centroid_strain():
    """post stack on hex8: element strain/stress at the element centre (the grads24 slots)."""
    case = hex_case(4, 3, 2, jitter=0.2)
    P = case.packing
    s = gpu_hex_system(case, 1.0, 0.0)
    A = np.array([[1.0, 2.0, -3.0], [0.5, -1.0, 2.0], [3.0, 1.0, 0.25]]) * 1e-4
    u = (case.mesh.coords @ A.T).astype(np.float32).reshape(-1)
    from cwf import post
    ds = post.compute_derived_fields(P, case.materials, system=s, displacement=u)
    ef, nf = ds.elements.astype(np.float64), ds.nodes.astype(np.float64)
    # a linear field has the same strain everywhere: eps = sym(A) in engineering Voigt
    want = np.array([A[0, 0], A[1, 1], A[2, 2], A[0, 1] + A[1, 0], A[1, 2] + A[2, 1], A[0, 2] + A[2, 0]])
    assert np.abs(ef[:, :6] - want).max() <= 1e-5 * np.abs(want).max()
    sig = D_STEEL.reshape(6, 6) @ want
    assert np.abs(ef[:, 6:12] - sig).max() <= 1e-5 * np.abs(sig).max()
    assert np.abs(nf[:, :6] - want).max() <= 1e-5 * np.abs(want).max()


@pytest.mark.gpu
def test_gpu_hex8_gmsh_scenario_end_to_end(tmp_path):
    """YAML + Gmsh hex8 mesh -> cwf.run (FAST) -> VTU (VTK_HEXAHEDRON cells) and probes."""
    from cwf import run
    from scenario_files import write_block_scenario
    y = write_block_scenario(str(tmp_path), 6, 3, 3, tol=1e-6, stride=1, element="hex8")
    with pytest.raises(run.ScenarioError):  # the reference path (PARITY) keeps rejecting hex8
        run.run_scenario(y, 1, None, _lib.MODE_PARITY, log=lambda s: None)
    out = tmp_path / "out"
    s = run.run_scenario(y, 2, str(out), _lib.MODE_FAST, log=lambda s: None)
    assert s["steps"] == 2 and s["last"]["converged"] and s["tets"] == 6 * 3 * 3
    vtu = (out / "vtu" / "frame_00001.vtu").read_bytes()
    assert b'NumberOfCells="54"' in vtu
