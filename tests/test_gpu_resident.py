"""The resident one-launch solve of a structured block (csrc/resident.hip, csrc/resident.cpp) against the pinned oracle
and against the launch-per-iteration fused schedule (lattice_fused.inc) it replaces on blocks that fit on chip.

The resident kernel runs lattice_fused.inc's per-node arithmetic (r, z, p, x formed by fused_form, the brick rows'
difference form, the shell's cell form); only the grouping of its fp64 dot sums differs (boxes of the lattice instead of
bricks), so it carries the FAST tolerance contract: solves at tol 1e-6 within 1e-4 (relative) of the oracle's solution in
its iteration count +-10%, and within 1e-5 of the fused schedule's x after 1, 2, 3 and 20 fixed iterations. Covered: the
box decomposition on blocks whose boxes are uneven or one cell thin, partial Dirichlet masks (rollers), Rayleigh scalars,
native hex8 cells, the max-iterations stop, run-to-run determinism and Newmark steps against the PARITY Stepper."""
import numpy as np
import pytest

import oracle as O
from cwf import _lib, pcg, scenarios
from cwf.stepper import Stepper
from helpers import oracle_system

pytestmark = pytest.mark.gpu

CASES = {
    "8x3x4": lambda: scenarios.block_case(8, 3, 4, h=0.1, tol=1e-6, max_iterations=600),
    "33x9x5": lambda: scenarios.block_case(33, 9, 5, h=0.1, tol=1e-6, max_iterations=800),
    "40x17x9": lambda: scenarios.block_case(40, 17, 9, h=0.1, tol=1e-6, max_iterations=1500),
    "thin-3x3x60": lambda: scenarios.block_case(3, 3, 60, h=0.1, tol=1e-6, max_iterations=2000),
    "rayleigh": lambda: scenarios.block_case(6, 4, 3, h=0.1, xi=0.05, w=(10.0, 100.0), tol=1e-6, max_iterations=600),
    "rollers": lambda: scenarios.roller_case(12, 10, 7, tol=1e-6, max_iterations=1500),
    "c1": lambda: scenarios.config_case("c1"),
}


def _kernel(s):
    return (_lib.load().cwf_hip_system_keff_kernel(s.handle()) or b"").decode()


def _system(case, monkeypatch=None, fused=None):
    if monkeypatch is not None:
        if fused is None:
            monkeypatch.delenv("CWF_FUSED", raising=False)
        else:
            monkeypatch.setenv("CWF_FUSED", fused)
    return pcg.MatrixFreeSystem.from_packing(case.packing, case.materials, *case.scalars(), mode=_lib.MODE_FAST)


def _solve(s, rhs, its, tol):
    x, r = np.zeros_like(rhs), np.zeros_like(rhs)
    t = pcg.solve_pcg(s, rhs, pcg.PcgSettings(its, tol), pcg.PcgVectors(x, r)).value()
    return t, x, r


@pytest.mark.parametrize("name", sorted(CASES))
def test_resident_solve_matches_oracle(name, monkeypatch):
    case = CASES[name]()
    s = _system(case, monkeypatch)
    assert _kernel(s).startswith("k_pcg_resident"), _kernel(s)
    rhs = case.static_rhs()
    mi = case.cfg.solver.max_iterations
    t, x, r = _solve(s, rhs, mi, 1e-6)
    ref = oracle_system(case.packing, case.materials, *case.scalars()).solve_pcg(rhs, mi, 1e-6)
    assert t.converged and ref["telemetry"].converged
    print(f"{name}: resident {t.iterations} it, oracle {ref['telemetry'].iterations} it")
    assert np.linalg.norm(x - ref["x"]) <= 1e-4 * np.linalg.norm(ref["x"])
    n_ref = ref["telemetry"].iterations
    assert abs(t.iterations - n_ref) <= max(3, n_ref // 10)
    # the r output is the solve's residual, its norm the telemetry's
    assert abs(np.linalg.norm(r.astype(np.float64)) - t.residual_norm) <= 1e-3 * t.residual_norm
    assert t.residual_norm <= 1e-6 * np.linalg.norm(rhs.astype(np.float64)) * 1.0001


@pytest.mark.parametrize("name", ["33x9x5", "40x17x9", "rollers", "c1"])
def test_resident_follows_the_fused_schedule(name, monkeypatch):
    """Fixed iteration counts (tol 1e-30): the resident x stays within 1e-5 of the fused launch-per-iteration x (the
    same per-node arithmetic, the dots grouped differently), and the full solves converge in counts within 5%."""
    case = CASES[name]()
    rhs = case.static_rhs()
    sr = _system(case, monkeypatch)
    assert _kernel(sr).startswith("k_pcg_resident")  # (the schedule is taken at the first ask, under this env)
    sf = _system(case, monkeypatch, fused="1")
    assert _kernel(sf).startswith("k_pcg_lattice")
    for its in (1, 2, 3, 20):
        tr, xr, _ = _solve(sr, rhs, its, 1e-30)
        tf, xf, _ = _solve(sf, rhs, its, 1e-30)
        assert tr.iterations == tf.iterations == its and not tr.converged
        d = np.linalg.norm(xr.astype(np.float64) - xf) / np.linalg.norm(xf.astype(np.float64))
        assert d <= 1e-5, (its, d)
        assert abs(tr.residual_norm - tf.residual_norm) <= 1e-4 * tf.residual_norm
    mi = case.cfg.solver.max_iterations
    tr, _, _ = _solve(sr, rhs, mi, 1e-6)
    tf, _, _ = _solve(sf, rhs, mi, 1e-6)
    assert tr.converged and tf.converged
    assert abs(tr.iterations - tf.iterations) <= max(3, tf.iterations // 20), (tr.iterations, tf.iterations)


def test_resident_hex8_solve(monkeypatch):
    """Native hex8 cells (the 27-point stencil, its 64-pair cell form on the surface) against the fp64 solve of the
    oracle's hex8 operator (parity unpinned by nature: the reference rejects hex8)."""
    case = scenarios.block_case(33, 9, 5, h=0.1, element="hex8", tol=1e-6, max_iterations=800)
    s = _system(case, monkeypatch)
    assert _kernel(s).startswith("k_pcg_resident<true, LatHex"), _kernel(s)
    rhs = case.static_rhs()
    t, x, _ = _solve(s, rhs, 800, 1e-6)
    assert t.converged
    P = case.packing
    ref = O.hex8_solve64(case.mesh.coords, case.mesh.tets, P.material_index, O.make_stiffness(30.0e9, 0.2),
                         *case.scalars(), P.lumped_mass, P.bc_mask, rhs)
    assert np.linalg.norm(x - ref) <= 1e-4 * np.linalg.norm(ref)


def test_resident_max_iterations_and_history(monkeypatch):
    case = CASES["40x17x9"]()
    s = _system(case, monkeypatch)
    rhs = case.static_rhs()
    t, _, _ = _solve(s, rhs, 7, 1e-12)
    assert (t.iterations, t.converged) == (7, False)
    h = pcg.residual_history(s)
    assert h.shape == (8,) and np.all(np.isfinite(h)) and h[-1] == t.residual_norm
    sf = _system(case, monkeypatch, fused="1")
    tf, _, _ = _solve(sf, rhs, 7, 1e-12)
    hf = pcg.residual_history(sf)
    assert np.allclose(h, hf, rtol=1e-5, atol=0.0)


def test_resident_run_to_run_deterministic(monkeypatch):
    case = CASES["40x17x9"]()
    rhs = case.static_rhs()
    s = _system(case, monkeypatch)
    runs = [_solve(s, rhs, 1500, 1e-6), _solve(s, rhs, 1500, 1e-6), _solve(_system(case, monkeypatch), rhs, 1500, 1e-6)]
    for t, x, r in runs[1:]:
        assert t.iterations == runs[0][0].iterations and t.residual_norm == runs[0][0].residual_norm
        assert np.array_equal(x.view(np.uint32), runs[0][1].view(np.uint32))
        assert np.array_equal(r.view(np.uint32), runs[0][2].view(np.uint32))


def test_resident_stepper_steps(monkeypatch):
    """Three Newmark steps (Rayleigh: the damping SpMV between solves, warm starts) against the PARITY Stepper."""
    monkeypatch.delenv("CWF_FUSED", raising=False)
    case = scenarios.block_case(10, 5, 6, h=0.1, xi=0.05, w=(10.0, 100.0), tol=1e-6, max_iterations=1500)
    P = case.packing
    ref = Stepper(P, case.materials, case.rayleigh, case.cfg.solver, case.cfg.time, mode=_lib.MODE_PARITY)
    fast = Stepper(P, case.materials, case.rayleigh, case.cfg.solver, case.cfg.time, mode=_lib.MODE_FAST)
    assert _kernel(fast.system).startswith("k_pcg_resident")
    for k in range(3):
        tr = ref.step(0.01 * k).value()
        tf = fast.step(0.01 * k).value()
        assert tf.pcg.converged and tr.pcg.converged
        assert abs(tf.pcg.iterations - tr.pcg.iterations) <= max(3, tr.pcg.iterations // 10)
    for what in (Stepper.DISPLACEMENT, Stepper.VELOCITY):
        ur, uf = ref.get_state(what), fast.get_state(what)
        assert np.linalg.norm(uf - ur) <= 1e-4 * np.linalg.norm(ur)


@pytest.mark.parametrize("element", ["tet4", "hex8"])
def test_resident_c3_slab_block_follows_two_kernels(element, monkeypatch):
    """The C3/8 slab's size (149 x 149 x 19 cells, 427k nodes): the 4-node instantiation with r, Ap, x in LDS and the
    box's own boundary-type stencils only (hex8: the 27-offset table of the box's types is what lets its image fit
    the LDS). After 3 and 20 fixed iterations x within 1e-5 of the two-kernel schedule's (CWF_FUSED=0)."""
    case = scenarios.block_case(149, 149, 19, h=0.1, element=element, tol=1e-30, max_iterations=20)
    rhs = case.static_rhs()
    sr = _system(case, monkeypatch)
    e = "LatHex" if element == "hex8" else "LatKuhn"
    assert _kernel(sr) == f"k_pcg_resident<true, {e}, 4, 3, false>", _kernel(sr)
    sk = _system(case, monkeypatch, fused="0")
    assert _kernel(sk).startswith("k_keff_lattice"), _kernel(sk)
    for its in (3, 20):
        tr, xr, _ = _solve(sr, rhs, its, 1e-30)
        tk, xk, _ = _solve(sk, rhs, its, 1e-30)
        assert tr.iterations == tk.iterations == its
        d = np.linalg.norm(xr.astype(np.float64) - xk) / np.linalg.norm(xk.astype(np.float64))
        assert d <= 1e-5, (its, d)
