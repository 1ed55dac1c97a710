"""Every BASELINE.json config through the HIP path at its full size.

C2 and C3 live in test_gpu_fullsize.py; this file covers the other three.

C1 = configs[0] (cantilever 20x5x10 hex -> 6,000 Kuhn tets, 4,158 DOF, tol 2e-4 as cantilever.yaml:23):
  PARITY solve_pcg and three Stepper steps bit-exact against the pinned oracle, FAST within tolerance.
C4 = configs[3] (jittered + permuted 118^3 block -> 9.86M tets, 5.06M DOF, harmonic tip load
  F0 sin(2 pi 5 t) as a 64-point curve): PARITY apply_keff bit-exact over the whole vector, the FAST
  properties, and the harmonic load rewritten on the device every step (cwf_hip_stepper_set_load_scale),
  bitwise the host's assemble_load_vector; on the small jittered mesh five harmonic-load Newmark steps are
  bit-exact against the oracle Stepper fed the host vector (viewer.cpp:262-266 rewrites external_force).
C5 = configs[4] (slab 800x400x50 -> 96M tets, 49.1M DOF on one GPU): PARITY apply_keff bit-exact over the
  whole vector and the FAST properties.

FAST tolerances: the fp32 element math of FAST K_eff is within 2e-5 of the bit-exact operator relative to
its scale (max |row|); the constrained operator is symmetric to 1e-5 of a^T K a; solves at tol 1e-6 agree
with the oracle's to 1e-4 relative; a FAST Newmark step converges in the PARITY step's iteration count +-15%.
"""
import numpy as np
import pytest

import oracle as O
from cwf import _lib, pcg, scenarios
from cwf.stepper import Stepper
from helpers import assert_bitwise, check_step_against_parity, oracle_system

pytestmark = pytest.mark.gpu


def _system(case, mode, sK=None, sM=None):
    s0, m0 = case.scalars()
    return pcg.MatrixFreeSystem.from_packing(case.packing, case.materials, s0 if sK is None else sK,
                                             m0 if sM is None else sM, mode=mode)


def _oracle_stepper(case, o):
    r = case.rayleigh
    s = case.cfg.solver
    return O.Stepper(o, case.packing.external_force, case.packing.bc_value, (r.alpha, r.beta), s.runtime_tolerance,
                     s.pause_tolerance, s.max_iterations, case.cfg.time.initial_dt)


def _fast_properties(case, sp, sf, seed):
    """FAST within 2e-5 of PARITY (operator scale) and symmetric on the free dofs; returns PARITY K x."""
    P = case.packing
    o = oracle_system(P, case.materials, *case.scalars())
    rng = np.random.Generator(np.random.PCG64(seed))
    x = rng.uniform(-1, 1, P.dof_count).astype(np.float32)
    yp, yf = np.zeros_like(x), np.zeros_like(x)
    pcg.apply_keff(sp, x, yp).value()
    assert_bitwise(yp, o.apply_keff(x), f"{case.name} apply_keff")
    del o
    pcg.apply_keff(sf, x, yf).value()
    assert np.max(np.abs(yf.astype(np.float64) - yp)) <= 2e-5 * np.max(np.abs(yp))
    free = (np.repeat(P.bc_mask, 3) & np.tile(np.array([1, 2, 4], np.uint32), P.node_count)) == 0
    a = np.where(free, rng.standard_normal(P.dof_count), 0.0).astype(np.float32)
    b = np.where(free, rng.standard_normal(P.dof_count), 0.0).astype(np.float32)
    Ka, Kb = np.zeros_like(a), np.zeros_like(b)
    pcg.apply_keff(sf, a, Ka).value()
    pcg.apply_keff(sf, b, Kb).value()
    ab, ba = float(b.astype(np.float64) @ Ka), float(a.astype(np.float64) @ Kb)
    assert abs(ab - ba) <= 1e-5 * abs(float(a.astype(np.float64) @ Ka))


# ------------------------------------------------------------------------------------------------ C1
@pytest.fixture(scope="module")
def c1():
    return scenarios.config_case("c1")


def test_c1_config_shape(c1):
    assert (c1.packing.node_count, c1.packing.element_count, c1.packing.dof_count) == (1386, 6000, 4158)
    assert c1.cfg.solver.runtime_tolerance == 2e-4


def test_c1_parity_solve_bitwise_with_history(c1):
    s = _system(c1, _lib.MODE_PARITY)
    o = oracle_system(c1.packing, c1.materials, *c1.scalars())
    rhs = c1.static_rhs()
    tol = c1.cfg.solver.runtime_tolerance
    x, r = np.zeros_like(rhs), np.zeros_like(rhs)
    t = pcg.solve_pcg(s, rhs, pcg.PcgSettings(2000, tol), pcg.PcgVectors(x, r)).value()
    ref = o.solve_pcg(rhs, 2000, tol, history=True)
    rt = ref["telemetry"]
    assert t.converged and (t.iterations, t.converged) == (rt.iterations, bool(rt.converged))
    assert (t.residual_norm, t.rhs_norm, t.alpha_last, t.beta_last) == (rt.residual_norm, rt.rhs_norm,
                                                                          rt.alpha_last, rt.beta_last)
    assert_bitwise(x, ref["x"], "C1 x")
    assert_bitwise(r, ref["r"], "C1 r")
    assert np.array_equal(pcg.residual_history(s), ref["history"])


def test_c1_parity_stepper_three_steps_bitwise(c1):
    P = c1.packing
    st = Stepper(P, c1.materials, c1.rayleigh, c1.cfg.solver, c1.cfg.time)
    ost = _oracle_stepper(c1, oracle_system(P, c1.materials, *c1.scalars()))
    for k in range(3):
        t = st.step(k * 0.01).value()
        rt = ost.step(k * 0.01)
        assert t.pcg.converged
        assert (t.pcg.iterations, t.pcg.residual_norm) == (rt.pcg.iterations, rt.pcg.residual_norm)
    for which, ref in ((Stepper.DISPLACEMENT, ost.u), (Stepper.VELOCITY, ost.v), (Stepper.ACCELERATION, ost.a)):
        assert_bitwise(st.get_state(which), ref, f"C1 state {which}")


def test_c1_fast_solve_close(c1):
    s = _system(c1, _lib.MODE_FAST)
    o = oracle_system(c1.packing, c1.materials, *c1.scalars())
    rhs = c1.static_rhs()
    x = np.zeros_like(rhs)
    t = pcg.solve_pcg(s, rhs, pcg.PcgSettings(3000, 1e-6), pcg.PcgVectors(x, np.zeros_like(rhs))).value()
    ref = o.solve_pcg(rhs, 3000, 1e-6)
    assert t.converged and ref["telemetry"].converged
    assert np.linalg.norm(x - ref["x"]) <= 1e-4 * np.linalg.norm(ref["x"])
    assert abs(t.iterations - ref["telemetry"].iterations) <= max(3, ref["telemetry"].iterations // 10)


# ------------------------------------------------------------------------------------------------ C4
def _harmonic_run(case, mode, steps, oracle=False):
    """`steps` Newmark steps with the harmonic tip load rewritten before each one on the device
    (set_load_scale); returns the Stepper, its telemetries and (oracle=True) the oracle Stepper that was fed
    the host's load vector at the same times."""
    P = case.packing
    st = Stepper(P, case.materials, case.rayleigh, case.cfg.solver, case.cfg.time, mode=mode)
    st.set_load_pattern(*case.load_pattern())
    ost = _oracle_stepper(case, oracle_system(P, case.materials, *case.scalars())) if oracle else None
    tels = []
    t = 0.0
    for k in range(steps):
        st.set_load_scale(case.load_scale(t))
        f = case.external_force_at(t)
        assert_bitwise(st.get_state(Stepper.EXTERNAL_FORCE), f, f"device load at t={t}")
        tel = st.step(t).value()
        tels.append(tel)
        if ost is not None:
            ost.set_external_force(f)
            rt = ost.step(t)
            assert (tel.pcg.iterations, tel.pcg.residual_norm) == (rt.pcg.iterations, rt.pcg.residual_norm), k
        t += case.cfg.time.initial_dt
    return st, tels, ost


def test_c4_small_harmonic_parity_steps_bitwise():
    """Five Newmark steps under F0 sin(2 pi 5 t) (the C4 load) on a small jittered + permuted mesh: the
    device-rewritten load equals the host vector bit for bit and u / v / a equal the oracle Stepper's."""
    case = scenarios.block_case(7, 6, 5, h=0.1, jitter=True, harmonic=5.0, tol=1e-6, max_iterations=800)
    st, tels, ost = _harmonic_run(case, _lib.MODE_PARITY, 5, oracle=True)
    assert all(t.pcg.converged for t in tels)
    for which, ref in ((Stepper.DISPLACEMENT, ost.u), (Stepper.VELOCITY, ost.v), (Stepper.ACCELERATION, ost.a)):
        assert_bitwise(st.get_state(which), ref, f"harmonic state {which}")
    assert np.abs(ost.u).max() > 0


def test_c4_small_harmonic_fast_steps_close():
    case = scenarios.block_case(7, 6, 5, h=0.1, jitter=True, harmonic=5.0, tol=1e-6, max_iterations=800)
    sp, tp, _ = _harmonic_run(case, _lib.MODE_PARITY, 5)
    sf, tf, _ = _harmonic_run(case, _lib.MODE_FAST, 5)  # renumbered handle: the pattern is permuted too
    for a, b in zip(tp, tf):
        assert b.pcg.converged and abs(a.pcg.iterations - b.pcg.iterations) <= max(3, a.pcg.iterations // 10)
    up, uf = sp.get_state(Stepper.DISPLACEMENT), sf.get_state(Stepper.DISPLACEMENT)
    assert np.linalg.norm(uf - up) <= 1e-4 * np.linalg.norm(up)


@pytest.fixture(scope="module")
def c4():
    return scenarios.config_case("c4")


def test_c4_config_shape(c4):
    P = c4.packing
    assert (P.node_count, P.element_count, P.dof_count) == (1685159, 9858192, 5055477)
    assert c4.load_curve is not None


@pytest.mark.timeout(600)
def test_c4_parity_apply_bitwise_and_fast_properties(c4):
    sp = _system(c4, _lib.MODE_PARITY)
    sf = _system(c4, _lib.MODE_FAST)
    _fast_properties(c4, sp, sf, 41)
    sp.close()
    sf.close()


@pytest.mark.timeout(600)
def test_c4_harmonic_newmark_step_fast_matches_parity(c4):
    """One full-size C4 Newmark step at t = 0.01 under the harmonic load written on the device: FAST converges in the
    PARITY step's iteration count +-15% to the PARITY step's increment and displacement within
    helpers.STEP_REL_TOL (both steps start from rest, so both solve the same RHS), and both handles hold the host's
    load vector."""
    its, out = {}, {}
    P = c4.packing
    for mode in (_lib.MODE_PARITY, _lib.MODE_FAST):
        st = Stepper(P, c4.materials, c4.rayleigh, c4.cfg.solver, c4.cfg.time, mode=mode)
        st.set_load_pattern(*c4.load_pattern())
        st.set_load_scale(c4.load_scale(0.01))
        assert_bitwise(st.get_state(Stepper.EXTERNAL_FORCE), c4.external_force_at(0.01), "C4 device load")
        tel = st.step(0.01).value()
        assert tel.pcg.converged
        its[mode] = tel.pcg.iterations
        out[mode] = (tel.pcg, st.get_state(Stepper.SOLUTION).copy(), st.get_state(Stepper.DISPLACEMENT).copy())
        st.close()
        st.system.close()
    assert abs(its[_lib.MODE_FAST] - its[_lib.MODE_PARITY]) <= 0.15 * its[_lib.MODE_PARITY]
    (_, xp, up), (_, xf, uf) = out[_lib.MODE_PARITY], out[_lib.MODE_FAST]
    check_step_against_parity(xf, xp, uf, up, "C4 step")


# ------------------------------------------------------------------------------------------------ C5
@pytest.mark.timeout(1200)
def test_c5_parity_apply_bitwise_and_fast_properties():
    c5 = scenarios.config_case("c5")
    P = c5.packing
    assert (P.node_count, P.element_count, P.dof_count) == (16381251, 96000000, 49143753)
    sp = _system(c5, _lib.MODE_PARITY)
    sf = _system(c5, _lib.MODE_FAST)
    _fast_properties(c5, sp, sf, 51)
    sp.close()
    sf.close()
