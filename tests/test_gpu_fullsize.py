"""BASELINE.json's full sizes on the GPU.

C2 = configs[1] (69^3 hex block -> 1,971,054 Kuhn tets, 1.03M DOF): PARITY is bit-exact against the
pinned oracle at full size: apply_keff, the block-Jacobi inverse, and 25 PCG iterations (x, r, the fp64
residual history, the max-iterations stop).
C2 in FAST, the benchmarked kernel at the benchmarked size: the resident one-launch solve
k_pcg_resident (245 workgroups, one per box) and the fused launch-per-iteration k_pcg_lattice (its one-round grid of 436
workgroups, 112 of them shell workgroups, 436 x 5 shares folded per prologue) each solve a static system at tol 1e-6 to the PARITY solution (which is the oracle's solve_pcg bit for bit: the 25-iteration
test below and the full C1 solve in test_gpu_configs.py) within 1e-4 relative, in its iteration count +-5%; and two
Newmark steps at the config's runtime tolerance follow the PARITY Stepper's (iterations +-3, u / v / the increment
within helpers.STEP_REL_TOL = 1e-4 relative, where 0.9e-6 is measured).
C3 = configs[2] (149^3 -> 19.8M tets, 10.1M DOF, Rayleigh): PARITY apply_keff bit-exact against the
oracle over the whole vector, 8 PARITY PCG iterations bit-exact (multi-block scalar folds), plus size-independent
properties of the FAST path: symmetry of the constrained operator, rigid translation in the interior, FAST within 2e-5
of PARITY (relative to the operator scale), and a FAST Newmark step that converges with the PARITY step's iteration
count +-15% to the PARITY step's increment and displacement within helpers.STEP_REL_TOL, as C2's.
"""
import numpy as np
import pytest

from cwf import _lib, pcg, scenarios
from cwf.stepper import Stepper
from helpers import STEP_REL_TOL, assert_bitwise, check_step_against_parity, oracle_system

pytestmark = pytest.mark.gpu

def _kernel(s):
    return (_lib.load().cwf_hip_system_keff_kernel(s.handle()) or b"").decode()




@pytest.fixture(scope="module")
def c2():
    return scenarios.config_case("c2")


@pytest.fixture(scope="module")
def c3():
    return scenarios.config_case("c3")


def _system(case, mode):
    return pcg.MatrixFreeSystem.from_packing(case.packing, case.materials, *case.scalars(), mode=mode)


def test_c2_parity_apply_and_block_jacobi_bitwise(c2):
    s = _system(c2, _lib.MODE_PARITY)
    o = oracle_system(c2.packing, c2.materials, *c2.scalars())
    x = np.random.Generator(np.random.PCG64(21)).uniform(-1, 1, c2.packing.dof_count).astype(np.float32)
    y = np.zeros_like(x)
    pcg.apply_keff(s, x, y).value()
    assert_bitwise(y, o.apply_keff(x), "C2 apply_keff")
    inv = np.zeros(9 * c2.packing.node_count, np.float32)
    pcg.build_block_jacobi_inverse(s, None, inv).value()
    assert_bitwise(inv, o.block_jacobi(), "C2 block inverse")
    s.close()


def test_c2_parity_pcg_25_iterations_bitwise(c2):
    s = _system(c2, _lib.MODE_PARITY)
    o = oracle_system(c2.packing, c2.materials, *c2.scalars())
    rhs = c2.static_rhs()
    x, r = np.zeros_like(rhs), np.zeros_like(rhs)
    t = pcg.solve_pcg(s, rhs, pcg.PcgSettings(25, 1e-12), pcg.PcgVectors(x, r)).value()
    ref = o.solve_pcg(rhs, 25, 1e-12, history=True)
    rt = ref["telemetry"]
    assert (t.iterations, t.converged) == (rt.iterations, bool(rt.converged)) == (25, False)
    assert (t.residual_norm, t.alpha_last, t.beta_last) == (rt.residual_norm, rt.alpha_last, rt.beta_last)
    assert_bitwise(x, ref["x"], "C2 x")
    assert_bitwise(r, ref["r"], "C2 r")
    assert np.array_equal(pcg.residual_history(s), ref["history"])
    s.close()


def test_c2_parity_streamed_folds_match_fold_kernels(c2, monkeypatch):
    """The default single-handle PARITY loop folds alpha and beta in workgroup 0 of the passes that produce the chunk
    partials (tagged granules polled while the other workgroups produce: kernels_parity.hip fold_stream); the
    CWF_PARITY_STREAM=0 loop runs the separate fold kernels. Both must give the same bits over a whole solve to
    convergence (the 25-iteration test above pins the default against the oracle): x, r, history, telemetry."""
    rhs = c2.static_rhs()
    out = []
    for env in ("1", "0"):
        monkeypatch.setenv("CWF_PARITY_STREAM", env)
        s = _system(c2, _lib.MODE_PARITY)
        x, r = np.zeros_like(rhs), np.zeros_like(rhs)
        t = pcg.solve_pcg(s, rhs, pcg.PcgSettings(3000, 1e-6), pcg.PcgVectors(x, r)).value()
        out.append((t, x, r, pcg.residual_history(s)))
        s.close()
    (ta, xa, ra, ha), (tb, xb, rb, hb) = out
    assert ta.converged and (ta.iterations, ta.residual_norm, ta.alpha_last, ta.beta_last) == (
        tb.iterations, tb.residual_norm, tb.alpha_last, tb.beta_last)
    assert_bitwise(xa, xb, "C2 x streamed vs fold kernels")
    assert_bitwise(ra, rb, "C2 r streamed vs fold kernels")
    assert np.array_equal(ha, hb)


@pytest.mark.timeout(900)
def test_c3_parity_pcg_8_iterations_bitwise(c3):
    """C3's 39,551 reduction chunks span ten 4,096-partial blocks of the ordered scalar folds (C2's 4,020 fit in
    one), so this pins the multi-block fold (waves 1-3 staging the next block while thread 0 folds) and the
    fused chunk partials at 10M DOF: x, r and the fp64 history bit-exact after 8 iterations."""
    s = _system(c3, _lib.MODE_PARITY)
    o = oracle_system(c3.packing, c3.materials, *c3.scalars())
    rhs = c3.static_rhs()
    x, r = np.zeros_like(rhs), np.zeros_like(rhs)
    t = pcg.solve_pcg(s, rhs, pcg.PcgSettings(8, 1e-12), pcg.PcgVectors(x, r)).value()
    ref = o.solve_pcg(rhs, 8, 1e-12, history=True)
    rt = ref["telemetry"]
    assert (t.iterations, t.converged) == (rt.iterations, bool(rt.converged)) == (8, False)
    assert (t.residual_norm, t.alpha_last, t.beta_last) == (rt.residual_norm, rt.alpha_last, rt.beta_last)
    assert_bitwise(x, ref["x"], "C3 x")
    assert_bitwise(r, ref["r"], "C3 r")
    assert np.array_equal(pcg.residual_history(s), ref["history"])
    s.close()


def test_c3_parity_apply_bitwise_and_fast_properties(c3):
    P = c3.packing
    sp = _system(c3, _lib.MODE_PARITY)
    sf = _system(c3, _lib.MODE_FAST)
    o = oracle_system(P, c3.materials, *c3.scalars())
    rng = np.random.Generator(np.random.PCG64(31))
    x = rng.uniform(-1, 1, P.dof_count).astype(np.float32)
    yp, yf = np.zeros_like(x), np.zeros_like(x)
    pcg.apply_keff(sp, x, yp).value()
    assert_bitwise(yp, o.apply_keff(x), "C3 apply_keff")
    pcg.apply_keff(sf, x, yf).value()
    # FAST (fp32 element math, FMA) vs the bit-exact path, relative to the operator scale
    assert np.max(np.abs(yf.astype(np.float64) - yp)) <= 2e-5 * np.max(np.abs(yp))
    # symmetry of the constrained operator: a, b zero on Dirichlet dofs
    free = (np.repeat(P.bc_mask, 3) & np.tile(np.array([1, 2, 4], np.uint32), P.node_count)) == 0
    a = np.where(free, rng.standard_normal(P.dof_count), 0.0).astype(np.float32)
    b = np.where(free, rng.standard_normal(P.dof_count), 0.0).astype(np.float32)
    Ka, Kb = np.zeros_like(a), np.zeros_like(b)
    pcg.apply_keff(sf, a, Ka).value()
    pcg.apply_keff(sf, b, Kb).value()
    ab, ba = float(b.astype(np.float64) @ Ka), float(a.astype(np.float64) @ Kb)
    assert abs(ab - ba) <= 1e-5 * abs(float(a.astype(np.float64) @ Ka))
    sp.close()
    sf.close()
    # rigid translation: stiffness-only FAST operator, interior nodes (away from the fixed face) carry ~0
    sk = pcg.MatrixFreeSystem.from_packing(P, c3.materials, 1.0, 0.0, mode=_lib.MODE_FAST)
    t = np.tile(np.array([1e-3, -2e-3, 5e-4], np.float32), P.node_count)
    y = np.zeros_like(t)
    pcg.apply_keff(sk, t, y).value()
    xs = c3.mesh.coords[:, 0]
    far = (xs > xs.min() + 0.25) & (xs < xs.max() - 1e-9)
    yr = y.reshape(-1, 3)
    assert np.abs(yr[far]).max() <= 1e-6 * 30.0e9 * 0.1 * 2e-3
    sk.close()


def _first_step(case, mode):
    P = case.packing
    st = Stepper(P, case.materials, case.rayleigh, case.cfg.solver, case.cfg.time, mode=mode)
    tel = st.step(0.0).value()
    assert tel.pcg.converged
    out = (tel.pcg, st.get_state(Stepper.SOLUTION).copy(), st.get_state(Stepper.DISPLACEMENT).copy(),
           _kernel(st.system))
    st.close()
    st.system.close()
    return out


@pytest.mark.timeout(600)
def test_c3_fast_newmark_step_matches_parity(c3):
    tp, xp, up, _ = _first_step(c3, _lib.MODE_PARITY)
    tf, xf, uf, kf = _first_step(c3, _lib.MODE_FAST)
    assert kf.startswith("k_keff_lattice"), kf  # C3's grid exceeds one round: the two-kernel iteration
    assert abs(tf.iterations - tp.iterations) <= 0.15 * tp.iterations
    check_step_against_parity(xf, xp, uf, up, "C3 step 1")


# ------------------------------------------------------------------------------------------------ C2 FAST (the bench)
# the benchmarked path (the default: the resident one-launch solve, one 512-thread workgroup per 14 x 10 x 10 box) and
# the launch-per-iteration fused schedule it replaced (CWF_FUSED=1: its one-round grid of 436 workgroups)
C2_SCHEDULES = {"resident": (None, "k_pcg_resident<true, LatKuhn, 3, 2, false>"),
                "fused": ("1", "k_pcg_lattice<true, LatKuhn, true, true, false, false>")}


@pytest.mark.parametrize("schedule", sorted(C2_SCHEDULES))
def test_c2_fast_static_solve_matches_parity(c2, schedule, monkeypatch):
    env, want = C2_SCHEDULES[schedule]
    if env is None:
        monkeypatch.delenv("CWF_FUSED", raising=False)
    else:
        monkeypatch.setenv("CWF_FUSED", env)
    sf = _system(c2, _lib.MODE_FAST)
    k = _kernel(sf)
    assert k == want, k
    sp = _system(c2, _lib.MODE_PARITY)
    rhs = c2.static_rhs()
    out = {}
    for name, s in (("fast", sf), ("parity", sp)):
        x, r = np.zeros_like(rhs), np.zeros_like(rhs)
        t = pcg.solve_pcg(s, rhs, pcg.PcgSettings(4000, 1e-6), pcg.PcgVectors(x, r)).value()
        assert t.converged, name
        out[name] = (t, x, r)
    (tf, xf, rf), (tp, xp, _) = out["fast"], out["parity"]
    rel = float(np.linalg.norm(xf.astype(np.float64) - xp) / np.linalg.norm(xp.astype(np.float64)))
    print(f"C2 static tol 1e-6 ({schedule}): FAST {tf.iterations} it, PARITY {tp.iterations} it, "
          f"|x_f - x_p|/|x_p| = {rel:.3e}")
    assert rel <= 1e-4
    assert abs(tf.iterations - tp.iterations) <= max(3, tp.iterations // 20), (tf.iterations, tp.iterations)
    # the r output is the solve's own residual (fp32 recurrence) and meets the tolerance
    assert tf.residual_norm <= 1e-6 * np.linalg.norm(rhs.astype(np.float64)) * 1.0001
    assert abs(np.linalg.norm(rf.astype(np.float64)) - tf.residual_norm) <= 1e-3 * tf.residual_norm
    sf.close()
    sp.close()


@pytest.mark.parametrize("schedule", sorted(C2_SCHEDULES))
def test_c2_fast_newmark_steps_follow_the_parity_stepper(c2, schedule, monkeypatch):
    env, want = C2_SCHEDULES[schedule]
    if env is None:
        monkeypatch.delenv("CWF_FUSED", raising=False)
    else:
        monkeypatch.setenv("CWF_FUSED", env)
    P = c2.packing
    sts = {m: Stepper(P, c2.materials, c2.rayleigh, c2.cfg.solver, c2.cfg.time, mode=m)
           for m in (_lib.MODE_PARITY, _lib.MODE_FAST)}
    assert _kernel(sts[_lib.MODE_FAST].system) == want, _kernel(sts[_lib.MODE_FAST].system)
    for k in range(2):
        tp = sts[_lib.MODE_PARITY].step(0.01 * k).value().pcg
        tf = sts[_lib.MODE_FAST].step(0.01 * k).value().pcg
        assert tp.converged and tf.converged
        print(f"C2 step {k + 1}: PARITY {tp.iterations} it, FAST {tf.iterations} it")
        assert abs(tf.iterations - tp.iterations) <= 3, (k, tf.iterations, tp.iterations)
        xs = {m: st.get_state(Stepper.SOLUTION).copy() for m, st in sts.items()}
        us = {m: st.get_state(Stepper.DISPLACEMENT).copy() for m, st in sts.items()}
        if k == 0:  # from rest both steps solve the same RHS: compare the increments too
            check_step_against_parity(xs[_lib.MODE_FAST], xs[_lib.MODE_PARITY],
                                      us[_lib.MODE_FAST], us[_lib.MODE_PARITY], "C2 step 1")
        else:  # the RHS now carries each path's own step-1 state: the states themselves stay within STEP_REL_TOL
            for which, name in ((Stepper.DISPLACEMENT, "u"), (Stepper.VELOCITY, "v")):
                a, b = (sts[m].get_state(which).astype(np.float64) for m in (_lib.MODE_FAST, _lib.MODE_PARITY))
                rel = float(np.linalg.norm(a - b) / np.linalg.norm(b))
                print(f"C2 step 2: |{name}_f - {name}_p|/|{name}_p| = {rel:.3e}")
                assert rel <= STEP_REL_TOL, (name, rel)
    for st in sts.values():
        st.close()
        st.system.close()
