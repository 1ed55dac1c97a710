"""Parity of the HIP path (libcwf_hip.so on cuda:0) with the pinned oracle and the committed
golden fixtures. PARITY mode: bit-exact (integer/fp32 words compared as bits, fp64 telemetry
compared with ==). FAST mode: tolerance stated per test."""
import os

import numpy as np
import pytest

import oracle as O
from cwf import _lib, pack, pcg, physics, scenarios
from cwf.stepper import Stepper
from helpers import assert_bitwise, kuhn16_reference_case, oracle_system

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def gpu_system(case, mode=_lib.MODE_PARITY, sK=None, sM=None):
    s0, m0 = case.scalars()
    return pcg.MatrixFreeSystem.from_packing(case.packing, case.materials, s0 if sK is None else sK,
                                             m0 if sM is None else sM, mode=mode)


CASES = {
    "c1_small": lambda: scenarios.block_case(8, 3, 4, h=0.1, tol=1e-6, max_iterations=600),
    "jitter": lambda: scenarios.block_case(7, 6, 5, h=0.1, jitter=True, tol=1e-6, max_iterations=600),
    "rayleigh": lambda: scenarios.block_case(6, 4, 3, h=0.1, xi=0.05, w=(10.0, 100.0), tol=1e-6,
                                             max_iterations=600),
}


@pytest.fixture(scope="module", params=sorted(CASES))
def case(request):
    return CASES[request.param]()


def test_device_fp64_div_sqrt_correctly_rounded(case):
    # the PCG scalars (alpha = rho/denom, |r| = sqrt) must round like the host: check via a solve
    s = gpu_system(case)
    o = oracle_system(case.packing, case.materials, *case.scalars())
    rhs = case.static_rhs()
    x = np.zeros_like(rhs)
    t = pcg.solve_pcg(s, rhs, pcg.PcgSettings(5, 1e-12), pcg.PcgVectors(x, np.zeros_like(rhs))).value()
    ref = o.solve_pcg(rhs, 5, 1e-12)["telemetry"]
    assert (t.alpha_last, t.beta_last, t.residual_norm) == (ref.alpha_last, ref.beta_last, ref.residual_norm)


def test_apply_keff_bitwise(case):
    s = gpu_system(case)
    o = oracle_system(case.packing, case.materials, *case.scalars())
    rng = np.random.Generator(np.random.PCG64(3))
    x = rng.uniform(-1, 1, case.packing.dof_count).astype(np.float32)
    y = np.zeros_like(x)
    assert pcg.apply_keff(s, x, y).has_value()
    assert_bitwise(y, o.apply_keff(x), "apply_keff")


def test_apply_keff_input_size_mismatch_error(case):
    s = gpu_system(case)
    r = pcg.apply_keff(s, np.zeros(5, np.float32), np.zeros(5, np.float32))
    assert not r.has_value() and r.error().message == "input/output span size mismatch"


def test_block_jacobi_bitwise(case):
    s = gpu_system(case)
    o = oracle_system(case.packing, case.materials, *case.scalars())
    inv = np.zeros(case.packing.node_count * 9, np.float32)
    assert pcg.build_block_jacobi_inverse(s, None, inv).has_value()
    assert_bitwise(inv, o.block_jacobi(), "block_jacobi")


def test_dot_and_partials_bitwise(case):
    s = gpu_system(case)
    o = oracle_system(case.packing, case.materials, *case.scalars())
    rng = np.random.Generator(np.random.PCG64(5))
    a = rng.standard_normal(case.packing.dof_count).astype(np.float32)
    b = rng.standard_normal(case.packing.dof_count).astype(np.float32)
    parts = np.zeros(case.packing.reduction_partials, np.float64)
    r = pcg.dot(s, a, b, parts)
    ref, ref_parts = o.dot(a, b)
    assert r.value() == ref
    assert_bitwise(parts, ref_parts, "partials")


def test_solve_pcg_bitwise_with_history(case):
    s = gpu_system(case)
    o = oracle_system(case.packing, case.materials, *case.scalars())
    rhs = case.static_rhs()
    x, r = np.zeros_like(rhs), np.zeros_like(rhs)
    t = pcg.solve_pcg(s, rhs, pcg.PcgSettings(600, 1e-6), pcg.PcgVectors(x, r)).value()
    ref = o.solve_pcg(rhs, 600, 1e-6, history=True)
    rt = ref["telemetry"]
    assert (t.iterations, t.converged) == (rt.iterations, bool(rt.converged))
    assert (t.residual_norm, t.rhs_norm, t.alpha_last, t.beta_last) == (rt.residual_norm, rt.rhs_norm,
                                                                          rt.alpha_last, rt.beta_last)
    assert_bitwise(x, ref["x"], "x")
    assert_bitwise(r, ref["r"], "r")
    h = pcg.residual_history(s)
    assert np.array_equal(h, ref["history"])  # fp64 residual norms bit-comparable


def test_solve_pcg_bitwise_with_reduction_block_100():
    """A reduction chunk other than 256 DOFs (pack_cpu_elements' reduction_block_size): the fused K_eff / update
    chunk partials give way to the separate dot pass, and the solve stays bit-exact."""
    import dataclasses
    case = CASES["jitter"]()
    D = case.packing.dof_count
    P = dataclasses.replace(case.packing, reduction_block=100, reduction_partials=(D + 99) // 100)
    s0, m0 = case.scalars()
    s = pcg.MatrixFreeSystem.from_packing(P, case.materials, s0, m0, mode=_lib.MODE_PARITY)
    o = oracle_system(P, case.materials, s0, m0, reduction_block=100)
    rhs = case.static_rhs()
    x, r = np.zeros_like(rhs), np.zeros_like(rhs)
    t = pcg.solve_pcg(s, rhs, pcg.PcgSettings(600, 1e-6), pcg.PcgVectors(x, r)).value()
    ref = o.solve_pcg(rhs, 600, 1e-6, history=True)
    assert (t.iterations, t.residual_norm, t.alpha_last) == (ref["telemetry"].iterations,
                                                             ref["telemetry"].residual_norm, ref["telemetry"].alpha_last)
    assert_bitwise(x, ref["x"], "x rb100")
    assert np.array_equal(pcg.residual_history(s), ref["history"])


def test_solve_pcg_warm_start_bitwise(case):
    s = gpu_system(case)
    o = oracle_system(case.packing, case.materials, *case.scalars())
    rhs = case.static_rhs()
    x0 = (np.arange(rhs.size) % 7 * 1e-7).astype(np.float32)
    x = x0.copy()
    t = pcg.solve_pcg(s, rhs, pcg.PcgSettings(50, 1e-5, True), pcg.PcgVectors(x, np.zeros_like(rhs))).value()
    ref = o.solve_pcg(rhs, 50, 1e-5, warm_start=True, x=x0)
    assert t.iterations == ref["telemetry"].iterations
    assert_bitwise(x, ref["x"], "x warm")


def test_stepper_three_steps_bitwise(case):
    P = case.packing
    st = Stepper(P, case.materials, case.rayleigh, case.cfg.solver, case.cfg.time)
    sK, sM = case.scalars()
    o = oracle_system(P, case.materials, sK, sM)
    r = case.rayleigh
    ost = O.Stepper(o, P.external_force, P.bc_value, (r.alpha, r.beta), case.cfg.solver.runtime_tolerance,
                    case.cfg.solver.pause_tolerance, case.cfg.solver.max_iterations, case.cfg.time.initial_dt)
    for k in range(3):
        t = st.step(k * 0.01).value()
        rt = ost.step(k * 0.01)
        assert t.pcg.iterations == rt.pcg.iterations and t.pcg.residual_norm == rt.pcg.residual_norm
    for which, ref in ((Stepper.DISPLACEMENT, ost.u), (Stepper.VELOCITY, ost.v), (Stepper.ACCELERATION, ost.a)):
        assert_bitwise(st.get_state(which), ref, f"state {which}")
    assert st.current_time() == ost.current_time and st.time_step() == ost.time_step


@pytest.mark.parametrize("name", ["single_tet", "kuhn4x3x2", "jitter6"])
def test_golden_fixtures_bitwise(name):
    g = np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False)
    mesh = pack.Mesh(g["coords"], g["tets"], None, {"SOLID": 1}, {}, [])
    sK, sM, ra, rb, dt, tol, ptol, maxit = g["scalars"]
    pre = pack.preprocess(mesh, physics.Config(materials=[physics.Material("steel", 30e9, 0.2, 2500.0)],
                                               assignments=[physics.Assignment("SOLID", "steel")]))
    mats = [physics.make_properties(physics.Material("steel", 30e9, 0.2, 2500.0))]
    N = mesh.node_count
    s = pcg.MatrixFreeSystem(pre["conn8"], pre["grads"], pre["volume"], pre["material_index"], mats, pre["mass32"],
                             g["bc_mask"], N, mesh.element_count, 3 * N, sK, sM)
    y = np.zeros(3 * N, np.float32)
    assert pcg.apply_keff(s, g["keff_in"], y).has_value()
    assert_bitwise(y, g["keff_out"], "keff")
    inv = np.zeros(9 * N, np.float32)
    pcg.build_block_jacobi_inverse(s, None, inv).value()
    assert_bitwise(inv, g["bj_inv"], "bj")
    x, r = np.zeros(3 * N, np.float32), np.zeros(3 * N, np.float32)
    t = pcg.solve_pcg(s, g["pcg_rhs"], pcg.PcgSettings(400, 1e-6),
                      pcg.PcgVectors(x, r)).value()
    assert t.iterations == int(g["pcg_tel"][0])
    assert t.residual_norm == g["pcg_tel"][1]
    assert_bitwise(x, g["pcg_x"], "pcg x")
    assert np.array_equal(pcg.residual_history(s), g["pcg_hist"])


def test_kuhn16_reference_solve_on_gpu():
    """The survey's recorded reference run, reproduced on the GPU: 162 iterations,
    |r| = 0.14640172515227148, FNV-1a(x) = f10c27935f2e7a58."""
    case, rhs = kuhn16_reference_case()
    s = gpu_system(case)
    x = np.zeros_like(rhs)
    t = pcg.solve_pcg(s, rhs, pcg.PcgSettings(500, 3e-4), pcg.PcgVectors(x, np.zeros_like(rhs))).value()
    assert t.iterations == 162
    assert t.residual_norm == 0.14640172515227148
    assert O.fnv1a64_words(x) == "f10c27935f2e7a58"


def test_stagnation_error_path_matches_reference_text():
    case = scenarios.block_case(8, 8, 8, h=1.0, gravity=(0.0, 0.0, 0.0), point_group="CORNER")
    ez = case.packing.external_force.reshape(-1, 3)[:, 2]
    i = np.arange(case.packing.dof_count)
    rhs = (ez[i // 3] * (i % 3 == 2).astype(np.float32)).astype(np.float32)
    s = gpu_system(case)
    x = np.zeros_like(rhs)
    r = pcg.solve_pcg(s, rhs, pcg.PcgSettings(500, 1e-8), pcg.PcgVectors(x, np.zeros_like(rhs)))
    assert not r.has_value()
    assert r.error().message == "CG denominator approached zero"
    assert r.error().context == ["iteration=133"]


def test_max_iterations_zero_error():
    case = CASES["c1_small"]()
    s = gpu_system(case)
    rhs = case.static_rhs()
    r = pcg.solve_pcg(s, rhs, pcg.PcgSettings(0, 1e-6), pcg.PcgVectors(np.zeros_like(rhs), None))
    assert r.error().message == "max_iterations must be >= 1" and r.error().context == ["max_iterations=0"]


def test_pause_mode_and_adaptive_dt():
    # tests/newmark_stepper_test.cpp:241-269
    case = scenarios.block_case(3, 2, 2, h=0.1, tol=3e-4, max_iterations=64)
    st = Stepper(case.packing, case.materials, case.rayleigh, case.cfg.solver, case.cfg.time)
    t = st.step(0.0, True).value()
    assert t.paused_mode and abs(t.applied_tolerance - case.cfg.solver.pause_tolerance) < 1e-12
    ts = physics.TimeSettings(0.01, True, 0.0, 0.02)
    from cwf.stepper import AdaptivePolicy

    st2 = Stepper(case.packing, case.materials, case.rayleigh, case.cfg.solver, ts, AdaptivePolicy(1.0, 2.0, 0.5))
    t2 = st2.step(0.0).value()
    assert t2.dt_increased and t2.dt_clamped_max and abs(st2.time_step() - 0.02) < 1e-12


# ---------------------------------------------------------------- fast mode (tolerance) ----
def test_fast_mode_apply_keff_close(case):
    s = gpu_system(case, mode=_lib.MODE_FAST)
    o = oracle_system(case.packing, case.materials, *case.scalars())
    rng = np.random.Generator(np.random.PCG64(3))
    x = rng.uniform(-1, 1, case.packing.dof_count).astype(np.float32)
    y = np.zeros_like(x)
    pcg.apply_keff(s, x, y).value()
    ref = o.apply_keff(x).astype(np.float64)
    # fp32 element math vs fp64: relative to the operator scale (max |row|)
    assert np.max(np.abs(y - ref)) <= 2e-5 * np.max(np.abs(ref))


def test_fast_mode_128_lane_tiles_close(case, monkeypatch):
    """The 128-lane fan-group tiles (CWF_GROUP_NT=128, no longer the default) keep the FAST tolerance."""
    monkeypatch.setenv("CWF_GROUP_NT", "128")
    s = gpu_system(case, mode=_lib.MODE_FAST)
    o = oracle_system(case.packing, case.materials, *case.scalars())
    rng = np.random.Generator(np.random.PCG64(5))
    x = rng.uniform(-1, 1, case.packing.dof_count).astype(np.float32)
    y = np.zeros_like(x)
    pcg.apply_keff(s, x, y).value()
    ref = o.apply_keff(x).astype(np.float64)
    assert np.max(np.abs(y - ref)) <= 2e-5 * np.max(np.abs(ref))


def test_fast_mode_solve_close(case):
    s = gpu_system(case, mode=_lib.MODE_FAST)
    o = oracle_system(case.packing, case.materials, *case.scalars())
    rhs = case.static_rhs()
    x = np.zeros_like(rhs)
    t = pcg.solve_pcg(s, rhs, pcg.PcgSettings(600, 1e-6), pcg.PcgVectors(x, np.zeros_like(rhs))).value()
    ref = o.solve_pcg(rhs, 600, 1e-6)
    assert t.converged
    # tolerance: the solve itself only guarantees |r| <= 1e-6 |rhs|; solutions agree to 1e-4 relative
    assert np.linalg.norm(x - ref["x"]) <= 1e-4 * np.linalg.norm(ref["x"])
    assert abs(t.iterations - ref["telemetry"].iterations) <= max(3, ref["telemetry"].iterations // 10)


def test_fast_block_inverse_reused_only_for_unchanged_scalars(case):
    """A FAST handle keeps its block inverse while (s_K, s_M) are unchanged and rebuilds it when they change
    or when the reference inverse was exported through it: every solve is bitwise the same solve on a fresh
    handle with the same scalars (FAST is deterministic: fixed fold orders, no atomics)."""
    sK, sM = case.scalars()
    rhs = case.static_rhs()

    def solve(s):
        x, r = np.zeros_like(rhs), np.zeros_like(rhs)
        t = pcg.solve_pcg(s, rhs, pcg.PcgSettings(40, 1e-12), pcg.PcgVectors(x, r)).value()
        return x, r, t.residual_norm

    def same(a, b):
        assert_bitwise(a[0], b[0], "x")
        assert_bitwise(a[1], b[1], "r")
        assert a[2] == b[2]

    s = gpu_system(case, mode=_lib.MODE_FAST)
    first = solve(s)
    same(solve(s), first)  # the second solve reuses the inverse
    s.stiffness_scale, s.mass_factor = 1.5 * sK, 0.5 * sM + 1.0
    changed = solve(s)
    same(changed, solve(gpu_system(case, mode=_lib.MODE_FAST, sK=1.5 * sK, sM=0.5 * sM + 1.0)))
    ref_inv = np.zeros(9 * case.packing.node_count, np.float32)
    assert pcg.build_block_jacobi_inverse(s, None, ref_inv).has_value()  # overwrites the handle's copy
    same(solve(s), changed)
    s.stiffness_scale, s.mass_factor = sK, sM
    same(solve(s), first)


def _upper_sym(inv9):
    b = inv9.reshape(-1, 3, 3)
    return np.stack([b[:, 0, 0], b[:, 0, 1], b[:, 0, 2], b[:, 1, 1], b[:, 1, 2], b[:, 2, 2]], 1)


def test_fast_block_inverse_record_matches_host_packing_of_reference_inverse():
    """The device's 16-B records are the host packing (blockinv_pack.hpp) of the reference inverse
    (oracle, symmetrised: upper triangle), word for word; the exported applied operator is their decode."""
    case = scenarios.roller_case(9, 5, 4, tol=1e-6, max_iterations=800)
    P = case.packing
    s = gpu_system(case, mode=_lib.MODE_FAST)
    applied = np.zeros(9 * P.node_count, np.float32)
    packed = np.zeros(4 * P.node_count, np.uint32)
    nfall = pcg.fast_block_inverse(s, applied, packed).value()
    ref = oracle_system(P, case.materials, *case.scalars()).block_jacobi()
    up = _upper_sym(ref)
    want_w = np.zeros_like(packed)
    want_d = np.zeros((P.node_count, 6), np.float32)
    fb = 0
    for n in range(P.node_count):
        ok, w, d = pcg.pack_block_inverse(up[n], int(P.bc_mask[n]))
        want_w[4 * n:4 * n + 4] = w
        want_d[n] = d
        fb += not ok
    assert nfall == fb == 0
    assert_bitwise(packed, want_w, "16-B records")
    assert_bitwise(_upper_sym(applied), want_d, "applied inverse")
    a = applied.reshape(-1, 3, 3)
    assert np.array_equal(a, np.transpose(a, (0, 2, 1)))  # symmetric
    # the reference-semantics export is unchanged in FAST mode
    inv = np.zeros_like(applied)
    pcg.build_block_jacobi_inverse(s, None, inv).value()
    assert_bitwise(inv, ref, "reference inverse (FAST handle)")


@pytest.mark.parametrize("shape", [(9, 5, 4), (16, 6, 6)])
def test_fast_solve_with_partial_masks(shape):
    """Rollers on three faces (most constrained nodes keep free axes) in physical units (E = 30 GPa):
    FAST converges like the oracle. The old single-scale fp16 packing flushed these nodes' free entries
    (~1e-10) to zero and stalled at max_iterations."""
    case = scenarios.roller_case(*shape, tol=1e-6, max_iterations=2000)
    s = gpu_system(case, mode=_lib.MODE_FAST)
    o = oracle_system(case.packing, case.materials, *case.scalars())
    rhs = case.static_rhs()
    x = np.zeros_like(rhs)
    t = pcg.solve_pcg(s, rhs, pcg.PcgSettings(2000, 1e-6), pcg.PcgVectors(x, np.zeros_like(rhs))).value()
    ref = o.solve_pcg(rhs, 2000, 1e-6)
    assert t.converged and ref["telemetry"].converged
    assert abs(t.iterations - ref["telemetry"].iterations) <= max(3, ref["telemetry"].iterations // 10)
    assert np.linalg.norm(x - ref["x"]) <= 1e-4 * np.linalg.norm(ref["x"])


def test_fast_stepper_with_partial_masks():
    case = scenarios.roller_case(12, 4, 4, tol=1e-6, max_iterations=1500)
    P = case.packing
    ref = Stepper(P, case.materials, case.rayleigh, case.cfg.solver, case.cfg.time, mode=_lib.MODE_PARITY)
    fast = Stepper(P, case.materials, case.rayleigh, case.cfg.solver, case.cfg.time, mode=_lib.MODE_FAST)
    for k in range(3):
        tr = ref.step(0.01 * k).value()
        tf = fast.step(0.01 * k).value()
        assert tf.pcg.converged and tr.pcg.converged
        assert abs(tf.pcg.iterations - tr.pcg.iterations) <= max(3, tr.pcg.iterations // 10)
    ur, uf = ref.get_state(Stepper.DISPLACEMENT), fast.get_state(Stepper.DISPLACEMENT)
    assert np.linalg.norm(uf - ur) <= 1e-4 * np.linalg.norm(ur)


_LAZY_X_SCRIPT = r"""
import hashlib, sys, numpy as np
sys.path[:0] = sys.argv[1:3]
from cwf import _lib, pcg, scenarios
case = scenarios.block_case(7, 6, 5, h=0.1, jitter=True, tol=1e-6, max_iterations=600)
s0, m0 = case.scalars()
s = pcg.MatrixFreeSystem.from_packing(case.packing, case.materials, s0, m0, mode=_lib.MODE_FAST)
rhs = case.static_rhs()
out = []
for it in (5, 6, 7, 8, 600):
    x = np.zeros_like(rhs)
    t = pcg.solve_pcg(s, rhs, pcg.PcgSettings(it, 1e-6), pcg.PcgVectors(x, np.zeros_like(rhs))).value()
    out += [hashlib.sha256(x.tobytes()).hexdigest(), str(t.iterations)]
print(" ".join(out))
"""


def test_fast_lazy_x_is_bitwise_the_eager_update():
    """FAST PCG applies x += alpha_j p_j every 4th iteration (k_pcg_update_tiles) and flushes the rest
    after the solve (k_x_flush); the FMA chain in iteration order is bitwise the per-iteration update
    (CWF_XLAG=1). Solves stopping at every iteration count mod 4 (max_iterations 5..8) and a converged one."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    args = [sys.executable, "-c", _LAZY_X_SCRIPT, os.path.join(root, "civiwave-fem_amd"), os.path.join(root, "tests")]
    runs = {}
    for lag in ("4", "1"):
        env = dict(os.environ, CWF_XLAG=lag)
        r = subprocess.run(args, env=env, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        runs[lag] = r.stdout.split()
    assert runs["4"] == runs["1"]


def test_cpp_mirror_single_tet_reference_outputs(tmp_path):
    """tests/cpp/pcg_api_test.cpp: the reference's single-tet fixture through include/cwf_hip.hpp."""
    import subprocess

    from test_host import _build_cpp_test

    exe = _build_cpp_test(tmp_path)
    out = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr


def test_fast_short_solve_after_long_solves_matches_fresh_handle():
    """The first PCG batch is sized from the handle's last two solves when they agree (abi.cpp run_pcg_group);
    a short warm-started solve after two long ones must still stop at its own convergence: x, r, the
    iteration count and the fp64 residual history equal a fresh handle's (which batches from 4), bit for bit,
    including the lazy x flush of an iteration count that is not a multiple of 4."""
    case = CASES["jitter"]()
    rhs = case.static_rhs()
    s = gpu_system(case, mode=_lib.MODE_FAST)
    for _ in range(2):
        x_long = np.zeros_like(rhs)
        t_long = pcg.solve_pcg(s, rhs, pcg.PcgSettings(600, 1e-6), pcg.PcgVectors(x_long, np.zeros_like(rhs))).value()
        assert t_long.converged and t_long.iterations > 60
    rhs2 = (1.01 * rhs).astype(np.float32)
    out = []
    for h in (s, gpu_system(case, mode=_lib.MODE_FAST)):
        x, r = x_long.copy(), np.zeros_like(rhs)
        t = pcg.solve_pcg(h, rhs2, pcg.PcgSettings(600, 1e-3, True), pcg.PcgVectors(x, r)).value()
        out.append((x, r, t, pcg.residual_history(h)))
    (x1, r1, t1, h1), (x2, r2, t2, h2) = out
    assert t1.converged and 0 < t1.iterations < t_long.iterations // 2
    assert (t1.iterations, t1.residual_norm) == (t2.iterations, t2.residual_norm)
    assert_bitwise(x1, x2, "x")
    assert_bitwise(r1, r2, "r")
    assert np.array_equal(h1, h2)
