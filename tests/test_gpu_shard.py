"""Sharded FAST PCG on one GPU (LOCAL communicator: every rank's handle in this process, exchanges
as device copies). The kernels, the per-iteration schedule (p.Ap all-gather, r.r / r.z all-gather,
z halo) and the ghost-row handling are the ones RCCL ranks run; only the transport differs.
Tolerance: the sharded solve must converge to the single-process oracle solution within 1e-4
relative (the solve guarantees |r| <= 1e-6 |rhs|) in the same iteration count +-10%."""
import numpy as np
import oracle as O
import pytest

from cwf import _lib, pcg, scenarios, shard
from helpers import assert_bitwise, oracle_system

pytestmark = pytest.mark.gpu


def _sharded_solve(glob, nranks, rel_tol=1e-6, max_iterations=800, from_slabs=None):
    sK, sM = glob.scalars()
    P = glob.packing
    comm = shard.Comm.local(nranks)
    systems, shards, rhs, xs = [], [], [], []
    for r in range(nranks):
        if from_slabs:
            case, node_global, begin = scenarios.slab_case_shape(from_slabs, nranks, r, tol=rel_tol)
            src = pcg.MatrixFreeSystem.from_packing(case.packing, case.materials, sK, sM, mode=_lib.MODE_FAST)
            sh = shard.build_shard(src, begin, r, node_global)
            rhs.append(sh.local_dofs(case.static_rhs()))
        else:
            src = pcg.MatrixFreeSystem.from_packing(P, glob.materials, sK, sM, mode=_lib.MODE_FAST)
            sh = shard.build_shard(src, shard.slab_ranges(P.node_count, nranks), r)
            rhs.append(sh.local_dofs(glob.static_rhs()))
        s = sh.system(glob.materials, sK, sM)
        comm.attach(s, sh)
        systems.append(s)
        shards.append(sh)
        xs.append(np.zeros(3 * sh.local_nodes, np.float32))
    tel = shard.solve_pcg_group(systems, rhs, pcg.PcgSettings(max_iterations, rel_tol), xs).value()
    x = np.zeros((P.node_count, 3), np.float32)
    for sh, xl in zip(shards, xs):
        x[sh.node_global[: sh.owned_nodes].astype(np.int64)] = xl.reshape(-1, 3)[: sh.owned_nodes]
        # x is halo-consistent on return: ghost rows carry the owners' values
    for sh, xl in zip(shards, xs):
        assert np.array_equal(xl.reshape(-1, 3)[sh.owned_nodes:], x[sh.node_global[sh.owned_nodes:].astype(np.int64)])
    comm.close()
    return tel, x.reshape(-1)


@pytest.mark.parametrize("nranks", [2, 3])
def test_local_sharded_solve_matches_oracle(nranks):
    glob = scenarios.block_case(10, 6, 12, h=0.1, tol=1e-6)
    sK, sM = glob.scalars()
    tel, x = _sharded_solve(glob, nranks)
    ref = oracle_system(glob.packing, glob.materials, sK, sM).solve_pcg(glob.static_rhs(), 800, 1e-6)
    assert tel.converged
    assert np.linalg.norm(x - ref["x"]) <= 1e-4 * np.linalg.norm(ref["x"])
    n_ref = ref["telemetry"].iterations
    assert abs(tel.iterations - n_ref) <= max(3, n_ref // 10)


def test_local_sharded_from_slab_submeshes():
    """The bench's decomposition: every rank builds only its slab sub-mesh (+ ghost layer)."""
    nranks = 3
    shape = (8, 5, 4)
    glob = scenarios.block_case(shape[0], shape[1], shape[2] * nranks, h=0.1, tol=1e-6)
    sK, sM = glob.scalars()
    tel, x = _sharded_solve(glob, nranks, from_slabs=shape)
    ref = oracle_system(glob.packing, glob.materials, sK, sM).solve_pcg(glob.static_rhs(), 800, 1e-6)
    assert tel.converged
    assert np.linalg.norm(x - ref["x"]) <= 1e-4 * np.linalg.norm(ref["x"])


def test_local_group_requires_group_call():
    glob = scenarios.block_case(4, 3, 4, h=0.1)
    sK, sM = glob.scalars()
    P = glob.packing
    comm = shard.Comm.local(2)
    src = pcg.MatrixFreeSystem.from_packing(P, glob.materials, sK, sM, mode=_lib.MODE_FAST)
    sh = shard.build_shard(src, shard.slab_ranges(P.node_count, 2), 0)
    s = sh.system(glob.materials, sK, sM)
    comm.attach(s, sh)
    rhs = sh.local_dofs(glob.static_rhs())
    e = pcg.solve_pcg(s, rhs, pcg.PcgSettings(10, 1e-6), pcg.PcgVectors(np.zeros_like(rhs), None))
    assert not e.has_value() and "solve_pcg_group" in e.error().message
    comm.close()


def test_rccl_single_rank_sharded_schedule():
    """The RCCL transport on one GPU: dlopen + unique id + a 1-rank communicator, a handle attached to it
    (the sharded schedule: per-rank scalar folds, all-gathers, the halo group call) solving the whole
    mesh. Multi-rank RCCL needs one GPU per rank and runs in the driver's 8-GPU bench."""
    glob = scenarios.block_case(8, 5, 6, h=0.1, tol=1e-6)
    sK, sM = glob.scalars()
    P = glob.packing
    comm = shard.Comm.rccl(1, 0, shard.Comm.unique_id(), 0)
    src = pcg.MatrixFreeSystem.from_packing(P, glob.materials, sK, sM, mode=_lib.MODE_FAST)
    sh = shard.build_shard(src, shard.slab_ranges(P.node_count, 1), 0)
    s = sh.system(glob.materials, sK, sM)
    comm.attach(s, sh)
    x = [np.zeros(3 * sh.local_nodes, np.float32)]
    tel = shard.solve_pcg_group([s], [sh.local_dofs(glob.static_rhs())], pcg.PcgSettings(800, 1e-6), x).value()
    ref = oracle_system(P, glob.materials, sK, sM).solve_pcg(glob.static_rhs(), 800, 1e-6)
    xg = np.zeros((P.node_count, 3), np.float32)
    xg[sh.node_global[: sh.owned_nodes].astype(np.int64)] = x[0].reshape(-1, 3)[: sh.owned_nodes]
    assert tel.converged
    assert np.linalg.norm(xg.reshape(-1) - ref["x"]) <= 1e-4 * np.linalg.norm(ref["x"])
    s.close()
    comm.close()


def _parity_sharded(glob, nranks, ranges=None, from_slabs=None, rel_tol=1e-6, max_iterations=800, warm=None):
    """LOCAL PARITY solve over `nranks` shards -> (telemetry or error, global x, global r, members' histories)."""
    sK, sM = glob.scalars()
    P = glob.packing
    comm = shard.Comm.local(nranks)
    systems, shards, rhs, xs, rs = [], [], [], [], []
    for k in range(nranks):
        if from_slabs:
            case, node_global, begin = scenarios.slab_case_shape(from_slabs, nranks, k, tol=rel_tol)
            src = pcg.MatrixFreeSystem.from_packing(case.packing, case.materials, sK, sM, mode=_lib.MODE_PARITY)
            sh = shard.build_shard(src, begin, k, node_global)
            rhs.append(sh.local_dofs(case.static_rhs()))
        else:
            src = pcg.MatrixFreeSystem.from_packing(P, glob.materials, sK, sM, mode=_lib.MODE_PARITY)
            sh = shard.build_shard(src, ranges, k)
            rhs.append(sh.local_dofs(glob.static_rhs()))
        s = sh.system(glob.materials, sK, sM, mode=_lib.MODE_PARITY)
        comm.attach(s, sh)
        systems.append(s)
        shards.append(sh)
        if warm is None:
            xs.append(np.zeros(3 * sh.local_nodes, np.float32))
        else:  # by global node id (a slab sub-mesh numbers its nodes locally)
            xs.append(np.ascontiguousarray(warm.reshape(-1, 3)[sh.node_global.astype(np.int64)].reshape(-1)))
        rs.append(np.zeros(3 * sh.local_nodes, np.float32))
    res = shard.solve_pcg_group(systems, rhs, pcg.PcgSettings(max_iterations, rel_tol, warm is not None), xs,
                                residuals=rs)
    x = np.zeros((P.node_count, 3), np.float32)
    r = np.zeros((P.node_count, 3), np.float32)
    for sh, xl, rl in zip(shards, xs, rs):
        g = sh.node_global[: sh.owned_nodes].astype(np.int64)
        x[g] = xl.reshape(-1, 3)[: sh.owned_nodes]
        r[g] = rl.reshape(-1, 3)[: sh.owned_nodes]
    hists = [pcg.residual_history(s) for s in systems] if res.has_value() else []
    comm.close()
    return res, x.reshape(-1), r.reshape(-1), hists


@pytest.mark.parametrize("nranks", [2, 3])
def test_local_sharded_parity_solve_bitwise_equals_single_handle(nranks):
    """SURVEY.md 8e parity gate: owned ranges aligned to 256 nodes, every rank's 256-DOF chunk partials
    all-gathered and folded in global chunk order -> x, r, the telemetry and the fp64 residual history of
    the sharded PARITY solve equal the single-handle PARITY solve (and the oracle) bit for bit."""
    glob = scenarios.block_case(10, 6, 12, h=0.1, tol=1e-6)  # 1,001 nodes
    sK, sM = glob.scalars()
    P = glob.packing
    ranges = shard.slab_ranges(P.node_count, nranks, align=256)
    res, x, r, hists = _parity_sharded(glob, nranks, ranges=ranges)
    tel = res.value()
    single = pcg.MatrixFreeSystem.from_packing(P, glob.materials, sK, sM, mode=_lib.MODE_PARITY)
    rhs = glob.static_rhs()
    x1, r1 = np.zeros_like(rhs), np.zeros_like(rhs)
    t1 = pcg.solve_pcg(single, rhs, pcg.PcgSettings(800, 1e-6), pcg.PcgVectors(x1, r1)).value()
    h1 = pcg.residual_history(single)
    assert tel.converged and (tel.iterations, tel.residual_norm, tel.rhs_norm, tel.alpha_last, tel.beta_last) == (
        t1.iterations, t1.residual_norm, t1.rhs_norm, t1.alpha_last, t1.beta_last)
    assert_bitwise(x, x1, "sharded PARITY x")
    assert_bitwise(r, r1, "sharded PARITY r")
    for h in hists:
        assert np.array_equal(h, h1)
    ref = oracle_system(P, glob.materials, sK, sM).solve_pcg(rhs, 800, 1e-6, history=True)
    assert_bitwise(x, ref["x"], "sharded PARITY x vs oracle")
    assert np.array_equal(hists[0], ref["history"])


def test_local_sharded_parity_from_slab_submeshes_warm_start():
    """The bench's decomposition in PARITY mode: 15 x 15 cross-sections (256 nodes per plane, so every slab
    boundary is chunk-aligned), each rank builds only its slab sub-mesh; a warm-started solve is bitwise the
    single-handle one."""
    nranks, shape = 3, (15, 15, 2)
    glob = scenarios.block_case(15, 15, 2 * nranks, h=0.1, tol=1e-6)
    sK, sM = glob.scalars()
    P = glob.packing
    warm = (np.arange(P.dof_count) % 5 * 1e-7).astype(np.float32)
    res, x, r, hists = _parity_sharded(glob, nranks, from_slabs=shape, warm=warm)
    tel = res.value()
    ref = oracle_system(P, glob.materials, sK, sM).solve_pcg(glob.static_rhs(), 800, 1e-6, warm_start=True, x=warm,
                                                             history=True)
    assert tel.iterations == ref["telemetry"].iterations and tel.residual_norm == ref["telemetry"].residual_norm
    assert_bitwise(x, ref["x"], "slab PARITY x")
    assert_bitwise(r, ref["r"], "slab PARITY r")
    assert np.array_equal(hists[1], ref["history"])


def test_local_sharded_parity_rejects_unaligned_ranges():
    glob = scenarios.block_case(10, 6, 12, h=0.1, tol=1e-6)
    res, *_ = _parity_sharded(glob, 2, ranges=shard.slab_ranges(glob.packing.node_count, 2))  # cut at 500 nodes
    assert not res.has_value()
    assert res.error().message.startswith("sharded PARITY needs contiguous owned node ranges")
    assert res.error().context == ["rank=0", "first_node=0", "owned_nodes=500"]


@pytest.mark.parametrize("nranks", [2, 3])
def test_local_sharded_hex8_solve(nranks):
    """Native hex8 shards (north_star: 'the 8-GPU target on a hex mesh'): every rank builds its hex slab
    sub-mesh; the sharded FAST solve converges to the fp64 hex8 solution (oracle hex8_solve64) within 1e-4
    relative, in the single handle's iteration count +-10%."""
    shape = (8, 5, 3)
    glob = scenarios.block_case(shape[0], shape[1], shape[2] * nranks, h=0.1, element="hex8", tol=1e-6)
    sK, sM = glob.scalars()
    P = glob.packing
    comm = shard.Comm.local(nranks)
    systems, shards, rhs, xs = [], [], [], []
    for k in range(nranks):
        case, node_global, begin = scenarios.slab_case_shape(shape, nranks, k, tol=1e-6, element="hex8")
        src = pcg.MatrixFreeSystem.from_packing(case.packing, case.materials, sK, sM, mode=_lib.MODE_FAST)
        sh = shard.build_shard(src, begin, k, node_global)
        s = sh.system(glob.materials, sK, sM)
        comm.attach(s, sh)
        systems.append(s)
        shards.append(sh)
        rhs.append(sh.local_dofs(case.static_rhs()))
        xs.append(np.zeros(3 * sh.local_nodes, np.float32))
    tel = shard.solve_pcg_group(systems, rhs, pcg.PcgSettings(3000, 1e-6), xs).value()
    x = np.zeros((P.node_count, 3), np.float32)
    for sh, xl in zip(shards, xs):
        x[sh.node_global[: sh.owned_nodes].astype(np.int64)] = xl.reshape(-1, 3)[: sh.owned_nodes]
    comm.close()
    D = np.concatenate([np.asarray(m.stiffness, np.float64).reshape(-1) for m in glob.materials])
    ref = O.hex8_solve64(glob.mesh.coords, glob.mesh.tets, P.material_index, D, sK, sM, P.lumped_mass, P.bc_mask,
                         glob.static_rhs())
    single = pcg.MatrixFreeSystem.from_packing(P, glob.materials, sK, sM, mode=_lib.MODE_FAST)
    rhs1 = glob.static_rhs()
    x1 = np.zeros_like(rhs1)
    t1 = pcg.solve_pcg(single, rhs1, pcg.PcgSettings(3000, 1e-6), pcg.PcgVectors(x1, np.zeros_like(rhs1))).value()
    assert tel.converged and t1.converged
    assert np.linalg.norm(x.reshape(-1) - ref) <= 1e-4 * np.linalg.norm(ref)
    assert abs(tel.iterations - t1.iterations) <= max(3, t1.iterations // 10)


def test_local_rcb_sharded_c4_like_solve_matches_oracle():
    """C4's decomposition on one GPU: a jittered + randomly permuted mesh (C4's generator at 14 x 12 x 10),
    nodes split over 4 ranks by RCB and renumbered part after part (scenarios.rcb_case's partition); the
    sharded FAST solve converges to the one-process oracle solution within 1e-4 relative in the oracle's
    iteration count +-10%, and each rank's halo stays a small fraction of its owned nodes."""
    nranks = 4
    glob = scenarios.block_case(14, 12, 10, h=0.1, jitter=True, tol=1e-6)
    sK, sM = glob.scalars()
    P = glob.packing
    gid, begin = shard.rcb_node_ranges(glob.mesh.coords, nranks)
    comm = shard.Comm.local(nranks)
    src = pcg.MatrixFreeSystem.from_packing(P, glob.materials, sK, sM, mode=_lib.MODE_FAST)
    systems, shards, rhs, xs = [], [], [], []
    for k in range(nranks):
        sh = shard.build_shard(src, begin, k, gid)
        s = sh.system(glob.materials, sK, sM)
        comm.attach(s, sh)
        systems.append(s)
        shards.append(sh)
        rhs.append(sh.local_dofs(glob.static_rhs()))
        xs.append(np.zeros(3 * sh.local_nodes, np.float32))
        halo_bytes = 12 * (sh.local_nodes - sh.owned_nodes)
        assert halo_bytes < 12 * sh.owned_nodes, (k, halo_bytes)
    tel = shard.solve_pcg_group(systems, rhs, pcg.PcgSettings(1500, 1e-6), xs).value()
    x = np.zeros((P.node_count, 3), np.float32)
    for sh, xl in zip(shards, xs):
        x[sh.node_source[: sh.owned_nodes].astype(np.int64)] = xl.reshape(-1, 3)[: sh.owned_nodes]
    comm.close()
    ref = oracle_system(P, glob.materials, sK, sM).solve_pcg(glob.static_rhs(), 1500, 1e-6)
    assert tel.converged
    assert np.linalg.norm(x.reshape(-1) - ref["x"]) <= 1e-4 * np.linalg.norm(ref["x"])
    n_ref = ref["telemetry"].iterations
    assert abs(tel.iterations - n_ref) <= max(3, n_ref // 10)
