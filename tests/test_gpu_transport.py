"""The multi-rank RCCL code path of comm.cpp, run as 2 and 3 processes on one GPU.

RCCL refuses two ranks on one device ("Duplicate GPU detected"), so these tests put the host-staged test
transport (tests/transport/host_nccl.cpp: the nine NCCL entry points comm.cpp resolves, over Unix sockets
through host memory) under libcwf_hip.so with CWF_RCCL_LIB. Everything above the transport is the product
path the driver's 8-GPU bench runs: one process per rank, cwf_hip_comm_create_rccl, attach, the collective
cwf_hip_solve_pcg with its grouped all-gathers and halo send/recv.

- PARITY: x, r, the telemetry and every rank's fp64 residual history equal the single-handle PARITY solve
  bit for bit (the SURVEY 8e gate across processes).
- FAST: bitwise equal to the same decomposition solved in one process over the LOCAL communicator (same
  kernels, same rank-order folds; only the transport differs), and within 1e-4 of the oracle solution.
- PARITY Newmark steps (the bench's Stepper over a shard, Rayleigh beta_R != 0): u, v, a and every step's
  telemetry equal the one-handle Stepper bit for bit.
"""
import multiprocessing as mp
import os
import subprocess
import tempfile

import numpy as np
import pytest

from cwf import _lib, pcg, scenarios, shard
from helpers import assert_bitwise, oracle_system

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
TRANSPORT = os.path.join(HERE, "transport", "libcwf_host_nccl.so")


@pytest.fixture(scope="module")
def transport():
    subprocess.run(["make", "-s", "-C", os.path.dirname(TRANSPORT)], check=True)
    return TRANSPORT


def _uid() -> bytes:
    """The transport's unique id is its rendezvous directory (made here, so this process's own RCCL state,
    real RCCL loaded by earlier tests, is not involved)."""
    d = tempfile.mkdtemp(prefix="cwf_host_nccl.").encode()
    assert len(d) < _lib.COMM_ID_BYTES
    return d + b"\0" * (_lib.COMM_ID_BYTES - len(d))


def _run(spec, nranks, transport, target="run_rank"):
    import transport_worker

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    uid = _uid()
    old = os.environ.get("CWF_RCCL_LIB")
    os.environ["CWF_RCCL_LIB"] = transport  # inherited by the spawned ranks only when set before start()
    try:
        fn = getattr(transport_worker, target)
        procs = [ctx.Process(target=fn, args=(k, nranks, uid, spec, q)) for k in range(nranks)]
        for p in procs:
            p.start()
        out = {}
        for _ in range(nranks):
            rank, status, payload = q.get(timeout=240)
            assert status == "ok", f"rank {rank}: {payload}"
            out[rank] = payload
        for p in procs:
            p.join(timeout=60)
            assert p.exitcode == 0
    finally:
        if old is None:
            os.environ.pop("CWF_RCCL_LIB", None)
        else:
            os.environ["CWF_RCCL_LIB"] = old
    return out


def _assemble(out, P):
    x = np.zeros((P.node_count, 3), np.float32)
    r = np.zeros((P.node_count, 3), np.float32)
    for d in out.values():
        x[d["nodes"]] = d["x"].reshape(-1, 3)
        r[d["nodes"]] = d["r"].reshape(-1, 3)
    return x.reshape(-1), r.reshape(-1)


@pytest.mark.parametrize("nranks", [2, 3])
def test_multiprocess_parity_solve_bitwise_equals_single_handle(transport, nranks):
    spec = dict(mode="parity", block=(10, 6, 12), tol=1e-6, max_iterations=800)
    glob = scenarios.block_case(10, 6, 12, h=0.1, tol=1e-6, max_iterations=800)  # 1,001 nodes
    P = glob.packing
    sK, sM = glob.scalars()
    spec["ranges"] = [int(v) for v in shard.slab_ranges(P.node_count, nranks, align=256)]
    out = _run(spec, nranks, transport)
    x, r = _assemble(out, P)
    single = pcg.MatrixFreeSystem.from_packing(P, glob.materials, sK, sM, mode=_lib.MODE_PARITY)
    rhs = glob.static_rhs()
    x1, r1 = np.zeros_like(rhs), np.zeros_like(rhs)
    t1 = pcg.solve_pcg(single, rhs, pcg.PcgSettings(800, 1e-6), pcg.PcgVectors(x1, r1)).value()
    h1 = pcg.residual_history(single)
    for d in out.values():
        assert d["telemetry"] == (t1.iterations, t1.converged, t1.residual_norm, t1.rhs_norm, t1.alpha_last,
                                  t1.beta_last)
        assert np.array_equal(d["history"], h1)
    assert t1.converged
    assert_bitwise(x, x1, "multi-process PARITY x")
    assert_bitwise(r, r1, "multi-process PARITY r")
    single.close()


@pytest.mark.parametrize("nranks", [2, 3])
def test_multiprocess_fast_solve_equals_local_communicator(transport, nranks):
    spec = dict(mode="fast", block=(10, 6, 12), tol=1e-6, max_iterations=800)
    glob = scenarios.block_case(10, 6, 12, h=0.1, tol=1e-6, max_iterations=800)
    P = glob.packing
    sK, sM = glob.scalars()
    ranges = shard.slab_ranges(P.node_count, nranks)
    spec["ranges"] = [int(v) for v in ranges]
    out = _run(spec, nranks, transport)
    x, _ = _assemble(out, P)
    # the same decomposition in this process over the LOCAL communicator
    comm = shard.Comm.local(nranks)
    systems, shards, rhs, xs = [], [], [], []
    for k in range(nranks):
        src = pcg.MatrixFreeSystem.from_packing(P, glob.materials, sK, sM, mode=_lib.MODE_FAST)
        sh = shard.build_shard(src, ranges, k)
        s = sh.system(glob.materials, sK, sM)
        comm.attach(s, sh)
        systems.append(s)
        shards.append(sh)
        rhs.append(sh.local_dofs(glob.static_rhs()))
        xs.append(np.zeros(3 * sh.local_nodes, np.float32))
    tl = shard.solve_pcg_group(systems, rhs, pcg.PcgSettings(800, 1e-6), xs).value()
    xl = np.zeros((P.node_count, 3), np.float32)
    for sh, v in zip(shards, xs):
        xl[sh.node_global[: sh.owned_nodes].astype(np.int64)] = v.reshape(-1, 3)[: sh.owned_nodes]
    comm.close()
    for d in out.values():
        assert d["telemetry"][:3] == (tl.iterations, tl.converged, tl.residual_norm)
    assert_bitwise(x, xl.reshape(-1), "multi-process FAST x vs LOCAL")
    ref = oracle_system(P, glob.materials, sK, sM).solve_pcg(glob.static_rhs(), 800, 1e-6)
    assert tl.converged
    assert np.linalg.norm(x - ref["x"]) <= 1e-4 * np.linalg.norm(ref["x"])


def test_multiprocess_parity_newmark_steps_bitwise_equal_single_handle(transport):
    """Three PARITY Newmark steps (Rayleigh beta_R != 0, so the damping K_eff product runs on the shards too) on
    2 processes: u, v, a and every step's PCG telemetry equal the one-handle Stepper's bit for bit."""
    from cwf.stepper import Stepper

    spec = dict(block=(10, 6, 12), tol=1e-6, max_iterations=800, rayleigh=True, steps=3)
    import transport_worker

    glob = transport_worker.case_for(spec)
    P = glob.packing
    spec["ranges"] = [int(v) for v in shard.slab_ranges(P.node_count, 2, align=256)]
    out = _run(spec, 2, transport, target="run_rank_stepper")
    st = Stepper(P, glob.materials, glob.rayleigh, glob.cfg.solver, glob.cfg.time)
    ref_tel = []
    t = 0.0
    for _ in range(spec["steps"]):
        tel = st.step(t).value()
        ref_tel.append((tel.pcg.iterations, tel.pcg.converged, tel.pcg.residual_norm))
        t += glob.cfg.time.initial_dt
    assert abs(glob.rayleigh.beta) > 0
    for d in out.values():
        assert d["telemetry"] == ref_tel
    for key, which in (("u", Stepper.DISPLACEMENT), ("v", Stepper.VELOCITY), ("a", Stepper.ACCELERATION)):
        ref = st.get_state(which)
        got = np.zeros((P.node_count, 3), np.float32)
        for d in out.values():
            got[d["nodes"]] = d[key].reshape(-1, 3)
        assert_bitwise(got.reshape(-1), ref, f"multi-process PARITY Stepper {key}")
    st.close()
