"""The PEER communicator (peer.hip): 2 and 3 processes on one GPU, each rank's mailbox IPC-mapped by the others.

The exchange steps are device-initiated stores into the peers' mailboxes and a flag per step instead of RCCL
groups; the kernels, fold orders and halo plans above them are the ones the LOCAL communicator runs, so:
- the FAST iteration on structured slab sub-meshes (the lattice stencil; two exchange steps per iteration: p.Ap,
  then {r.r, r.z} with the z halo) equals the LOCAL solve of the same decomposition bit for bit;
- so does the FAST iteration on a global-mesh node partition (the fan-group tiles);
- a PARITY solve over PEER is refused (its chunk-partial all-gathers stay on RCCL / LOCAL);
- the exchange latency per step is measured (printed; DESIGN.md section 7 uses it). Two processes on one GPU
  share its CUs, so this is the protocol's latency on one device, not an xGMI figure;
- the mailboxes are uncached device memory (hipDeviceMallocUncached, IPC-exported): another device's stores are
  visible to the receiver without trusting its L2;
- a rank that connects and then never exchanges ends the others' solve with CWF_ERR_COMM within the wait's bound
  (10 s), and the exchange trial cwf_hip_comm_time_exchange reports the dead communicator;
- the resident solve of the slabs (resident.hip, the default where every rank can plan it: one launch per solve,
  the send planes' records and the rank totals stored into the peers' mailboxes by the kernel) follows the LOCAL
  fused schedule within 1e-5 after fixed iteration counts and the oracle within 1e-4 at convergence (its dots are
  grouped by box, so it is tolerance-equal, not bit-equal), repeats itself bit for bit. The bit-exact cases above run with CWF_RESIDENT=0 (a peer that never arrives fails
  the schedule vote's exchange before any resident launch; one lost mid-solve ends it at the polls' bound)."""
import multiprocessing as mp
import os
import tempfile

import numpy as np
import pytest

import oracle as O
from cwf import _lib, pcg, scenarios, shard
from helpers import assert_bitwise, oracle_system

pytestmark = pytest.mark.gpu


def _run(spec, nranks):
    import transport_worker

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    rdv = tempfile.mkdtemp(prefix="cwf_peer.")
    procs = [ctx.Process(target=transport_worker.run_rank_peer, args=(k, nranks, rdv, spec, q)) for k in range(nranks)]
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
    return out


def _local_slab(shape, nranks, tol, mi, element="tet4"):
    glob = scenarios.block_case(shape[0], shape[1], shape[2] * nranks, h=0.1, element=element, tol=tol,
                                max_iterations=mi)
    sK, sM = glob.scalars()
    comm = shard.Comm.local(nranks)
    systems, shards, rhs, xs = [], [], [], []
    for r in range(nranks):
        case, node_global, begin = scenarios.slab_case_shape(shape, nranks, r, element=element, tol=tol)
        src = pcg.MatrixFreeSystem.from_packing(case.packing, case.materials, sK, sM, mode=_lib.MODE_FAST)
        sh = shard.build_shard(src, begin, r, node_global)
        s = sh.system(glob.materials, sK, sM)
        comm.attach(s, sh)
        systems.append(s)
        shards.append(sh)
        rhs.append(sh.local_dofs(case.static_rhs()))
        xs.append(np.zeros(3 * sh.local_nodes, np.float32))
    t = shard.solve_pcg_group(systems, rhs, pcg.PcgSettings(mi, tol), xs).value()
    x = np.zeros((glob.packing.node_count, 3), np.float32)
    for sh, v in zip(shards, xs):
        x[sh.node_global[: sh.owned_nodes].astype(np.int64)] = v.reshape(-1, 3)[: sh.owned_nodes]
    comm.close()
    return glob, t, x.reshape(-1)


def _assemble(out, n):
    x = np.zeros((n, 3), np.float32)
    for d in out.values():
        x[d["nodes"]] = d["x"].reshape(-1, 3)
    return x.reshape(-1)


@pytest.mark.parametrize("element", ["tet4", "hex8"])
@pytest.mark.parametrize("inkernel", [True, False, "persistent"],
                         ids=["in_kernel_exchange", "exchange_step", "in_kernel_persistent"])
@pytest.mark.parametrize("nranks", [2, 3])
def test_peer_lattice_slabs_equal_local(nranks, inkernel, element, monkeypatch):
    """in_kernel_exchange: the fused launches push their Ap send rows, rank totals and epoch flags themselves and
    wait for the peers' in their prologue (lattice_fused.inc fused_peer_wait / fused_peer_publish: no exchange
    launch); exchange_step (CWF_PEER_FUSED=0): one k_peer_step launch after each fused launch. Both equal the LOCAL
    solve bit for bit, and a second solve on the same communicator repeats the first (the epochs carry over).
    in_kernel_persistent: the same with an 8-workgroup grid walking the items (CWF_FUSED=2), in both the PEER
    processes and the LOCAL reference (the last workgroup's rank-total fold over the grid's shares). hex8: the
    27-point stencil's shard instantiations (two-deep prefetch with the mailbox's ghost Ap planes)."""
    shape = (13, 9, 4)
    spec = dict(slab=shape, tol=1e-6, max_iterations=800, timing_steps=1000, element=element,
                env={"CWF_RESIDENT": "0"})
    if not inkernel:
        spec["env"] = {"CWF_PEER_FUSED": "0", "CWF_RESIDENT": "0"}
    if inkernel == "persistent":
        spec["env"] = {"CWF_FUSED": "2", "CWF_FUSED_MAXWG": "8"}
        monkeypatch.setenv("CWF_FUSED", "2")
        monkeypatch.setenv("CWF_FUSED_MAXWG", "8")
    out = _run(spec, nranks)
    glob, tl, xl = _local_slab(shape, nranks, 1e-6, 800, element)
    x = _assemble(out, glob.packing.node_count)
    for d in out.values():
        # the fused lattice iteration with its ghost-plane stores (SHARD), on every rank (rank 0's affine planes too)
        assert d["kernel"].startswith("k_pcg_lattice") and d["kernel"].endswith(
            "true, true>" if inkernel == "persistent" else "true, false>"), d["kernel"]
        assert d["schedule"] == (2 if inkernel else 1), d["schedule"]
        assert d["mailbox_kind"] == _lib.PEER_MAILBOX_UNCACHED, d["mailbox_kind"]
        assert d["telemetry"] == (tl.iterations, tl.converged, tl.residual_norm)
        assert d["telemetry2"] == d["telemetry"]
        assert_bitwise(d["x2"], d["x"], "second solve x")
        # refused (the slabs are not whole reduction chunks, and PEER carries the FAST schedule only), never a hang
        assert d["parity_error"] and ("FAST schedule" in d["parity_error"] or "whole" in d["parity_error"]
                                      or "reduction" in d["parity_error"]
                                      or "hex8 elements run in CWF_MODE_FAST only" in d["parity_error"]), d["parity_error"]
    assert_bitwise(x, xl, "PEER lattice slabs x vs LOCAL")
    assert tl.converged
    if element == "hex8":  # the fp64 solve of the hex8 oracle operator
        P = glob.packing
        ref = {"x": O.hex8_solve64(glob.mesh.coords, glob.mesh.tets, P.material_index, O.make_stiffness(30.0e9, 0.2),
                                   *glob.scalars(), P.lumped_mass, P.bc_mask, glob.static_rhs())}
    else:
        ref = oracle_system(glob.packing, glob.materials, *glob.scalars()).solve_pcg(glob.static_rhs(), 800, 1e-6)
    assert np.linalg.norm(x - ref["x"]) <= 1e-4 * np.linalg.norm(ref["x"])
    print(f"PEER exchange step, {nranks} processes on one GPU: "
          + ", ".join(f"rank {k} {d['exchange_us']:.2f} us" for k, d in sorted(out.items())))


def test_peer_global_partition_equals_local():
    nranks = 2
    glob = scenarios.block_case(10, 6, 12, h=0.1, tol=1e-6, max_iterations=800)
    P = glob.packing
    sK, sM = glob.scalars()
    ranges = shard.slab_ranges(P.node_count, nranks)
    spec = dict(block=(10, 6, 12), tol=1e-6, max_iterations=800, ranges=[int(v) for v in ranges],
                env={"CWF_RESIDENT": "0"})
    out = _run(spec, nranks)
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
        assert d["telemetry"] == (tl.iterations, tl.converged, tl.residual_norm)
        assert d["parity_error"] and ("FAST schedule" in d["parity_error"] or "reduction" in d["parity_error"]
                                      or "contiguous" in d["parity_error"]), d["parity_error"]
    assert_bitwise(_assemble(out, P.node_count), xl.reshape(-1), "PEER global partition x vs LOCAL")
    print("PEER exchange step, 2 processes on one GPU: "
          + ", ".join(f"rank {k} {d['exchange_us']:.2f} us" for k, d in sorted(out.items())))


def test_peer_dead_rank_ends_the_solve_with_comm_error():
    shape = (9, 7, 4)
    out = _run(dict(slab=shape, tol=1e-6, max_iterations=400, dead_rank=1, env={"CWF_RESIDENT": "0"}), 2)
    live = out[0]
    assert out[1]["dead"] and not live["dead"]
    assert live["error"] == "peer exchange timed out", live["error"]
    # one bounded wait (10 s), not one per queued exchange step
    assert live["seconds"] < 60.0, live["seconds"]
    assert live["trial_error"] and "timed out" in live["trial_error"], live["trial_error"]


@pytest.mark.parametrize("element", ["tet4", "hex8"])
@pytest.mark.parametrize("nranks", [2, 3])
def test_peer_resident_slabs(nranks, element):
    """The resident solve on PEER slab shards: after 3 and 20 fixed iterations (tol 1e-30) x within 1e-5 (relative)
    of the LOCAL fused schedule's; converged (tol 1e-6) within 1e-4 of the oracle's x, in the LOCAL iteration count
    +-5%; a second solve on the same communicator equal bit for bit (the granule tags continue across solves)."""
    shape = (13, 9, 4)
    for its in (3, 20):
        out = _run(dict(slab=shape, tol=1e-30, max_iterations=its, timing_steps=50, element=element), nranks)
        glob, tl, xl = _local_slab(shape, nranks, 1e-30, its, element)
        x = _assemble(out, glob.packing.node_count)
        for d in out.values():
            assert d["kernel_after"].startswith("k_pcg_resident<") and d["kernel_after"].endswith(", true>"), \
                d["kernel_after"]
            assert d["schedule"] == 3, d["schedule"]
            assert d["telemetry"][0] == its == tl.iterations
            assert_bitwise(d["x2"], d["x"], "second solve x")
        assert np.linalg.norm(x - xl) <= 1e-5 * np.linalg.norm(xl), (its, np.linalg.norm(x - xl) / np.linalg.norm(xl))
    out = _run(dict(slab=shape, tol=1e-6, max_iterations=800, timing_steps=50, element=element), nranks)
    glob, tl, xl = _local_slab(shape, nranks, 1e-6, 800, element)
    x = _assemble(out, glob.packing.node_count)
    for d in out.values():
        assert d["telemetry"][1] and d["telemetry2"] == d["telemetry"]
        assert abs(d["telemetry"][0] - tl.iterations) <= max(2, tl.iterations // 20), (d["telemetry"], tl.iterations)
        assert_bitwise(d["x2"], d["x"], "second solve x")
    if element == "hex8":
        P = glob.packing
        ref = {"x": O.hex8_solve64(glob.mesh.coords, glob.mesh.tets, P.material_index, O.make_stiffness(30.0e9, 0.2),
                                   *glob.scalars(), P.lumped_mass, P.bc_mask, glob.static_rhs())}
    else:
        ref = oracle_system(glob.packing, glob.materials, *glob.scalars()).solve_pcg(glob.static_rhs(), 800, 1e-6)
    assert np.linalg.norm(x - ref["x"]) <= 1e-4 * np.linalg.norm(ref["x"])
    print(f"PEER resident, {nranks} ranks {element}: {out[0]['telemetry'][0]} it (LOCAL fused {tl.iterations})")



def test_peer_resident_needs_every_rank():
    """Slabs one cell thick: the ranks owning a single node plane can plan neither a resident solve (a box needs
    two planes) nor the fused launch, the last rank (two planes) could; the schedule vote is collective, so every
    rank runs the two kernels (schedule 0) and equals the LOCAL solve bit for bit, never a mixed schedule."""
    shape = (13, 9, 1)
    out = _run(dict(slab=shape, tol=1e-6, max_iterations=800, timing_steps=50), 3)
    glob, tl, xl = _local_slab(shape, 3, 1e-6, 800)
    assert tl.converged
    for d in out.values():
        assert d["kernel_after"].startswith("k_keff_lattice"), d["kernel_after"]
        assert d["schedule"] == 0, d["schedule"]
        assert d["telemetry"] == (tl.iterations, tl.converged, tl.residual_norm)
    assert_bitwise(_assemble(out, glob.packing.node_count), xl, "PEER one-cell slabs x vs LOCAL")
