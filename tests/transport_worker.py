"""One rank of a multi-process sharded solve on one GPU through the RCCL code path of comm.cpp, with the
host-staged test transport (tests/transport/host_nccl.cpp, loaded through CWF_RCCL_LIB) underneath.
Spawned by tests/test_gpu_transport.py; returns the rank's owned rows and telemetry through a queue."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "civiwave-fem_amd"), os.path.join(ROOT, "tests"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def case_for(spec):
    from cwf import scenarios

    nx, ny, nz = spec["block"]
    return scenarios.block_case(nx, ny, nz, h=0.1, tol=spec["tol"], max_iterations=spec["max_iterations"])


def run_rank(rank, nranks, uid, spec, queue):
    try:
        import numpy as np

        from cwf import _lib, pcg, shard

        mode = _lib.MODE_PARITY if spec["mode"] == "parity" else _lib.MODE_FAST
        glob = case_for(spec)
        sK, sM = glob.scalars()
        P = glob.packing
        ranges = np.asarray(spec["ranges"], np.uint64)
        src = pcg.MatrixFreeSystem.from_packing(P, glob.materials, sK, sM, mode=mode)
        sh = shard.build_shard(src, ranges, rank)
        s = sh.system(glob.materials, sK, sM, mode=mode)
        comm = shard.Comm.rccl(nranks, rank, uid, 0)
        comm.attach(s, sh)
        rhs = sh.local_dofs(glob.static_rhs())
        x = np.zeros(3 * sh.local_nodes, np.float32)
        r = np.zeros_like(x)
        res = pcg.solve_pcg(s, rhs, pcg.PcgSettings(spec["max_iterations"], spec["tol"]), pcg.PcgVectors(x, r))
        if not res.has_value():
            queue.put((rank, "error", str(res.error())))
            return
        t = res.value()
        hist = pcg.residual_history(s)
        g = sh.node_global[: sh.owned_nodes].astype(np.int64)
        own = 3 * sh.owned_nodes
        queue.put((rank, "ok", dict(
            telemetry=(t.iterations, t.converged, t.residual_norm, t.rhs_norm, t.alpha_last, t.beta_last),
            nodes=g, x=x[:own].copy(), r=r[:own].copy(), history=hist,
            halo_consistent=bool(np.all(np.isfinite(x))))))
        s.close()
        comm.close()
    except Exception as e:  # reported to the parent, which fails the test with it
        import traceback

        queue.put((rank, "error", f"{e!r}\n{traceback.format_exc()}"))
