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
    extra = {"xi": 0.05, "w": (10.0, 100.0)} if spec.get("rayleigh") else {}
    return scenarios.block_case(nx, ny, nz, h=0.1, tol=spec["tol"], max_iterations=spec["max_iterations"], **extra)


def run_rank_stepper(rank, nranks, uid, spec, queue):
    """`spec["steps"]` PARITY Newmark steps on this rank's shard (the bench's Stepper over a shard); returns the
    owned rows of u / v / a and each step's telemetry."""
    try:
        import numpy as np

        from cwf import _lib, pcg, shard
        from cwf.stepper import Stepper

        glob = case_for(spec)
        P = glob.packing
        sK, sM = glob.scalars()
        ranges = np.asarray(spec["ranges"], np.uint64)
        src = pcg.MatrixFreeSystem.from_packing(P, glob.materials, sK, sM, mode=_lib.MODE_PARITY)
        sh = shard.build_shard(src, ranges, rank)
        s = sh.system(glob.materials, 1.0, 0.0, mode=_lib.MODE_PARITY)
        comm = shard.Comm.rccl(nranks, rank, uid, 0)
        comm.attach(s, sh)

        class _LocalPacking:
            external_force = sh.local_dofs(P.external_force)
            bc_value = sh.local_dofs(P.bc_value)
            dof_count = 3 * sh.local_nodes
            node_count = sh.local_nodes

        st = Stepper(_LocalPacking, glob.materials, glob.rayleigh, glob.cfg.solver, glob.cfg.time,
                     mode=_lib.MODE_PARITY, system=s)
        tels = []
        t = 0.0
        for _ in range(spec["steps"]):
            tel = st.step(t).value()
            tels.append((tel.pcg.iterations, tel.pcg.converged, tel.pcg.residual_norm))
            t += glob.cfg.time.initial_dt
        own = 3 * sh.owned_nodes
        out = {k: st.get_state(w)[:own].copy() for k, w in (("u", Stepper.DISPLACEMENT), ("v", Stepper.VELOCITY),
                                                               ("a", Stepper.ACCELERATION))}
        out.update(nodes=sh.node_global[: sh.owned_nodes].astype(np.int64), telemetry=tels)
        queue.put((rank, "ok", out))
        st.close()
        comm.close()
    except Exception as e:
        import traceback

        queue.put((rank, "error", f"{e!r}\n{traceback.format_exc()}"))


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
