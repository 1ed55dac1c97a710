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


def run_rank_peer(rank, nranks, rdv, spec, queue):
    """One rank over the PEER communicator (peer.hip): the IPC handles of the ranks' mailboxes are exchanged through
    files in the rendezvous directory `rdv`. spec["slab"] = (nx, ny, nz per rank): the bench's slab sub-meshes
    (structured block: the lattice stencil); else spec["ranges"] over
    the global block. Returns the owned x, the telemetry, the exchange latency and the error of a PARITY solve."""
    try:
        import time

        import numpy as np

        for k, v in spec.get("env", {}).items():
            os.environ[k] = v
        from cwf import _lib, pcg, scenarios, shard

        if spec.get("slab"):
            shape = tuple(spec["slab"])
            element = spec.get("element", "tet4")
            glob = scenarios.block_case(shape[0], shape[1], shape[2] * nranks, h=0.1, element=element, tol=spec["tol"],
                                        max_iterations=spec["max_iterations"])
            sK, sM = glob.scalars()
            case, node_global, begin = scenarios.slab_case_shape(shape, nranks, rank, element=element, tol=spec["tol"])
            src = pcg.MatrixFreeSystem.from_packing(case.packing, case.materials, sK, sM, mode=_lib.MODE_FAST)
            sh = shard.build_shard(src, begin, rank, node_global)
            rhs = sh.local_dofs(case.static_rhs())
        else:
            glob = case_for(spec)
            sK, sM = glob.scalars()
            src = pcg.MatrixFreeSystem.from_packing(glob.packing, glob.materials, sK, sM, mode=_lib.MODE_FAST)
            sh = shard.build_shard(src, np.asarray(spec["ranges"], np.uint64), rank)
            rhs = sh.local_dofs(glob.static_rhs())
        s = sh.system(glob.materials, sK, sM)
        comm = shard.Comm.peer(nranks, rank, 0)
        comm.attach(s, sh)
        with open(os.path.join(rdv, f"rank{rank}.tmp"), "wb") as fh:
            fh.write(comm.handle())
        os.replace(os.path.join(rdv, f"rank{rank}.tmp"), os.path.join(rdv, f"rank{rank}.bin"))
        t0 = time.time()
        while not all(os.path.exists(os.path.join(rdv, f"rank{p}.bin")) for p in range(nranks)):
            if time.time() - t0 > 120:
                raise RuntimeError("rendezvous timed out")
            time.sleep(0.05)
        comm.connect([open(os.path.join(rdv, f"rank{p}.bin"), "rb").read() for p in range(nranks)])
        kern = (_lib.load().cwf_hip_system_keff_kernel(s.handle()) or b"").decode()
        mkind = comm.mailbox_kind()
        if spec.get("dead_rank") is not None:
            # one rank connects and then never exchanges; the others' solve must end with CWF_ERR_COMM, in bounded time
            if rank == spec["dead_rank"]:
                queue.put((rank, "ok", dict(dead=True, mailbox_kind=mkind)))
                t0 = time.time()
                while not os.path.exists(os.path.join(rdv, "done")) and time.time() - t0 < 200:
                    time.sleep(0.05)
            else:
                x = np.zeros(3 * sh.local_nodes, np.float32)
                t0 = time.time()
                res = pcg.solve_pcg(s, rhs, pcg.PcgSettings(spec["max_iterations"], spec["tol"]),
                                    pcg.PcgVectors(x, None))
                el = time.time() - t0
                us_err = None
                try:
                    shard.Comm.time_exchange(s, 4)
                except RuntimeError as e:
                    us_err = str(e)
                with open(os.path.join(rdv, "done"), "w") as fh:
                    fh.write("1")
                queue.put((rank, "ok", dict(dead=False, mailbox_kind=mkind, seconds=el,
                                            kernel_after=(_lib.load().cwf_hip_system_keff_kernel(s.handle())
                                                          or b"").decode(),
                                            error=None if res.has_value() else res.error().message,
                                            trial_error=us_err)))
            s.close()
            comm.close()
            return
        x = np.zeros(3 * sh.local_nodes, np.float32)
        res = pcg.solve_pcg(s, rhs, pcg.PcgSettings(spec["max_iterations"], spec["tol"]), pcg.PcgVectors(x, None))
        if not res.has_value():
            queue.put((rank, "error", str(res.error())))
            return
        t = res.value()
        sched = _lib.load().cwf_hip_system_exchange_schedule(s.handle())
        kern_after = (_lib.load().cwf_hip_system_keff_kernel(s.handle()) or b"").decode()  # the agreed schedule's
        # a second solve on the same communicator (the in-kernel exchange's epochs continue across solves)
        x2 = np.zeros(3 * sh.local_nodes, np.float32)
        t0 = time.perf_counter()
        t2 = pcg.solve_pcg(s, rhs, pcg.PcgSettings(spec["max_iterations"], spec["tol"]),
                           pcg.PcgVectors(x2, None)).value()
        solve2_s = time.perf_counter() - t0
        us = shard.Comm.time_exchange(s, spec.get("timing_steps", 200))
        # PARITY over PEER is refused (its chunk-partial all-gathers need RCCL / LOCAL)
        s.mode = _lib.MODE_PARITY  # (the handle takes the system's mode at every call)
        try:
            pres = pcg.solve_pcg(s, rhs, pcg.PcgSettings(10, spec["tol"]), pcg.PcgVectors(np.zeros_like(x), None))
            perr = None if pres.has_value() else pres.error().message
        except pcg.PcgException as e:  # hex8: the handle refuses PARITY itself
            perr = str(e)
        s.mode = _lib.MODE_FAST
        own = 3 * sh.owned_nodes
        queue.put((rank, "ok", dict(telemetry=(t.iterations, t.converged, t.residual_norm), kernel=kern,
                                    kernel_after=kern_after,
                                    nodes=sh.node_global[: sh.owned_nodes].astype(np.int64), x=x[:own].copy(),
                                    exchange_us=us, parity_error=perr, mailbox_kind=mkind, schedule=sched,
                                    telemetry2=(t2.iterations, t2.converged, t2.residual_norm),
                                    x2=x2[:own].copy(), solve2_s=solve2_s)))
        s.close()
        comm.close()
    except Exception as e:
        import traceback

        queue.put((rank, "error", f"{e!r}\n{traceback.format_exc()}"))
