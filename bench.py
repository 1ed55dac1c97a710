#!/usr/bin/env python3
"""Benchmark of the matrix-free implicit Newmark/PCG hot path on MI355X.

One "step" = one full Stepper::step (predictor -> RHS -> Dirichlet clamp -> block-Jacobi PCG with
warm start -> corrector) on the configs[1] workload of BASELINE.json: the 69^3-hex block expanded to
1,971,054 Kuhn tets (343,000 nodes, 1,029,000 DOF), all inputs resident in HBM before timing.

Prints ONE JSON line (rank 0). value = PCG DOF-iterations per second over the whole job
(sum over ranks of DOFs x PCG iterations / max-over-ranks wall time of the K timed steps).
Extra fields: pcg_iterations_per_sec, dof_updates_per_sec (D x steps/s), the live roofline of the
dominant kernel (K_eff, timed with hipEvents on the handle's stream inside the timed steps) and a
bounded single-thread CPU baseline (the oracle restatement of the reference's solve_pcg).

Multi-GPU (python -m torch.distributed.run ... bench.py --gpus N): weak scaling, one process per
GPU. The global block stacks N copies of the per-GPU workload along z; rank r owns a contiguous range
of node planes, builds only its slab sub-mesh (+ one ghost cell layer) and solves as one shard of the
global system: all-gathers of the PCG scalars (p.Ap, r.r / r.z, 8-16 B per rank) and one halo of z per
iteration over xGMI, by default through the PEER communicator (csrc/peer.hip: one launch per exchange step,
device stores into the neighbours' IPC-mapped mailboxes), with RCCL groups (csrc/comm.cpp) when any rank
cannot map its peers (--comm auto; --comm rccl / peer to force one). value = sum over ranks of owned DOFs x
PCG iterations / max-over-ranks wall time.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "civiwave-fem_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec 8.0 TB/s)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="c2", help="BASELINE config key (c1..c5)")
    ap.add_argument("--mode", default="fast", choices=["fast", "parity"])
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"],
                    help="N>1: weak = the config's block per GPU (N stacked copies), strong = the config's block "
                         "split over the N GPUs (SURVEY 8e: C3's fixed 10.1M DOF at 1/2/4/8 GPUs). Unstructured "
                         "configs (c4) always scale strong over an RCB node partition")
    ap.add_argument("--element", default="tet4", choices=["tet4", "hex8"],
                    help="tet4: the Kuhn expansion the reference runs (the headline); hex8: native hexes "
                         "(SURVEY 8f4, FAST only, parity unpinned)")
    ap.add_argument("--max-iterations", type=int, default=2000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--keff-sample", type=int, default=5,
                    help="hipEvent-time every k-th K_eff launch of the timed steps (1 = all). Coprime with the lazy-x "
                         "period (4): every 4th update also writes x, and sampling every 4th launch timed only the "
                         "launches right after those (C3: 105 us against rocprofv3's 98 us average)")
    ap.add_argument("--cpu-iterations", type=int, default=40)
    ap.add_argument("--no-general-roofline", action="store_true",
                    help="skip roofline_general (the fan-group tiles kernel on C3 with the lattice stencil off)")
    ap.add_argument("--comm", default="auto", choices=["rccl", "peer", "auto"],
                    help="N>1 exchange steps: RCCL groups, or the PEER communicator's device-initiated stores into "
                         "IPC-mapped mailboxes (FAST only); auto: PEER when every rank maps every peer and a trial "
                         "exchange completes on all of them, else RCCL")
    ap.add_argument("--no-general", action="store_true",
                    help="skip the 'general' block (the same workload on the fan-group tiles, CWF_LATTICE=0)")
    ap.add_argument("--no-parity", action="store_true",
                    help="skip the 'parity' block (the same workload in the bit-exact PARITY mode, c1/c2 only)")
    ap.add_argument("--no-hbm-roofline", action="store_true",
                    help="skip the live configs[2] K_eff roofline (N=1 runs of configs other than c3 add it)")
    ap.add_argument("--traffic", default="auto",
                    help="PMC summary json for roofline.traffic; 'auto' = newest profiles/r*_<config>_<mode>_pmc.json")
    return ap.parse_args()


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown CPU"


def cpu_baseline(case, sK, sM, iters):
    """The bit-exact CPU restatement (ours, oracle/cwf_oracle.c) of the reference's single-threaded solve_pcg,
    pinned to one core of this host for the CPU leg only (os.sched_setaffinity on this thread, restored
    afterwards): block-Jacobi setup + `iters` PCG iterations on the bench workload, plus a
    full C1 solve to its tolerance. The restatement omits the reference's per-call validate_system and its unused
    fp64 D*B product (pcg.cpp:82-139, 592-604), so it runs ~3x faster than the reference itself (the survey
    measured 5.25 M DOF-it/s on C2)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from helpers import oracle_system  # noqa: E402

    from cwf import scenarios

    prev = os.sched_getaffinity(0)
    core = min(prev)
    os.sched_setaffinity(0, {core})
    try:
        s = oracle_system(case.packing, case.materials, sK, sM)
        rhs = case.static_rhs()
        t0 = time.perf_counter()
        out = s.solve_pcg(rhs, iters, 1e-30)
        dt = time.perf_counter() - t0
        it = out["telemetry"].iterations
        c1 = scenarios.config_case("c1")
        s1 = oracle_system(c1.packing, c1.materials, *c1.scalars())
        t1 = time.perf_counter()
        o1 = s1.solve_pcg(c1.static_rhs(), c1.cfg.solver.max_iterations, c1.cfg.solver.runtime_tolerance)
        d1 = time.perf_counter() - t1
    finally:
        os.sched_setaffinity(0, prev)
    it1 = o1["telemetry"].iterations
    return dict(value=case.packing.dof_count * it / dt, unit="DOF-it/s", cores=1, kind="port",
                label="bit-exact restatement (ours), not the reference binary",
                cpu_model=cpu_model(), core=core, host_cpus=os.cpu_count(),
                sample=f"{case.name}: oracle solve_pcg (block-Jacobi setup + {it} PCG iterations), {dt:.2f} s, "
                       f"1 thread pinned to core {core}",
                c1_full_solve={"iterations": int(it1), "seconds": d1, "pcg_iterations_per_sec": it1 / d1,
                               "dof_it_per_sec": c1.packing.dof_count * it1 / d1,
                               "converged": bool(o1["telemetry"].converged)})


def pmc_traffic(paths, kname, src_hash):
    """HBM bytes per launch of kernel `kname` from the newest committed PMC summary among `paths` that profiled it
    AND recorded the running library's source hash of that kernel (cwf_hip_system_keff_source_hash): a profile of an
    older build of the same template instantiation is not this code's traffic. (None, None) when
    no profile of the current code exists."""
    for path in sorted(paths, reverse=True):
        pmc = json.load(open(path))
        if pmc.get("source_hash") == src_hash and any(same_kernel(kname, k) for k in pmc.get("kernels", {})):
            return pmc.get("hbm_bytes_per_launch"), os.path.relpath(path, ROOT)
    return None, None


def c3_pmc_traffic(kname, src_hash):
    import glob

    return pmc_traffic(glob.glob(os.path.join(ROOT, "profiles", "r*_c3_fast*_pmc.json")), kname, src_hash)


def hbm_roofline(L, device, key="c3", steps=2, sample=5, general=False):
    """The same PCG-mode K_eff kernel, live, on the configs[2] block (C2's working set sits in
    the 256 MB MALL, so its roofline is not an HBM figure; C3 moves 0.38 GB per launch): `steps` FAST Newmark
    steps of C3 after one untimed step, every `sample`-th K_eff launch hipEvent-timed on the handle's stream
    exactly as in the main timed steps (coprime with the lazy-x period). Round 2 timed a 200-iteration solve
    from x = 0 instead, which read ~10% above rocprofv3's average of the same kernel (109 vs 98 us); a C3
    Newmark step's launches read within 1% of it. Outside the timed Newmark steps, so it changes no other field.
    general=True: the same with the structured-block stencil switched off (CWF_LATTICE=0), i.e. the fan-group
    tiles kernel every unstructured mesh runs (C4's), on the same C3 block."""
    import ctypes as C

    from cwf import _lib, scenarios
    from cwf.stepper import Stepper

    case = scenarios.config_case(key)
    P = case.packing
    prev = os.environ.get("CWF_LATTICE")
    if general:
        os.environ["CWF_LATTICE"] = "0"
    try:
        st = Stepper(P, case.materials, case.rayleigh, case.cfg.solver, case.cfg.time, mode=_lib.MODE_FAST,
                     device=device)
        h = st.system.handle()
    finally:
        if general:
            if prev is None:
                os.environ.pop("CWF_LATTICE", None)
            else:
                os.environ["CWF_LATTICE"] = prev
    t = 0.0
    st.step(t).value()
    t += case.cfg.time.initial_dt
    L.cwf_hip_system_set_timing(h, sample)
    for _ in range(steps):
        st.step(t).value()
        t += case.cfg.time.initial_dt
    ms, n = C.c_double(), C.c_uint64()
    L.cwf_hip_system_timing(h, C.byref(ms), C.byref(n))
    L.cwf_hip_system_set_timing(h, 0)
    lay_b, ref_b = C.c_uint64(), C.c_uint64()
    L.cwf_hip_system_keff_traffic(h, C.byref(lay_b), C.byref(ref_b))
    avg = ms.value / max(1, n.value)
    ach = lay_b.value / (avg * 1e-3) / 1e9
    out = {"bound": "hbm", "workload": case.name + f" ({steps} FAST Newmark steps after 1 untimed)",
           "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBS,
           "kernel": (L.cwf_hip_system_keff_kernel(h) or b"").decode(), "avg_launch_ms": avg,
           "launches": int(n.value), "algorithmic_bytes_per_launch": float(lay_b.value),
           "reference_layout_equiv_gbs": ref_b.value / (avg * 1e-3) / 1e9}
    out["kernel_source_hash"] = (L.cwf_hip_system_keff_source_hash(h) or b"").decode()
    out["traffic"], out["traffic_source"] = c3_pmc_traffic(out["kernel"], out["kernel_source_hash"])
    st.close()
    st.system.close()
    return out


def operator_of(kname: str) -> str:
    """Which operator a K_eff kernel name is: the structured-block stencil (reached only by exact structured Kuhn /
    hex8 boxes of one material, lattice.cpp) or the general element tiles every other mesh runs."""
    if kname.startswith("k_pcg_resident"):
        return "structured-block stencil, resident one-launch PCG solve (vectors on chip, one workgroup per box)"
    if kname.startswith("k_pcg_lattice"):
        return "structured-block stencil, fused single-launch PCG iteration"
    if kname.startswith("k_keff_lattice"):
        return "structured-block stencil, two-kernel PCG iteration"
    if kname.startswith("k_keff_groups_pipe"):
        return "general mesh: fan-group element tiles"
    if kname.startswith("k_keff_parity"):
        return "bit-exact PARITY element pass + node fold"
    return "general mesh: element tiles (" + kname.split("<")[0] + ")"


def side_line(L, device, key, steps, warmup=1, sample=5, mode="general"):
    """A comparator on the same workload, timed like the headline (whole Newmark steps, K_eff hipEvent-sampled) after
    the headline's timed region, so the two are never conflated. mode="general": the structured-block stencil
    switched off (CWF_LATTICE=0), i.e. the fan-group tiles that any gmsh mesh, C4 and every non-lattice scenario run.
    mode="parity": the bit-exact PARITY path (the reference's fp64 element math and fold order, pcg.cpp:561-691),
    the only mode whose residuals match the reference bit for bit."""
    import ctypes as C

    from cwf import _lib, scenarios
    from cwf.stepper import Stepper

    case = scenarios.config_case(key)
    P = case.packing
    prev = os.environ.get("CWF_LATTICE")
    if mode == "general":
        os.environ["CWF_LATTICE"] = "0"
    try:
        st = Stepper(P, case.materials, case.rayleigh, case.cfg.solver, case.cfg.time,
                     mode=_lib.MODE_PARITY if mode == "parity" else _lib.MODE_FAST, device=device)
        h = st.system.handle()
    finally:
        if prev is None:
            os.environ.pop("CWF_LATTICE", None)
        else:
            os.environ["CWF_LATTICE"] = prev
    import torch

    t = 0.0
    for _ in range(warmup):
        st.step(t).value()
        t += case.cfg.time.initial_dt
    L.cwf_hip_system_set_timing(h, sample)
    torch.cuda.synchronize()
    iters = 0
    t0 = time.perf_counter()
    for _ in range(steps):
        iters += st.step(t).value().pcg.iterations
        t += case.cfg.time.initial_dt
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    ms, n = C.c_double(), C.c_uint64()
    L.cwf_hip_system_timing(h, C.byref(ms), C.byref(n))
    L.cwf_hip_system_set_timing(h, 0)
    kname = (L.cwf_hip_system_keff_kernel(h) or b"").decode()
    out = {"workload": case.name + (" with CWF_LATTICE=0" if mode == "general" else ", PARITY (bit-exact)"),
           "operator": operator_of(kname), "kernel": kname,
           "steps": steps, "pcg_iterations": int(iters), "pcg_iterations_per_sec": iters / el,
           "dof_iterations_per_sec": P.dof_count * iters / el, "ms_per_step": 1e3 * el / steps,
           "keff_avg_launch_ms": ms.value / max(1, n.value)}
    st.close()
    st.system.close()
    return out


def same_kernel(kname: str, profiled: str) -> bool:
    """rocprofv3 names a kernel 'ns::name<args>' (optionally with its parameter list): the base name and the
    template arguments must both match, so 'k_keff_tiles' is not taken for 'k_keff_tiles_pipe<...>'."""
    def split(k):
        k = k.replace("(anonymous namespace)::", "").split("(")[0].replace(" ", "")
        base, _, args = k.partition("<")
        args = ",".join(a.split("::")[-1] for a in args.rstrip(">").split(","))  # template args less namespaces
        return base.split("::")[-1], args

    return split(kname) == split(profiled)


def stream_copy_gbs(L, device, nbytes=2 << 30, reps=20):
    """STREAM-like 16-B-lane device copy measured on this GPU: read + write bytes / time."""
    import ctypes as C

    g = C.c_double()
    return g.value if L.cwf_hip_bandwidth_probe(device, nbytes, reps, C.byref(g)) == 0 else None


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import torch  # loaded before libcwf_hip.so so both share one HIP runtime

    # one GPU per rank; ranks beyond the visible GPUs share them round-robin (a 1-GPU rehearsal of the
    # multi-rank path; device_count() does not initialise the GPU)
    ngpu = max(1, torch.cuda.device_count())
    if world > 1:
        torch.cuda.set_device(local_rank % ngpu)

    dist = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("gloo", init_method="env://")  # bookkeeping only; the data path is PEER / RCCL
    import numpy as np

    from cwf import _lib, pcg, scenarios, shard
    from cwf.stepper import Stepper

    def barrier():
        if dist is not None:
            dist.barrier()

    device = local_rank % ngpu if world > 1 else 0
    mode = _lib.MODE_FAST if args.mode == "fast" else _lib.MODE_PARITY
    comm = None
    unstructured = bool(scenarios.meshgen.CONFIGS[args.config].get("jitter"))
    strong = args.scaling == "strong" or unstructured
    load_pattern = None  # (base, pattern) f64 in the stepper's node order, for a curve-scaled (harmonic) load
    halo_nodes = 0
    if world == 1:
        case = scenarios.config_case(args.config, max_iterations=args.max_iterations, element=args.element)
        P = case.packing
        sK, sM = case.scalars()
        stepper = Stepper(P, case.materials, case.rayleigh, case.cfg.solver, case.cfg.time, mode=mode,
                          device=device)
        owned_dofs, local_nodes, local_tets = P.dof_count, P.node_count, P.element_count
        if case.load_curve is not None:
            load_pattern = case.load_pattern()
    else:
        if mode != _lib.MODE_FAST:
            raise SystemExit("the multi-GPU bench runs the FAST path (the bit-exact sharded PARITY solve is "
                             "the parity gate in tests/test_gpu_shard.py)")
        if unstructured:  # C4: the whole mesh, RCB node partition, renumbered part after part
            if args.element != "tet4":
                raise SystemExit("the unstructured configs are tet4 meshes")
            case, node_global, begin = scenarios.rcb_case(args.config, world, max_iterations=args.max_iterations)
        else:
            case, node_global, begin = scenarios.slab_case(args.config, world, rank,
                                                           max_iterations=args.max_iterations, strong=strong,
                                                           element=args.element)
        P = case.packing
        sK, sM = case.scalars()
        src = pcg.MatrixFreeSystem.from_packing(P, case.materials, sK, sM, mode=mode)  # host arrays only
        sh = shard.build_shard(src, begin, rank, node_global)
        system = sh.system(case.materials, 1.0, 0.0, device=device)
        comm_kind = args.comm
        if comm_kind in ("peer", "auto"):  # device-initiated stores into IPC-mapped mailboxes (peer.hip)
            err = None
            try:
                comm = shard.Comm.peer(world, rank, device)
                comm.attach(system, sh)
            except Exception as e:  # noqa: BLE001 - reported, and agreed on below
                err = e
            handles = [None] * world
            dist.all_gather_object(handles, None if err else comm.handle())
            trial = None
            if err is None and all(hd is not None for hd in handles):
                try:
                    comm.connect(handles)
                    shard.Comm.time_exchange(system, 8)  # a peer that never arrives fails here (bounded wait)
                    # a short trial solve through the schedule the solves will run (on structured slabs the fused
                    # iteration with its exchange inside the launches): every rank folds the same gathered totals,
                    # so every rank must report the same finite residual, bit for bit
                    res = pcg.solve_pcg(system, np.ones(3 * sh.local_nodes, np.float32), pcg.PcgSettings(12, 1e-30),
                                        pcg.PcgVectors(np.zeros(3 * sh.local_nodes, np.float32), None))
                    if not res.has_value():
                        raise RuntimeError(f"trial solve: {res.error().message}")
                    trial = (int(res.value().iterations), float(res.value().residual_norm),
                             int(_lib.load().cwf_hip_system_exchange_schedule(system.handle())))
                    if not np.isfinite(trial[1]):
                        raise RuntimeError("trial solve: non-finite residual")
                except Exception as e:  # noqa: BLE001
                    err = e
            ok = [None] * world
            dist.all_gather_object(ok, (err is None and all(hd is not None for hd in handles), trial))
            if rank == 0 and all(o[0] for o in ok):
                print(f"# --comm auto: PEER trial solve on every rank: {ok[0][1]}", file=sys.stderr)
            if not all(o[0] for o in ok) or len({o[1] for o in ok}) != 1:
                if err is None:
                    err = RuntimeError(f"trial solves differ across ranks: {[o[1] for o in ok]}")
                if comm_kind == "peer":
                    raise SystemExit(f"rank {rank}: PEER communicator unavailable: {err}")
                if rank == 0:
                    print(f"# --comm auto: PEER unavailable on some rank ({err}); using RCCL", file=sys.stderr)
                if comm is not None:
                    comm.close()
                comm = None
                system.close()
                system = sh.system(case.materials, 1.0, 0.0, device=device)
                comm_kind = "rccl"
            else:
                comm_kind = "peer"
        if comm_kind == "rccl":
            uid = [shard.Comm.unique_id() if rank == 0 else None]
            dist.broadcast_object_list(uid, src=0)
            comm = shard.Comm.rccl(world, rank, uid[0], device)
            comm.attach(system, sh)
        args.comm = comm_kind

        class _LocalPacking:  # the Stepper's view of the shard: local node order, local vectors
            external_force = sh.local_dofs(P.external_force)
            bc_value = sh.local_dofs(P.bc_value)
            dof_count = 3 * sh.local_nodes
            node_count = sh.local_nodes

        stepper = Stepper(_LocalPacking, case.materials, case.rayleigh, case.cfg.solver, case.cfg.time, mode=mode,
                          device=device, system=system)
        owned_dofs, local_nodes, local_tets = 3 * sh.owned_nodes, sh.local_nodes, sh.local_elements
        halo_nodes = sh.local_nodes - sh.owned_nodes
        if case.load_curve is not None:
            base, pattern = case.load_pattern()
            load_pattern = (sh.local_dofs(base), sh.local_dofs(pattern))
        del src
    if load_pattern is not None:  # the harmonic tip load (C4), rewritten on the device before every step
        stepper.set_load_pattern(*load_pattern)

    def step(t):
        if load_pattern is not None:
            stepper.set_load_scale(case.load_scale(t))
        return stepper.step(t).value()

    L = _lib.load()
    h = stepper.system.handle()
    t_sim = 0.0
    for w in range(args.warmup):
        step(t_sim)
        t_sim += case.cfg.time.initial_dt
    import ctypes as C

    L.cwf_hip_system_set_timing(h, args.keff_sample)
    torch.cuda.synchronize()
    barrier()
    total_iters = 0
    steps_converged = 0
    t0 = time.perf_counter()
    for k in range(args.steps):
        tel = step(t_sim)
        total_iters += tel.pcg.iterations
        steps_converged += bool(tel.pcg.converged)
        t_sim += case.cfg.time.initial_dt
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    keff_ms, keff_n = C.c_double(), C.c_uint64()
    L.cwf_hip_system_timing(h, C.byref(keff_ms), C.byref(keff_n))
    L.cwf_hip_system_set_timing(h, 0)
    D = owned_dofs
    local = np.array([elapsed, D * total_iters, total_iters, D], np.float64)
    # the PCG schedule the ranks agreed on (cwf_hip_system_exchange_schedule): 0 two kernels + two exchange steps,
    # 1 fused + one exchange step, 2 fused with the exchange inside the launch (PEER), 3 the resident solve (PEER
    # slab shards: one launch per solve)
    sched = int(L.cwf_hip_system_exchange_schedule(h)) if world > 1 else None
    per_rank = [{"owned_dofs": int(D), "local_tets": int(local_tets), "halo_nodes": int(halo_nodes),
                 "halo_bytes_per_exchange": 12 * int(halo_nodes), "seconds": elapsed, "schedule": sched}]
    if dist is not None:
        gathered = [None] * world
        dist.all_gather_object(gathered, per_rank[0])
        per_rank = gathered
        t = torch.from_numpy(local.copy())
        tmax = t.clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        elapsed = float(tmax[0])
        dof_iters, iters_sum, dofs_sum = float(t[1]), float(t[2]), float(t[3])
    else:
        dof_iters, iters_sum, dofs_sum = local[1], local[2], local[3]
    avg_keff_ms = keff_ms.value / max(1, keff_n.value)
    # algorithmic bytes of one K_eff launch: the handle's own layout, every array the
    # kernel touches counted once (it reads less than the reference layout's 32 B/node + 72 B/tet,
    # which is reported beside it as the layout-independent comparator)
    lay_b, ref_b = C.c_uint64(), C.c_uint64()
    L.cwf_hip_system_keff_traffic(h, C.byref(lay_b), C.byref(ref_b))
    alg_bytes, ref_bytes = float(lay_b.value), float(ref_b.value)
    achieved = alg_bytes / (avg_keff_ms * 1e-3) / 1e9 if keff_n.value else None
    ref_equiv = ref_bytes / (avg_keff_ms * 1e-3) / 1e9 if keff_n.value else None
    kname = (L.cwf_hip_system_keff_kernel(h) or b"").decode()
    src_hash = (L.cwf_hip_system_keff_source_hash(h) or b"").decode()
    traffic, traffic_src = None, None
    tpath = args.traffic
    if tpath == "auto":
        import glob

        tag = f"{args.config}_{args.mode}" + ("_hex8" if args.element == "hex8" else "")
        cands = glob.glob(os.path.join(ROOT, "profiles", f"r*_{tag}_pmc.json"))
    else:
        cands = [tpath] if tpath and os.path.exists(tpath) else []
    if world == 1:
        # only a profile of the same kernel built from the same sources counts: the newest such
        traffic, traffic_src = pmc_traffic(cands, kname, src_hash)
    result = None
    stepper.close()
    stepper.system.close()
    hbm = hbm_general = None
    if (rank == 0 and world == 1 and not args.no_hbm_roofline and args.mode == "fast" and args.element == "tet4"
            and args.config != "c3"):
        hbm = hbm_roofline(L, device)
        if not args.no_general_roofline:
            hbm_general = hbm_roofline(L, device, general=True)
    general = None
    if (rank == 0 and world == 1 and not args.no_general and args.mode == "fast" and args.element == "tet4"
            and operator_of(kname).startswith("structured")):
        general = side_line(L, device, args.config, min(args.steps, 5))
    parity = None
    if (rank == 0 and world == 1 and not args.no_parity and args.mode == "fast" and args.element == "tet4"
            and args.config in ("c1", "c2")):
        parity = side_line(L, device, args.config, min(args.steps, 3), mode="parity")
    copy_gbs = stream_copy_gbs(L, device) if rank == 0 else None
    for rl in (hbm, hbm_general):
        if rl and copy_gbs:
            rl["frac_of_measured_copy"] = rl["achieved"] / copy_gbs
    if rank == 0:
        cpu = None
        if not args.no_cpu_baseline and world == 1 and args.element == "tet4":  # rank 0 at N=1 only
            cpu = cpu_baseline(case, sK, sM, args.cpu_iterations)
        result = {
            "metric": "PCG DOF-iterations/sec per Newmark step (PCG-it/s x DOFs); DOF-updates/s and "
                      "K_eff HBM GB/s vs roofline reported alongside",
            "value": dof_iters / elapsed,
            "unit": "DOF-it/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * elapsed / args.steps,
            "higher_is_better": True,
            "scaling": "strong" if (strong and world > 1) or args.scaling == "strong" else "weak",
            "vs_baseline": None,
            # FAST: fp32 element / stencil arithmetic, the block-Jacobi inverse applied from a 16-B record of fp16 row
            # scales and correlations (blockinv_pack.hpp), fp64 dot reductions (configs[4]'s mixed path); PARITY: the
            # reference's fp64 element math on fp32 data, bit-exact
            "dtype": "f32 SpMV, fp16-packed block-Jacobi, f64 reductions" if args.mode == "fast" else "f64",
            "data": ("synthetic (native hex8 block, gravity + tip load)" if args.element == "hex8" else
                     "synthetic (jittered + permuted hex block -> Kuhn tets, gravity + harmonic tip load "
                     "F0 sin(2 pi 5 t) from a 64-point curve, rewritten on the device every step)"
                     if load_pattern is not None else
                     "synthetic (structured hex block -> Kuhn tets, gravity + tip load)"),
            "operator": operator_of(kname),
            "config": {"workload": case.name, "nodes_per_gpu": local_nodes,
                       ("hexes_per_gpu" if args.element == "hex8" else "tets_per_gpu"): local_tets,
                       "dofs": int(dofs_sum), "mode": args.mode,
                       "parallelism": (f"{'RCB' if unstructured else 'slab'} node-range shards x{world} "
                                       f"({'PEER mailbox' if args.comm == 'peer' else 'RCCL'} halo + all-gather, "
                                       f"{'strong' if strong else 'weak'} scaling)")
                       if world > 1 else "single"},
            "ranks": per_rank if world > 1 else None,
            "pcg_iterations": int(iters_sum),
            # steps whose PCG met the tolerance (C5's slender slab runs block-Jacobi PCG into max_iterations:
            # its DOF-updates/s then times capped, unconverged steps; PCG-it/s is the meaningful figure there)
            "steps_converged": steps_converged,
            "pcg_iterations_per_sec": iters_sum / world / elapsed,
            "dof_updates_per_sec": dofs_sum * args.steps / elapsed,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": (achieved / HBM_PEAK_GBS) if achieved else None, "traffic": traffic,
                         "traffic_source": traffic_src,
                         "kernel": kname, "kernel_source_hash": src_hash,
                         "avg_launch_ms": avg_keff_ms, "launches": int(keff_n.value),
                         "algorithmic_bytes_per_launch": alg_bytes,
                         "reference_layout_bytes_per_launch": ref_bytes,
                         "reference_layout_equiv_gbs": ref_equiv,
                         "measured_copy_gbs": copy_gbs,
                         "frac_of_measured_copy": (achieved / copy_gbs) if achieved and copy_gbs else None},
            "cpu_baseline": cpu,
            "roofline_hbm": hbm,
            # the unstructured-mesh SpMV (fan-group tiles, what C4 and any non-lattice mesh run) on the same C3 block
            "roofline_general": hbm_general,
            # the same workload on the general operator (fan-group tiles), timed after the headline's region
            "general": general,
            # the bit-exact PARITY path on the same workload (the rate behind the 1e-10 residual target)
            "parity": parity,
        }
        if args.mode == "parity" and keff_n.value:
            # PARITY's roofline is priced against the REFERENCE layout's compulsory bytes (72 B per tet + 32 B per
            # node): the node-tile kernel's own compulsory bytes (the 64-B record, volume and incidence
            # tiles per tet, x, y, mass, mask and CSR offsets per node) are reported beside it
            result["roofline"]["layout_bytes_per_launch"] = alg_bytes
            result["roofline"]["layout_frac"] = result["roofline"]["frac"]
            result["roofline"]["achieved"] = ref_equiv
            result["roofline"]["frac"] = ref_equiv / HBM_PEAK_GBS
            result["roofline"]["algorithmic_bytes_per_launch"] = ref_bytes
            result["roofline"]["bytes_basis"] = "reference layout (72 B/tet + 32 B/node)"
            # each tet's fp64 element math once: strain 72, stress 24 (isotropic D), V s_K 1, 4 corner forces x
            # (18 + 3 scale) = 84, and the node fold adds 3 per incidence (12 per tet): 193 fp64 flops per tet
            # (kernels_parity.hip; halo tets are computed again by the neighbouring tile, not counted). The fp64
            # vector peak is AMD's MI355X spec (78.6 TFLOP/s, not in the microarch guide).
            flops = 193.0 * local_tets
            result["roofline_fp64"] = {"bound": "valu_fp64", "achieved": flops / (avg_keff_ms * 1e-3) / 1e12,
                                       "peak": 78.6, "unit": "TFLOP/s",
                                       "frac": flops / (avg_keff_ms * 1e-3) / 1e12 / 78.6,
                                       "flops_per_launch": flops, "kernel": kname}
        print(json.dumps(result), flush=True)
    if comm is not None:
        comm.close()
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
