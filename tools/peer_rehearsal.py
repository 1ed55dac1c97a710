#!/usr/bin/env python3
"""Per-iteration time of a sharded FAST solve over the PEER communicator, N processes on ONE GPU (a rehearsal of the
driver's N > 1 flow; the processes share the GPU's CUs, so absolute times are not xGMI figures), in the two fused
schedules: the exchange inside the launches (default) and one k_peer_step launch after each fused launch
(CWF_PEER_FUSED=0). Slab sub-meshes of NX x NY x NZ nodes per rank (the lattice stencil); a fixed iteration count
(tol 1e-30); the second solve is timed (wall clock, one host read-back per batch included).

usage: python tools/peer_rehearsal.py [NX NY NZ] [NRANKS] [ITERATIONS]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "civiwave-fem_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]


def main():
    a = sys.argv[1:]
    shape = tuple(int(v) for v in a[:3]) if len(a) >= 3 else (69, 69, 20)
    nranks = int(a[3]) if len(a) > 3 else 2
    its = int(a[4]) if len(a) > 4 else 400
    import time

    import numpy as np

    from cwf import _lib, pcg, scenarios
    from test_gpu_peer import _run

    # the same total work as one handle (the ranks' slabs stacked along z) in one process: no exchange at all
    case = scenarios.block_case(shape[0], shape[1], shape[2] * nranks, h=0.1, tol=1e-30, max_iterations=its)
    s = pcg.MatrixFreeSystem.from_packing(case.packing, case.materials, *case.scalars(), mode=_lib.MODE_FAST)
    rhs = case.static_rhs()
    for rep in range(2):
        x = np.zeros_like(rhs)
        t0 = time.perf_counter()
        t = pcg.solve_pcg(s, rhs, pcg.PcgSettings(its, 1e-30), pcg.PcgVectors(x, None)).value()
        el = time.perf_counter() - t0
    print(f"{'one handle':14s} block {shape[0]}x{shape[1]}x{shape[2] * nranks}: {t.iterations} iterations, "
          f"{el / max(t.iterations, 1) * 1e6:.2f} us per iteration", flush=True)
    s.close()
    for mode, env in (("in-kernel", {}), ("exchange step", {"CWF_PEER_FUSED": "0"})):
        spec = dict(slab=shape, tol=1e-30, max_iterations=its, timing_steps=200, env=env)
        out = _run(spec, nranks)
        per = [d["solve2_s"] / max(d["telemetry2"][0], 1) * 1e6 for _, d in sorted(out.items())]
        sch = sorted({d["schedule"] for d in out.values()})
        print(f"{mode:14s} slab {shape} x {nranks} ranks, schedule {sch}: {out[0]['telemetry2'][0]} iterations, "
              f"{max(per):.2f} us per iteration (max over ranks; exchange-step latency {out[0]['exchange_us']:.2f} us)",
              flush=True)


if __name__ == "__main__":
    main()
