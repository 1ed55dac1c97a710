#!/usr/bin/env python3
"""Per-iteration time of a FAST solve on one structured block, one handle (the compute a slab shard of that size runs
per PCG iteration, without its exchange): fixed iterations (tol 1e-30), the second solve timed (wall clock, host
read-backs included): the resident one-launch solve (the default where the block fits on chip, resident.hip), the fused
launch-per-iteration schedule (CWF_FUSED=1) and the two-kernel loop (CWF_FUSED=0).

usage: python tools/block_iter_time.py NX NY NZ [ITERATIONS]   (BLK_ELEMENT=hex8: the block as native hex8 cells)"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "civiwave-fem_amd")]


def main():
    a = sys.argv[1:]
    nx, ny, nz = (int(v) for v in a[:3])
    its = int(a[3]) if len(a) > 3 else 300
    import numpy as np

    from cwf import _lib, pcg, scenarios

    element = os.environ.get("BLK_ELEMENT", "tet4")
    case = scenarios.block_case(nx, ny, nz, h=0.1, tol=1e-30, max_iterations=its, element=element)
    rhs = case.static_rhs()
    # BLK_SCHEDULES=resident,1,0 (a comma list) limits the schedules (same-box A/B of library builds: CWF_LIB_PATH)
    for fused in os.environ.get("BLK_SCHEDULES", "resident,1,0").split(","):
        if fused == "resident":
            os.environ.pop("CWF_FUSED", None)
        else:
            os.environ["CWF_FUSED"] = fused
        s = pcg.MatrixFreeSystem.from_packing(case.packing, case.materials, *case.scalars(), mode=_lib.MODE_FAST)
        import ctypes as C

        L = _lib.load()
        reps = int(os.environ.get("BLK_REPEAT", "1"))  # timed solves after the first (each printed when > 1)
        for k in range(1 + reps):
            x = np.zeros_like(rhs)
            L.cwf_hip_system_set_timing(s.handle(), 1)  # the resident solve: its one launch, hipEvent-timed
            t0 = time.perf_counter()
            t = pcg.solve_pcg(s, rhs, pcg.PcgSettings(its, 1e-30), pcg.PcgVectors(x, None)).value()
            el = time.perf_counter() - t0
            ms, n = C.c_double(), C.c_uint64()
            L.cwf_hip_system_timing(s.handle(), C.byref(ms), C.byref(n))
            L.cwf_hip_system_set_timing(s.handle(), 0)
            kin = ms.value * 1e3 / max(n.value, 1)
            if reps > 1 and k:
                print(f"  solve {k}: {el / max(t.iterations, 1) * 1e6:.2f} us per iteration (in-kernel {kin:.2f})",
                      flush=True)
        kern = (_lib.load().cwf_hip_system_keff_kernel(s.handle()) or b"").decode()
        print(f"{nx}x{ny}x{nz} {element} ({3 * nx * ny * nz / 1e6:.2f}M DOF) { {'resident': 'resident', '1': 'fused'}.get(fused, 'two kernels')}: "
              f"{t.iterations} iterations, {el / max(t.iterations, 1) * 1e6:.2f} us per iteration, in-kernel {kin:.2f} "
              f"({kern})", flush=True)
        s.close()


if __name__ == "__main__":
    main()
