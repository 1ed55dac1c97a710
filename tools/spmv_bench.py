#!/usr/bin/env python3
"""Quick FAST/PARITY kernel timing on one config: standalone K_eff (apply path) and a fixed-length
PCG solve (tolerance 1e-30 so every iteration runs), with the in-loop hipEvent timing of the
K_eff tiles kernel. Usage: python tools/spmv_bench.py [--config c2] [--mode fast] [--iters 200]"""
import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "civiwave-fem_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (before libcwf_hip.so: one HIP runtime per process)

from cwf import _lib, pcg, scenarios  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--mode", default="fast")
    ap.add_argument("--iters", type=int, default=200)
    a = ap.parse_args()
    t0 = time.time()
    case = scenarios.config_case(a.config)
    t1 = time.time()
    P = case.packing
    mode = _lib.MODE_FAST if a.mode == "fast" else _lib.MODE_PARITY
    sK, sM = case.scalars()
    s = pcg.MatrixFreeSystem.from_packing(P, case.materials, sK, sM, mode=mode)
    L = _lib.load()
    h = s.handle()
    t2 = time.time()
    D = P.dof_count
    xin = torch.tensor(((np.arange(D, dtype=np.uint64) * 2654435761) % 1000).astype(np.float32) / 1000.0,
                       device="cuda")
    y = torch.zeros(D, device="cuda")
    ms = C.c_double()
    L.cwf_hip_keff_timed(h, _lib.ptr(xin), _lib.ptr(y), 50, C.byref(ms))
    L.cwf_hip_keff_timed(h, _lib.ptr(xin), _lib.ptr(y), 200, C.byref(ms))
    apply_ms = ms.value
    rhs = torch.from_numpy(case.static_rhs()).cuda()
    x = torch.zeros(D, device="cuda")
    r = torch.zeros(D, device="cuda")
    L.cwf_hip_system_set_timing(h, 1)
    torch.cuda.synchronize()
    t3 = time.perf_counter()
    tel = pcg.solve_pcg(s, rhs, pcg.PcgSettings(a.iters, 1e-30), pcg.PcgVectors(x, r)).value()
    torch.cuda.synchronize()
    t4 = time.perf_counter()
    kms, kn = C.c_double(), C.c_uint64()
    L.cwf_hip_system_timing(h, C.byref(kms), C.byref(kn))
    alg = 72.0 * P.element_count + 24.0 * P.node_count
    out = dict(config=a.config, mode=a.mode, nodes=P.node_count, tets=P.element_count, setup_s=round(t2 - t1, 2),
               mesh_s=round(t1 - t0, 2), apply_keff_us=apply_ms * 1e3, pcg_iterations=tel.iterations,
               solve_ms=(t4 - t3) * 1e3, us_per_iteration=(t4 - t3) * 1e6 / max(1, tel.iterations),
               pcg_it_per_s=tel.iterations / (t4 - t3), keff_pcg_us=kms.value * 1e3 / max(1, kn.value),
               keff_launches=kn.value, alg_bytes=alg,
               keff_alg_GBs=alg / (kms.value * 1e-3 / max(1, kn.value)) / 1e9 if kn.value else None)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
