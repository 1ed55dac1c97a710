#!/usr/bin/env python3
"""Diagnostic: time the PCG-mode tiles kernel with ablation bits (CWF_TIMED_PCG) on one config.
usage: python tools/ablate.py --config c3 --bits 0 64 128 256 ..."""
import argparse
import ctypes as C
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "civiwave-fem_amd"))


def child(config, bits):
    import numpy as np
    import torch  # noqa: F401
    from cwf import _lib, pcg, scenarios
    case = scenarios.config_case(config)
    P = case.packing
    sK, sM = case.scalars()
    s = pcg.MatrixFreeSystem.from_packing(P, case.materials, sK, sM, mode=_lib.MODE_FAST)
    L = _lib.load()
    h = s.handle()
    D = P.dof_count
    x = torch.tensor(((np.arange(D, dtype=np.uint64) * 2654435761) % 1000).astype(np.float32) / 1000.0,
                     device="cuda")
    y = torch.zeros(D, device="cuda")
    ms = C.c_double()
    out = []
    for b in bits:
        os.environ["CWF_TIMED_PCG"] = str(b)
        L.cwf_hip_keff_timed(h, _lib.ptr(x), _lib.ptr(y), 20, C.byref(ms))
        L.cwf_hip_keff_timed(h, _lib.ptr(x), _lib.ptr(y), 100, C.byref(ms))
        out.append((b, ms.value * 1e3))
    for b, us in out:
        print(f"{config} abl={b:5d}  {us:8.2f} us", flush=True)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--bits", type=int, nargs="+", default=[0, 64, 128, 256, 64 | 128, 64 | 128 | 256])
    a = ap.parse_args()
    child(a.config, a.bits)
