#!/usr/bin/env python3
"""Summarise the per-workgroup stamps of one fused lattice launch (CWF_FUSED_TRACE, ablation build; lattice_fused.inc
`stamp`). Phases per workgroup (s_memrealtime, 100 MHz = 10 ns ticks): dispatch offset from the launch's first
workgroup, t1 - t0 prologue (plane loads issued, share fold), t2 - t1 the first two planes formed (bricks), t3 - t2
the march (bricks) or the shell rows, t4 - t3 the block reduction and the share store; and how many workgroups each
CU ran (HW_ID cu/sh/se, XCC_ID).

usage: python tools/fused_trace.py TRACE [LAUNCH_INDEX]"""
import sys
from collections import Counter

import numpy as np


def launches(path):
    cur = None
    for line in open(path):
        if line.startswith("#"):
            if cur:
                yield cur
            cur = {"hdr": line.strip(), "rows": []}
        elif line.strip() and cur is not None:
            cur["rows"].append([int(v) for v in line.split()])
    if cur:
        yield cur


def main():
    ls = list(launches(sys.argv[1]))
    pick = int(sys.argv[2]) if len(sys.argv) > 2 else -1
    L = ls[pick]
    a = np.array(L["rows"], np.int64)
    wg, kind, hw, xcc = a[:, 0], a[:, 1], a[:, 2], a[:, 3]
    t = a[:, 4:9].astype(np.float64) * 0.01  # us
    t -= t[:, 0].min()
    shell = (kind & 1) == 1
    t[shell, 2] = t[shell, 1]  # a shell workgroup forms no brick planes (its stamp 2 is stale)
    print(f"{L['hdr']}: {len(a)} workgroups ({shell.sum()} shell), launch span {t[:, 4].max():.2f} us")
    names = ["start", "prologue", "first planes", "march/rows", "reduce+store", "total"]
    for lab, m in (("bricks", ~shell), ("shell", shell)):
        if not m.any():
            continue
        d = np.stack([t[m, 0], t[m, 1] - t[m, 0], t[m, 2] - t[m, 1], t[m, 3] - t[m, 2], t[m, 4] - t[m, 3],
                      t[m, 4] - t[m, 0]], 1)
        print(f"  {lab:6s} " + "  ".join(f"{n} {np.median(d[:, i]):.2f}/{d[:, i].max():.2f}" for i, n in
                                           enumerate(names)) + "  (median/max us)")
    if a.shape[1] >= 15:  # the first step's phases (stamps 8 .. 13): write k+1, write k+2, barrier, loads, row k, row k+1
        st = a[:, 9:15].astype(np.float64) * 0.01
        ph = np.diff(np.concatenate([t[:, 2:3] + 0 * st[:, :1] + (a[:, 6:7] * 0.01 - a[:, 6:7] * 0.01), st], 1), axis=1)
        st0 = a[:, 6] * 0.01  # t2 (absolute, before the origin shift)
        ph = np.diff(np.concatenate([st0[:, None], st], 1), axis=1)
        m = ~shell
        names2 = ["write k+1", "write k+2", "barrier", "issue loads", "row k", "row k+1"]
        print("  first step (bricks): " + "  ".join(f"{n} {np.median(ph[m, i]):.2f}/{ph[m, i].max():.2f}"
                                                   for i, n in enumerate(names2)) + "  (median/max us)")
    end = t[:, 4]
    order = np.argsort(end)[::-1][:8]
    print("  last to finish: " + ", ".join(f"wg {wg[i]} ({'shell' if shell[i] else 'brick'}, start {t[i, 0]:.2f},"
                                            f" end {end[i]:.2f})" for i in order[:5]))
    cu = ((xcc & 0xF) << 16) | (((hw >> 13) & 7) << 8) | (((hw >> 12) & 1) << 4) | ((hw >> 8) & 0xF)
    per = Counter(cu.tolist())
    hist = Counter(per.values())
    print(f"  CUs used {len(per)}; workgroups per CU: " + ", ".join(f"{k}: {v} CUs" for k, v in sorted(hist.items())))
    # workgroups sharing a CU with another: their total time vs alone
    share = np.array([per[c] for c in cu.tolist()])
    for k in sorted(set(share.tolist())):
        m = (share == k) & ~shell
        if m.any():
            print(f"  bricks on CUs running {k} workgroups: total median {np.median(t[m, 4] - t[m, 0]):.2f} us, "
                  f"max {np.max(t[m, 4] - t[m, 0]):.2f}")


if __name__ == "__main__":
    main()
