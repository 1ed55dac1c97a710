#!/usr/bin/env python3
"""Summarise the per-workgroup phase stamps of one resident-solve phase (CWF_RESIDENT_TRACE, resident.hip `stamp`):
per workgroup s_memrealtime (100 MHz) at 0 the phase's start (its polls begin), 1 every polled granule carries the
previous phase's tag, 2 the shares folded and the scalars decided, 3 the own and halo p formed into the image, 4 the
rows done, 5 the dots reduced, 6 the shares' granules stored (the phase's end). Prints the median / max of each span and when the last
workgroup arrived relative to the first one's release.

usage: python tools/resident_trace.py TRACE [INDEX]"""
import sys

import numpy as np


def blocks(path):
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
    bs = list(blocks(sys.argv[1]))
    B = bs[int(sys.argv[2]) if len(sys.argv) > 2 else -1]
    a = np.array(B["rows"], np.int64)
    t = a[:, 1:8].astype(np.float64) * 0.01  # us
    fold = (a[:, 8] - a[:, 2]).astype(np.float64) * 0.01 if a.shape[1] > 8 else None  # stamp 7: the fold done
    t -= t[:, 0].min()
    names = ["poll", "fold+decide", "form", "rows", "reduce", "shares"]
    print(f"{B['hdr']}: {len(a)} workgroups")
    for i, n in enumerate(names):
        d = t[:, i + 1] - t[:, i]
        print(f"  {n:12s} median {np.median(d):6.2f}  max {d.max():6.2f} us")
    if fold is not None and np.all(a[:, 8] > 0):
        print(f"  (fold alone median {np.median(fold):.2f} max {fold.max():.2f} us; decide the rest)")
    print(f"  phase start spread {t[:, 0].max() - t[:, 0].min():.2f} us, release (wait done) spread "
          f"{t[:, 1].max() - t[:, 1].min():.2f} us, last end {t[:, 6].max():.2f} us after the first start, "
          f"compute (release -> end) median {np.median(t[:, 6] - t[:, 1]):.2f} max {np.max(t[:, 6] - t[:, 1]):.2f}")
    # per box: the form + rows span by the number of block faces the box touches (box b = (bx, by, bz), x fastest)
    hdr = B["hdr"].split("boxes ")
    if len(hdr) > 1:
        gx, gy, gz = (int(v) for v in hdr[1].split("x"))
        b = a[:, 0]
        pos = np.stack([b % gx, (b // gx) % gy, b // (gx * gy)], 1)
        faces = ((pos == 0) | (pos == np.array([gx, gy, gz]) - 1)).sum(1)
        work = t[:, 4] - t[:, 2]
        for f in sorted(set(faces.tolist())):
            w = work[faces == f]
            print(f"  boxes on {f} block faces: {len(w):3d}, form + rows median {np.median(w):5.2f} max {w.max():5.2f} us")
        for ax, n in zip("xyz", (gx, gy, gz)):
            print(f"  along {ax}: " + " ".join(f"{np.median(work[pos[:, 'xyz'.index(ax)] == q]):.2f}" for q in range(n)))


if __name__ == "__main__":
    main()
