#!/usr/bin/env python3
"""Per-kernel average durations and the idle gaps between consecutive kernels from a rocprofv3 kernel trace
(kernel_trace.csv). usage: tools/kt_gaps.py DIR [--last N]"""
import argparse
import collections
import csv
import glob
import os
import re

ap = argparse.ArgumentParser()
ap.add_argument("dir")
ap.add_argument("--last", type=int, default=400, help="only the last N dispatches (the timed loop)")
a = ap.parse_args()
rows = []
for f in glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        m = re.search(r"cwf::(?:\(anonymous namespace\)::)?([\w<>, ]+)", r["Kernel_Name"])
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), m.group(1) if m else r["Kernel_Name"][:40]))
rows.sort()
rows = rows[-a.last:]
dur = collections.defaultdict(list)
gap = collections.defaultdict(list)
for i, (s, e, k) in enumerate(rows):
    dur[k].append(e - s)
    if i:
        gap[k].append(s - rows[i - 1][1])
span = rows[-1][1] - rows[0][0]
busy = sum(e - s for s, e, _ in rows)
print(f"{len(rows)} dispatches, span {span / 1e3:.1f} us, busy {busy / 1e3:.1f} us ({100 * busy / span:.1f}%)")
for k in sorted(dur, key=lambda k: -sum(dur[k])):
    d, g = dur[k], gap[k]
    print(f"  {k[:60]:60s} n={len(d):4d} avg {sum(d) / len(d) / 1e3:8.2f} us  gap-before avg {sum(g) / max(1, len(g)) / 1e3:6.2f} us")
