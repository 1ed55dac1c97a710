#!/usr/bin/env python3
"""Per-kernel averages of every counter in a tools/sq_profile.sh run (all passes merged).
usage: tools/sq_summary.py gpurun_out/sq_TAG [--kernel SUBSTR ...]"""
import argparse
import collections
import csv
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import norm  # noqa: E402  'ns::k<a, ns::B>' and 'k<a, B>' alike

ap = argparse.ArgumentParser()
ap.add_argument("dir")
ap.add_argument("--kernel", action="append", default=[])
a = ap.parse_args()
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(a.dir, "*", "*counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = norm(r["Kernel_Name"])
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in acc.items():
    if a.kernel and not any(s in k or norm(s) == k for s in a.kernel):
        continue
    print(k)
    avg = {c: sum(v) / len(v) for c, v in cs.items()}
    for c in sorted(avg):
        print(f"   {c:24s} {avg[c]:16.1f}")
    wc = avg.get("SQ_WAVE_CYCLES")
    if wc:
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                  "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VMEM"):
            if c in avg:
                print(f"   {c + ' / WAVE_CYCLES':40s} {avg[c] / wc:6.3f}")
    h, m = avg.get("TCC_HIT_sum"), avg.get("TCC_MISS_sum")
    if h is not None and m:
        print(f"   L2 hit rate {h / (h + m):.3f}")
