#!/usr/bin/env python3
"""Per-ablation averages of PMC counters from a rocprofv3 --pmc run over tools/ablate.py.
ablate.py runs 120 launches (20 + 100) of the PCG-mode tiles kernel per ablation bit set, in order;
this groups the tiles-kernel dispatches by that order. usage: abl_pmc.py DIR --bits 0 64 ..."""
import argparse
import collections
import csv
import glob
import os

ap = argparse.ArgumentParser()
ap.add_argument("dir")
ap.add_argument("--bits", type=int, nargs="+", required=True)
ap.add_argument("--kernel", default="_pipe")
ap.add_argument("--per", type=int, default=120)
a = ap.parse_args()
rows = collections.defaultdict(dict)
for f in glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if a.kernel in r["Kernel_Name"]:
            rows[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
ids = sorted(rows)
names = sorted({c for d in rows.values() for c in d})
print("bits   " + " ".join(f"{n:>22s}" for n in names))
for i, b in enumerate(a.bits):
    chunk = ids[i * a.per + 20:(i + 1) * a.per]  # the 100 timed launches
    if not chunk:
        break
    avg = {n: sum(rows[d].get(n, 0.0) for d in chunk) / len(chunk) for n in names}
    print(f"{b:5d}  " + " ".join(f"{avg[n]:22.0f}" for n in names))
