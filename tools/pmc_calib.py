#!/usr/bin/env python3
"""Ratio of rocprofv3's per-launch FETCH_SIZE / WRITE_SIZE (KiB) to the known bytes tools/pmc_calib moves.
usage: tools/pmc_calib.py DIR (with DIR/fetch, DIR/write from rocprofv3 --pmc passes, DIR/known.json)"""
import collections
import csv
import glob
import json
import os
import sys

d = sys.argv[1]
known = json.loads(open(os.path.join(d, "known.json")).read().strip().splitlines()[-1])


def per_kernel(sub, counter):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(glob.glob(os.path.join(d, sub, "*counter_collection.csv"))[0])):
        if r["Counter_Name"] == counter:
            acc[r["Kernel_Name"].split("(")[0].replace("void ", "")].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


fetch, write = per_kernel("fetch", "FETCH_SIZE"), per_kernel("write", "WRITE_SIZE")
out = {}
for k in ("rd16", "rd12", "rd12g", "rd12p", "wr12", "wr16"):
    f, w = fetch.get(k, 0.0) * 1024, write.get(k, 0.0) * 1024
    b = known[k]
    out[k] = {"known_bytes": b, "fetch_bytes": f, "write_bytes": w, "fetch_over_known": f / b,
              "write_over_known": w / b}
    if k == "rd12g":
        out[k]["fetch_over_known_incl_perm"] = f / (b + known["rd12g_perm"])
    if k == "rd12p":
        out[k]["fetch_over_unique"] = f / known["rd12p_unique"]
    print(f"{k:6s} known {b / 1e6:9.1f} MB  FETCH {f / 1e6:9.1f} MB ({f / b:5.3f} x)  WRITE {w / 1e6:9.1f} MB "
          f"({w / b:5.3f} x)")
json.dump(out, open(os.path.join(d, "calib.json"), "w"), indent=1)
