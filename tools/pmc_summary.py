#!/usr/bin/env python3
"""Summarise a tools/profile.sh run: per-kernel average duration (kernel trace) and per-launch HBM
traffic from the separate FETCH_SIZE / WRITE_SIZE PMC passes, corrected as MI355X_MICROARCH.md
prescribes for gfx950: FETCH_SIZE and WRITE_SIZE are KiB; FETCH_SIZE reports half the bytes of a
wide coalesced streaming read, so read bytes = 2 * FETCH_SIZE * 1024 (an upper-bound correction for
kernels whose reads are not all 16-B/lane streams); write bytes = WRITE_SIZE * 1024.

usage: tools/pmc_summary.py gpurun_out/prof_TAG [--kernel SUBSTR] [--json out.json]
"""
import argparse
import collections
import csv
import glob
import json
import os


def per_kernel(path, counter):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        acc[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def norm(k):
    """'cwf::k<1, cwf::LatKuhn>' and 'k<1, LatKuhn>' alike: namespaces off the name and its template arguments."""
    k = k.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0].replace(" ", "")
    base, _, args = k.partition("<")
    return base.split("::")[-1] + "<" + ",".join(x.split("::")[-1] for x in args.rstrip(">").split(",")) + ">"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--kernel", action="append", default=[])
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    stats = {}
    for r in csv.DictReader(open(glob.glob(os.path.join(a.dir, "kt", "*kernel_stats.csv"))[0])):
        stats[r["Name"]] = (int(r["Calls"]), float(r["AverageNs"]), float(r["Percentage"]))
    fetch = per_kernel(glob.glob(os.path.join(a.dir, "fetch", "*counter_collection.csv"))[0], "FETCH_SIZE")
    write = per_kernel(glob.glob(os.path.join(a.dir, "write", "*counter_collection.csv"))[0], "WRITE_SIZE")
    out = {}
    print(f"{'kernel':70s} {'calls':>6s} {'avg_us':>8s} {'%':>6s} {'rd_MB':>8s} {'wr_MB':>8s} {'GB/s':>8s}")
    for name, (calls, avg, pct) in sorted(stats.items(), key=lambda kv: -kv[1][2]):
        f = fetch.get(name)
        w = write.get(name)
        rd = 2 * f * 1024 if f is not None else None
        wr = w * 1024 if w is not None else None
        bw = (rd + wr) / (avg * 1e-9) / 1e9 if rd is not None and wr is not None else None
        short = name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][-70:]
        print(f"{short:70s} {calls:6d} {avg / 1e3:8.2f} {pct:6.2f} "
              f"{(rd or 0) / 1e6:8.2f} {(wr or 0) / 1e6:8.2f} {(bw or 0):8.1f}")
        out[short] = dict(calls=calls, avg_ns=avg, pct=pct, read_bytes=rd, write_bytes=wr,
                          hbm_bytes_per_launch=(rd + wr) if rd is not None and wr is not None else None,
                          hbm_gbs=bw)
    if a.json:
        sel = {k: v for k, v in out.items() if not a.kernel or any(s in k or norm(s) == norm(k) for s in a.kernel)}
        # provenance: the source hash of the profiled kernel as the profiled bench run printed it (bench.py only takes
        # this file's traffic for a library built from the same sources)
        src_hash, bench = None, None
        for log in sorted(glob.glob(os.path.join(a.dir, "bench_*.log"))):
            for line in open(log, errors="replace"):
                if line.startswith('{"metric"'):
                    bench = bench or json.loads(line)
                    src_hash = src_hash or bench["roofline"].get("kernel_source_hash")
        note = ("FETCH_SIZE x2 x1024 + WRITE_SIZE x1024 per launch, summed over the selected kernels "
                "(MI355X_MICROARCH.md HBM section)")
        # the resident solve is ONE launch per PCG solve: its per-launch figures are per solve. Profiled with
        # --warmup 0 every launch is a timed Newmark step's, so iterations per launch = the line's PCG iterations /
        # steps, and the figures bench.py prices per iteration are the per-launch ones divided by that
        for k, v in sel.items():
            if norm(k).startswith("k_pcg_resident") and bench and bench.get("warmup") == 0 and bench.get("steps"):
                ipl = bench["pcg_iterations"] / bench["steps"]
                v["iterations_per_launch"] = ipl
                v["avg_ns_per_iteration"] = v["avg_ns"] / ipl
                if v["hbm_bytes_per_launch"] is not None:
                    v["hbm_bytes_per_launch"] /= ipl
                    v["read_bytes"] /= ipl
                    v["write_bytes"] /= ipl
                note += "; k_pcg_resident: per PCG iteration (one launch = one solve of iterations_per_launch)"
        total = sum(v["hbm_bytes_per_launch"] or 0 for v in sel.values())
        json.dump(dict(kernels=sel, hbm_bytes_per_launch=total, source_hash=src_hash, note=note), open(a.json, "w"),
                  indent=1)


if __name__ == "__main__":
    main()
