#!/usr/bin/env python3
"""Collapse the per-pass bench JSON lines of `tools/gpu_run.sh ab|ablib` runs into profiles/ab_history.md rows.

usage: python tools/ab_table.py gpurun_out/TAG [...]   (prints one markdown row per A/B name found)"""
import glob
import json
import os
import re
import sys


def load(path):
    with open(path) as fh:
        for line in fh:
            if line.startswith('{"metric"'):
                return json.loads(line)
    return None


def main():
    for d in sys.argv[1:]:
        tag = os.path.basename(os.path.normpath(d))
        runs = {}
        for f in sorted(glob.glob(os.path.join(d, "*_p[0-9].json"))):
            m = re.match(r"(.+)_(new|alt)_p(\d+)\.json$", os.path.basename(f))
            if not m:
                continue
            b = load(f)
            if b:
                runs.setdefault(m.group(1), {"new": [], "alt": []})[m.group(2)].append(b)
        for name, v in sorted(runs.items()):
            def cell(bs):
                return ", ".join(f"{b['pcg_iterations_per_sec']:.0f} ({b['roofline']['avg_launch_ms'] * 1e3:.1f})"
                                 for b in bs)
            kern = sorted({b["roofline"]["kernel"] for b in v["new"] + v["alt"]})
            mean = lambda bs: sum(b["pcg_iterations_per_sec"] for b in bs) / len(bs)
            ch = f"{(mean(v['new']) / mean(v['alt']) - 1) * 100:+.1f}%" if v["new"] and v["alt"] else "-"
            wl = (v["new"] or v["alt"])[0]["config"]["workload"]
            print(f"| {tag}_{name} | {wl} | " + " / ".join(f"`{k}`" for k in kern)
                  + f" | {cell(v['new'])} | {cell(v['alt'])} | {ch} |")


if __name__ == "__main__":
    main()
