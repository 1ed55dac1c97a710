#!/bin/bash
# C5 as native hex8 (the BASELINE names a hex8 slab): one Newmark step, lattice path
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd $R
O=gpurun_out/round; mkdir -p $O
timeout -k 10 600 python -u bench.py --config c5 --element hex8 --steps 2 --warmup 1 --no-cpu-baseline --no-hbm-roofline \
  > $O/r03aj_bench_c5_hex8_fast.log 2>&1 && grep '^{"metric"' $O/r03aj_bench_c5_hex8_fast.log > $O/r03aj_bench_c5_hex8_fast.json &&
python3 -c "
import json; d=json.load(open('$O/r03aj_bench_c5_hex8_fast.json')); r=d['roofline']
print(round(d['value']/1e9,2), 'G DOF-it/s', round(d['pcg_iterations_per_sec']), 'it/s', round(d['ms_per_step'],1), 'ms/step keff', round(r['avg_launch_ms']*1e3,2), 'us', r.get('kernel'), 'conv', d['steps_converged'], d.get('pcg_iterations'))"
