#!/bin/bash
# round 3 evidence A: the bench line of every config (C2 default incl. CPU baseline + live C3 roofline, C3, C4, C5,
# hex8 C2/C3, PARITY C2) -> gpurun_out/round/${TAG}_bench_*.json
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r03n}
O=gpurun_out/round
mkdir -p $O
b() {
  local name=$1; shift
  timeout -k 10 400 python -u bench.py "$@" > $O/${TAG}_bench_${name}.log 2>&1 &&
  grep '^{"metric"' $O/${TAG}_bench_${name}.log > $O/${TAG}_bench_${name}.json &&
  python3 -c "
import json; d=json.load(open('$O/${TAG}_bench_${name}.json')); r=d['roofline']
print('$name', round(d['value']/1e9,2), 'G DOF-it/s', round(d['pcg_iterations_per_sec']), 'it/s', round(d['ms_per_step'],2), 'ms/step', 'keff', round(r['avg_launch_ms']*1e3,2), 'us frac', round(r['frac'],3), 'conv', d['steps_converged'], '/', d['steps'])"
}
b c2_fast &&
b c3_fast --config c3 --steps 3 --warmup 1 --no-cpu-baseline &&
b c4_fast --config c4 --steps 3 --warmup 1 --no-cpu-baseline --no-hbm-roofline &&
b c2_hex8_fast --element hex8 --no-cpu-baseline --no-hbm-roofline &&
b c3_hex8_fast --element hex8 --config c3 --steps 3 --warmup 1 --no-cpu-baseline &&
b c2_parity --mode parity --steps 3 --warmup 1 --no-cpu-baseline &&
b c5_fast --config c5 --steps 1 --warmup 0 --no-cpu-baseline --no-hbm-roofline
