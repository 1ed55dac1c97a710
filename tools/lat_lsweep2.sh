#!/bin/bash
# lattice planes per brick on C5 and C3 hex8 (one pass; C5 one Newmark step)
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd $R
O=gpurun_out/lsweep; mkdir -p $O
b() {
  local name=$1; shift
  timeout -k 10 400 python -u bench.py "$@" --no-cpu-baseline --no-hbm-roofline > $O/${name}.log 2>&1 &&
  python3 -c "
import json; d=[json.loads(l) for l in open('$O/${name}.log') if l.startswith('{\"metric\"')][0]; r=d['roofline']
print('$name', round(d['pcg_iterations_per_sec']), 'it/s keff', round(r['avg_launch_ms']*1e3,2), 'us')"
}
for L in 0 6 12 24; do
  if [ $L = 0 ]; then b c3h_Ldef --element hex8 --config c3 --steps 2 --warmup 1 || exit 2
  else CWF_LAT_L=$L b c3h_L$L --element hex8 --config c3 --steps 2 --warmup 1 || exit 2; fi
done
for L in 0 6 12 24; do
  if [ $L = 0 ]; then b c5_Ldef --config c5 --steps 1 --warmup 0 || exit 2
  else CWF_LAT_L=$L b c5_L$L --config c5 --steps 1 --warmup 0 || exit 2; fi
done
