#!/bin/bash
# lattice planes per brick (CWF_LAT_L) on C3 and C2, same box, two passes
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd $R
O=gpurun_out/lsweep; mkdir -p $O
b() {
  local name=$1; shift
  timeout -k 10 300 python -u bench.py "$@" --no-cpu-baseline --no-hbm-roofline > $O/${name}.log 2>&1 &&
  python3 -c "
import json; d=[json.loads(l) for l in open('$O/${name}.log') if l.startswith('{\"metric\"')][0]; r=d['roofline']
print('$name', round(d['pcg_iterations_per_sec']), 'it/s keff', round(r['avg_launch_ms']*1e3,2), 'us')"
}
for pass in 1 2; do
  for L in ${C3L:-0 8 11 20 28}; do
    if [ $L = 0 ]; then b c3_Ldef_p$pass --config c3 --steps 2 --warmup 1 || exit 2
    else CWF_LAT_L=$L b c3_L${L}_p$pass --config c3 --steps 2 --warmup 1 || exit 2; fi
  done
  for L in ${C2L:-0 3 6}; do
    if [ $L = 0 ]; then b c2_Ldef_p$pass || exit 2
    else CWF_LAT_L=$L b c2_L${L}_p$pass || exit 2; fi
  done
done
