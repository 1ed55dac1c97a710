#!/bin/bash
# update-pass workgroup cap (CWF_UPD_CAP: the shares every K_eff workgroup refolds) on C3 and C2 bench lines, two passes
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd $R
O=gpurun_out/cap; mkdir -p $O
b() {
  local name=$1; shift
  timeout -k 10 300 python -u bench.py "$@" --no-cpu-baseline --no-hbm-roofline > $O/${name}.log 2>&1 &&
  python3 -c "
import json; d=[json.loads(l) for l in open('$O/${name}.log') if l.startswith('{\"metric\"')][0]; r=d['roofline']
print('$name', round(d['pcg_iterations_per_sec']), 'it/s keff', round(r['avg_launch_ms']*1e3,2), 'us')"
}
for pass in 1 2; do
  for cap in 0 1024 512 256; do
    if [ $cap = 0 ]; then b c3_def_p$pass --config c3 --steps 2 --warmup 1 || exit 2
    else CWF_UPD_CAP=$cap b c3_cap${cap}_p$pass --config c3 --steps 2 --warmup 1 || exit 2; fi
  done
  for cap in 0 512; do
    if [ $cap = 0 ]; then b c2_def_p$pass || exit 2; else CWF_UPD_CAP=$cap b c2_cap${cap}_p$pass || exit 2; fi
  done
done
