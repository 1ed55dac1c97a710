#!/bin/bash
# shell workgroups first (default) vs last (CWF_LAT_SHELL_LAST=1): lattice tests with it on, C2 / C3 bench A/B
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd $R
O=gpurun_out/shell; mkdir -p $O
CWF_LAT_SHELL_LAST=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_lattice.py -m gpu -x -q --timeout 300 \
  --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
b() {
  local name=$1; shift
  timeout -k 10 300 python -u bench.py "$@" --no-cpu-baseline --no-hbm-roofline > $O/${name}.log 2>&1 &&
  python3 -c "
import json; d=[json.loads(l) for l in open('$O/${name}.log') if l.startswith('{\"metric\"')][0]; r=d['roofline']
print('$name', round(d['pcg_iterations_per_sec']), 'it/s keff', round(r['avg_launch_ms']*1e3,2), 'us')"
}
for pass in 1 2; do
  b c2_first_p$pass && CWF_LAT_SHELL_LAST=1 b c2_last_p$pass &&
  b c3_first_p$pass --config c3 --steps 2 --warmup 1 && CWF_LAT_SHELL_LAST=1 b c3_last_p$pass --config c3 --steps 2 --warmup 1 || exit 2
done
