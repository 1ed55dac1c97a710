#!/bin/bash
# lattice (structured Kuhn block) path: GPU tests, then the C2 and C3 bench lines
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r03y}
O=gpurun_out/round
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_lattice.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 \
  --timeout-method thread > $O/${TAG}_gpu_tests.log 2>&1; rc=$?; tail -3 $O/${TAG}_gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/${TAG}_bench_c2.log 2>&1 &&
grep '^{"metric"' $O/${TAG}_bench_c2.log > $O/${TAG}_bench_c2.json &&
timeout -k 10 300 python bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline --no-hbm-roofline \
  > $O/${TAG}_bench_c3.log 2>&1 && grep '^{"metric"' $O/${TAG}_bench_c3.log > $O/${TAG}_bench_c3.json
rc=$?
for f in $O/${TAG}_bench_*.json; do python3 -c "
import json; d=json.load(open('$f')); r=d['roofline']; h=d.get('roofline_hbm') or {}
print('$(basename $f)', round(d['value']/1e9,3), 'G DOF-it/s', round(d['pcg_iterations_per_sec']), 'it/s', round(d['ms_per_step'],2), 'ms', 'keff', round(r['avg_launch_ms']*1e3,2), 'frac', round(r['frac'],3), 'hbm', h.get('frac'), h.get('avg_launch_ms'))"; done
exit $rc
