#!/bin/bash
# round 3, lattice path: the whole -m gpu suite, smoke(), the default bench line and the C3 line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r03z}
O=gpurun_out/round
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread \
  > $O/${TAG}_gpu_tests.log 2>&1; rc=$?; tail -1 $O/${TAG}_gpu_tests.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" $O/${TAG}_gpu_tests.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/${TAG}_smoke.log 2>&1 && tail -1 $O/${TAG}_smoke.log &&
timeout -k 10 400 python bench.py > $O/${TAG}_bench_default.log 2>&1 &&
grep '^{"metric"' $O/${TAG}_bench_default.log > $O/${TAG}_bench_default.json &&
timeout -k 10 400 python bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline --no-hbm-roofline \
  > $O/${TAG}_bench_c3.log 2>&1 && grep '^{"metric"' $O/${TAG}_bench_c3.log > $O/${TAG}_bench_c3.json
rc=$?
for f in $O/${TAG}_bench_*.json; do python3 -c "
import json; d=json.load(open('$f')); r=d['roofline']; h=d.get('roofline_hbm') or {}
print('$(basename $f)', round(d['value']/1e9,3), 'G DOF-it/s', round(d['pcg_iterations_per_sec']), 'it/s', round(d['ms_per_step'],2), 'ms', 'keff', round(r['avg_launch_ms']*1e3,2), 'frac', round(r['frac'],3), 'hbm', h.get('frac'), h.get('avg_launch_ms'))"; done
exit $rc
