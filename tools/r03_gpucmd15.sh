#!/bin/bash
# round 3 final evidence: the whole -m gpu suite, smoke(), the default bench line, PARITY C2 and C3 lines
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r03w}
O=gpurun_out/round
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread \
  > $O/${TAG}_gpu_tests.log 2>&1 && tail -1 $O/${TAG}_gpu_tests.log &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/${TAG}_smoke.log 2>&1 && tail -1 $O/${TAG}_smoke.log &&
timeout -k 10 400 python bench.py > $O/${TAG}_bench_default.log 2>&1 &&
grep '^{"metric"' $O/${TAG}_bench_default.log > $O/${TAG}_bench_default.json &&
timeout -k 10 300 python bench.py --mode parity --steps 3 --warmup 1 --no-cpu-baseline --no-hbm-roofline \
  > $O/${TAG}_bench_c2_parity.log 2>&1 && grep '^{"metric"' $O/${TAG}_bench_c2_parity.log > $O/${TAG}_bench_c2_parity.json &&
timeout -k 10 400 python bench.py --mode parity --config c3 --steps 1 --warmup 0 --no-cpu-baseline --no-hbm-roofline \
  > $O/${TAG}_bench_c3_parity.log 2>&1 && grep '^{"metric"' $O/${TAG}_bench_c3_parity.log > $O/${TAG}_bench_c3_parity.json
rc=$?
for f in $O/${TAG}_bench_*.json; do python3 -c "
import json; d=json.load(open('$f')); r=d['roofline']; h=d.get('roofline_hbm') or {}
print('$(basename $f)', round(d['value']/1e9,3), 'G DOF-it/s', round(d['pcg_iterations_per_sec']), 'it/s', round(d['ms_per_step'],2), 'ms', 'keff', round(r['avg_launch_ms']*1e3,2), 'frac', round(r['frac'],3), 'hbm', h.get('frac'))"; done
exit $rc
