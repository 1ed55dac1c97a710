#!/bin/bash
# round 3 hex8 lattice: hex8 + lattice GPU tests, hex8 bench lines (C2, C3), C2/C3 hex8 kernel stats + PMC
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd $R
TAG=${1:-r03ac}
O=gpurun_out/round
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_hex8.py tests/test_gpu_lattice.py -m gpu -x -v --timeout 300 \
  --timeout-method thread > $O/${TAG}_gpu_tests.log 2>&1; rc=$?; tail -1 $O/${TAG}_gpu_tests.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" $O/${TAG}_gpu_tests.log | head -20; exit $rc; }
b() {
  local name=$1; shift
  timeout -k 10 500 python -u bench.py "$@" > $O/${TAG}_bench_${name}.log 2>&1 &&
  grep '^{"metric"' $O/${TAG}_bench_${name}.log > $O/${TAG}_bench_${name}.json &&
  python3 -c "
import json; d=json.load(open('$O/${TAG}_bench_${name}.json')); r=d['roofline']
print('$name', round(d['value']/1e9,2), 'G DOF-it/s', round(d['pcg_iterations_per_sec']), 'it/s', round(d['ms_per_step'],2), 'ms/step', 'keff', round(r['avg_launch_ms']*1e3,2), 'us frac', round(r['frac'],3), 'conv', d['steps_converged'], '/', d['steps'], r.get('kernel'))"
}
b c2_hex8_fast --element hex8 --no-cpu-baseline --no-hbm-roofline &&
b c3_hex8_fast --element hex8 --config c3 --steps 3 --warmup 1 --no-cpu-baseline --no-hbm-roofline &&
CWF_LATTICE=0 b c3_hex8_tiles --element hex8 --config c3 --steps 3 --warmup 1 --no-cpu-baseline --no-hbm-roofline || exit 2
for c in c3 c2; do
  NO_SQ=1 bash $R/tools/profile.sh ${TAG}_${c}_hex8 --element hex8 --config $c --steps 2 --warmup 1 --no-cpu-baseline \
    --no-hbm-roofline > /dev/null || exit 3
  python3 $R/tools/pmc_summary.py $R/gpurun_out/prof_${TAG}_${c}_hex8 --kernel "k_keff_lattice<1" \
    --json $R/gpurun_out/prof_${TAG}_${c}_hex8/pmc.json > $R/gpurun_out/prof_${TAG}_${c}_hex8/summary.txt || exit 4
  head -6 $R/gpurun_out/prof_${TAG}_${c}_hex8/summary.txt
done
