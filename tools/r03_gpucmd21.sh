#!/bin/bash
# round 3 lattice evidence (uniform-mass bricks, hex8 lattice): -m gpu suite, smoke(), every config's bench line, C2/C3 FAST kernel stats + PMC
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd $R
TAG=${1:-r03af}
O=gpurun_out/round
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread \
  > $O/${TAG}_gpu_tests.log 2>&1; rc=$?; tail -1 $O/${TAG}_gpu_tests.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" $O/${TAG}_gpu_tests.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/${TAG}_smoke.log 2>&1 && tail -1 $O/${TAG}_smoke.log || exit 1
b() {
  local name=$1; shift
  timeout -k 10 500 python -u bench.py "$@" > $O/${TAG}_bench_${name}.log 2>&1 &&
  grep '^{"metric"' $O/${TAG}_bench_${name}.log > $O/${TAG}_bench_${name}.json &&
  python3 -c "
import json; d=json.load(open('$O/${TAG}_bench_${name}.json')); r=d['roofline']
h=d.get('roofline_hbm') or {}; g=d.get('roofline_general') or {}
print('$name', round(d['value']/1e9,2), 'G DOF-it/s', round(d['pcg_iterations_per_sec']), 'it/s', round(d['ms_per_step'],2), 'ms/step', 'keff', round(r['avg_launch_ms']*1e3,2), 'us frac', round(r['frac'],3), 'conv', d['steps_converged'], '/', d['steps'], 'hbm', h.get('frac'), 'general', g.get('frac'))"
}
b default &&
b c3_fast --config c3 --steps 3 --warmup 1 --no-cpu-baseline &&
b c4_fast --config c4 --steps 3 --warmup 1 --no-cpu-baseline --no-hbm-roofline &&
b c5_fast --config c5 --steps 1 --warmup 0 --no-cpu-baseline --no-hbm-roofline &&
b c2_hex8_fast --element hex8 --no-cpu-baseline --no-hbm-roofline &&
b c3_hex8_fast --element hex8 --config c3 --steps 3 --warmup 1 --no-cpu-baseline --no-hbm-roofline &&
b c2_parity --mode parity --steps 3 --warmup 1 --no-cpu-baseline --no-hbm-roofline || exit 2
for c in c3 c2; do
  NO_SQ=1 bash $R/tools/profile.sh ${TAG}_$c --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-hbm-roofline > /dev/null || exit 3
  python3 $R/tools/pmc_summary.py $R/gpurun_out/prof_${TAG}_$c --kernel "k_keff_lattice<1" \
    --json $R/gpurun_out/prof_${TAG}_$c/pmc.json > $R/gpurun_out/prof_${TAG}_$c/summary.txt || exit 4
  head -6 $R/gpurun_out/prof_${TAG}_$c/summary.txt
done
