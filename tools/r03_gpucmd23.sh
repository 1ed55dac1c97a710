#!/bin/bash
# z from r (lattice lzr): lattice + hex8 + shard + parity GPU tests, then C2 / C3 A/B (CWF_LAT_ZR), two passes
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd $R
TAG=${1:-r03ah}
O=gpurun_out/round
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_lattice.py tests/test_hex8.py tests/test_gpu_shard.py \
  tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/${TAG}_gpu_tests.log 2>&1; rc=$?
tail -1 $O/${TAG}_gpu_tests.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" $O/${TAG}_gpu_tests.log | head -20; exit $rc; }
b() {
  local name=$1; shift
  timeout -k 10 300 python -u bench.py "$@" --no-cpu-baseline --no-hbm-roofline > $O/${TAG}_bench_${name}.log 2>&1 &&
  grep '^{"metric"' $O/${TAG}_bench_${name}.log > $O/${TAG}_bench_${name}.json &&
  python3 -c "
import json; d=json.load(open('$O/${TAG}_bench_${name}.json')); r=d['roofline']
print('$name', round(d['value']/1e9,2), 'G DOF-it/s', round(d['pcg_iterations_per_sec']), 'it/s keff', round(r['avg_launch_ms']*1e3,2), 'us', r.get('kernel'), 'conv', d['steps_converged'])"
}
for pass in 1 2; do
  b c2_zr_p$pass && CWF_LAT_ZR=0 b c2_z_p$pass &&
  b c3_zr_p$pass --config c3 --steps 2 --warmup 1 && CWF_LAT_ZR=0 b c3_z_p$pass --config c3 --steps 2 --warmup 1 || exit 2
done
b c3_hex8 --element hex8 --config c3 --steps 2 --warmup 1 || exit 2
