#!/bin/bash
# packed lattice rows: lattice / hex8 / shard / parity GPU tests, then a same-box A/B against lib_base (C2, C3, C3 hex8)
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd $R
O=gpurun_out/round; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_lattice.py tests/test_hex8.py tests/test_gpu_shard.py \
  tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/r03am_gpu_tests.log 2>&1; rc=$?
tail -1 $O/r03am_gpu_tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $O/r03am_gpu_tests.log | head -20; exit $rc; }
b() {
  local name=$1; shift
  timeout -k 10 300 python -u bench.py "$@" --no-cpu-baseline --no-hbm-roofline > $O/r03am_${name}.log 2>&1 &&
  python3 -c "
import json; d=[json.loads(l) for l in open('$O/r03am_${name}.log') if l.startswith('{\"metric\"')][0]; r=d['roofline']
print('$name', round(d['pcg_iterations_per_sec']), 'it/s keff', round(r['avg_launch_ms']*1e3,2), 'us')"
}
BASE=$PWD/civiwave-fem_amd/lib_base/libcwf_hip.so
for pass in 1 2; do
  b c2_new_p$pass && CWF_LIB_PATH=$BASE b c2_base_p$pass &&
  b c3_new_p$pass --config c3 --steps 2 --warmup 1 && CWF_LIB_PATH=$BASE b c3_base_p$pass --config c3 --steps 2 --warmup 1 &&
  b c3h_new_p$pass --element hex8 --config c3 --steps 2 --warmup 1 &&
  CWF_LIB_PATH=$BASE b c3h_base_p$pass --element hex8 --config c3 --steps 2 --warmup 1 || exit 2
done
