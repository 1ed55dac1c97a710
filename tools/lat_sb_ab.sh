#!/bin/bash
# brick super-block order (CWF_LAT_SB) A/B on C3 and C5, after the lattice tests
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd $R
O=gpurun_out/sb; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_lattice.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/tests.log 2>&1; rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $O/tests.log | head; exit $rc; }
b() {
  local name=$1; shift
  timeout -k 10 400 python -u bench.py "$@" --no-cpu-baseline --no-hbm-roofline > $O/${name}.log 2>&1 &&
  python3 -c "
import json; d=[json.loads(l) for l in open('$O/${name}.log') if l.startswith('{\"metric\"')][0]; r=d['roofline']
print('$name', round(d['pcg_iterations_per_sec']), 'it/s keff', round(r['avg_launch_ms']*1e3,2), 'us')"
}
for pass in 1 2; do
  for v in 0 4,3 8,2 2,6 19,1; do
    CWF_LAT_SB=$v b c3_sb${v/,/x}_p$pass --config c3 --steps 2 --warmup 1 || exit 2
  done
done
for v in 0 4,1 10,1; do CWF_LAT_SB=$v b c5_sb${v/,/x} --config c5 --steps 1 --warmup 0 || exit 2; done
