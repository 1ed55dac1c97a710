#!/bin/bash
# quick lattice check: the lattice GPU tests, then spmv_bench on C3 and C2 (lattice kernel timing)
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd $R
O=gpurun_out/latq; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_lattice.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" $O/tests.log | head -20; exit $rc; }
for c in c3 c2; do timeout -k 10 200 python tools/spmv_bench.py --config $c --iters 200 || exit 1; done
