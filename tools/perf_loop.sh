#!/bin/bash
# GPU-box perf iteration: FAST parity-tolerance tests, then K_eff / PCG timings on c2 and c3 and the
# tiles-kernel ablation sweep (CWF_TIMED_PCG dry path). Each GPU step has its own limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider ${TESTK:+-k "$TESTK"} > gpurun_out/pytest_fast.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_fast.log
if [ $rc -ne 0 ] && [ $rc -ne 5 ]; then exit $rc; fi
export CWF_VERBOSE=1
for c in ${CONFIGS:-c2 c3}; do
  timeout -k 10 300 python tools/spmv_bench.py --config $c --iters ${ITERS:-300} || exit $?
done
for a in ${ABL:-}; do
  CWF_TIMED_PCG=$a timeout -k 10 300 python tools/spmv_bench.py --config c2 --iters 50 || exit $?
done
exit 0
