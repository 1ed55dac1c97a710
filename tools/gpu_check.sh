#!/bin/bash
# GPU-box check: parity tests, smoke, short bench. Every GPU step has its own time limit; the
# script stops at the first crash/abort/timeout (exit >= 2 from pytest, or non-zero from others).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
STEPS=${STEPS:-3}
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ge 2 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; cat gpurun_out/smoke.log | tail -20; exit 3; }
tail -2 gpurun_out/smoke.log
timeout -k 10 600 python bench.py --steps $STEPS --warmup 1 ${BENCH_ARGS} > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench.log; exit 4; }
tail -3 gpurun_out/bench.log
exit $rc
