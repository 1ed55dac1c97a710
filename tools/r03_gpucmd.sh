#!/bin/bash
# round-3 GPU check: the BASELINE-config tests (C1/C4/C5 at full size) with per-test durations, then the rest
# of the -m gpu suite. A heartbeat file under gpurun_out/ marks progress during the multi-minute C5 test.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
tag=${1:-r03a}
(while sleep 30; do date >> gpurun_out/heartbeat.txt; done) &
hb=$!
timeout -k 10 1100 python -u -m pytest tests/test_gpu_configs.py -x -v -s --timeout 1200 --timeout-method thread \
  --durations=0 > gpurun_out/${tag}_configs.log 2>&1 &&
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    --ignore=tests/test_gpu_configs.py > gpurun_out/${tag}_tests.log 2>&1
rc=$?
kill $hb
tail -25 gpurun_out/${tag}_configs.log; tail -3 gpurun_out/${tag}_tests.log
exit $rc
