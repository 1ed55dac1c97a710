#!/bin/bash
# round 3: the whole -m gpu suite, then the default bench line (C2 + live C3 roofline + CPU baseline)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
tag=${1:-r03k}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread \
  > gpurun_out/${tag}_gpu_tests.log 2>&1 &&
timeout -k 10 400 python bench.py > gpurun_out/${tag}_bench.log 2>&1
rc=$?
tail -4 gpurun_out/${tag}_gpu_tests.log; tail -1 gpurun_out/${tag}_bench.log | cut -c1-300
exit $rc
