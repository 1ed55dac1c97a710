#!/bin/bash
# round 3: the full-size GPU tests (C2 / C3 incl. the multi-block PARITY fold test)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -v --timeout 900 --timeout-method thread \
  --durations=5 > gpurun_out/r03v_fullsize_tests.log 2>&1
rc=$?
tail -15 gpurun_out/r03v_fullsize_tests.log
exit $rc
