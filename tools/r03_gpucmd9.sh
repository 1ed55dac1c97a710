#!/bin/bash
# round 3: the multi-process RCCL-path tests through the host-staged transport (2 and 3 ranks on one GPU)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
tag=${1:-r03l}
timeout -k 10 600 python -u -m pytest tests/test_gpu_transport.py -m gpu -x -v --timeout 300 \
  --timeout-method thread > gpurun_out/${tag}_transport_tests.log 2>&1
rc=$?
tail -15 gpurun_out/${tag}_transport_tests.log
exit $rc
