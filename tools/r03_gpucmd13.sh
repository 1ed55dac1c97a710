#!/bin/bash
# round 3: same-box A/B of the in-tree lib against civiwave-fem_amd/lib_base (C2 + C3, two passes) and the FAST tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q -k "fast" \
  --timeout 200 --timeout-method thread > gpurun_out/ab_fast_tests.log 2>&1 && tail -2 gpurun_out/ab_fast_tests.log &&
bash tools/ab_lib.sh base
