#!/bin/bash
# round-3 GPU check 2: the GPU suite minus the full-size config files, then the default bench line and the C4
# (harmonic load, RCB-capable) line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
tag=${1:-r03b}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_post.py tests/test_gpu_renumber.py \
  tests/test_gpu_scenario.py tests/test_gpu_shard.py tests/test_hex8.py -m gpu -x -v --timeout 300 \
  --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 &&
  timeout -k 10 400 python -u bench.py > gpurun_out/${tag}_bench_c2.log 2>&1 &&
  timeout -k 10 400 python -u bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline --no-hbm-roofline \
    > gpurun_out/${tag}_bench_c4.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/${tag}_tests.log | tail -5; tail -3 gpurun_out/${tag}_tests.log
tail -c 1500 gpurun_out/${tag}_bench_c2.log; tail -c 1500 gpurun_out/${tag}_bench_c4.log
exit $rc
