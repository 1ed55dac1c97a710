#!/bin/bash
# new p stored by the tiles kernels owner slots (ping-pong p buffers): GPU suite, then same-box A/B against lib_base
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/g37_tests.log 2>&1; rc=$?
tail -3 gpurun_out/g37_tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/g37_tests.log | head -20; exit $rc; }
bash tools/ab_lib.sh base
