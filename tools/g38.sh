#!/bin/bash
# after a profile refresh: hex8 profiles + lines (g34), then the C2/C3 tet lines again so their
# roofline.traffic reads the PMC summary of the same build
set -o pipefail
bash tools/g34.sh &&
timeout -k 10 300 python -u bench.py > gpurun_out/hex/bench_c2.log 2>&1 && tail -1 gpurun_out/hex/bench_c2.log > gpurun_out/hex/r01_bench_c2_fast.json &&
timeout -k 10 300 python -u bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/hex/bench_c3.log 2>&1 && tail -1 gpurun_out/hex/bench_c3.log > gpurun_out/hex/r01_bench_c3_fast.json
