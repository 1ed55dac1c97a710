#!/bin/bash
# Full GPU evidence pass: whole GPU suite, default bench line (C2, with CPU baseline), C3 line, hex8 lines,
# rocprofv3 kernel-trace + FETCH/WRITE PMC passes over the C2 and C3 benches, summaries under
# gpurun_out/round/. usage: bash tools/gpu_round.sh TAG
set -o pipefail
TAG=${1:-r01}
O=gpurun_out/round
mkdir -p $O
K="k_keff_groups_pipe<true, false, 1,"
timeout -k 10 400 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $O/${TAG}_gpu_tests.log 2>&1; tail -1 $O/${TAG}_gpu_tests.log
timeout -k 10 300 python -u bench.py > $O/${TAG}_bench_c2.log 2>&1 && tail -1 $O/${TAG}_bench_c2.log > $O/${TAG}_bench_c2_fast.json &&
timeout -k 10 300 python -u bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline > $O/${TAG}_bench_c3.log 2>&1 && tail -1 $O/${TAG}_bench_c3.log > $O/${TAG}_bench_c3_fast.json &&
timeout -k 10 300 python -u bench.py --element hex8 --no-cpu-baseline > $O/${TAG}_bench_c2hex.log 2>&1 && tail -1 $O/${TAG}_bench_c2hex.log > $O/${TAG}_bench_c2_hex8_fast.json &&
timeout -k 10 300 python -u bench.py --element hex8 --config c3 --steps 3 --warmup 1 --no-cpu-baseline > $O/${TAG}_bench_c3hex.log 2>&1 && tail -1 $O/${TAG}_bench_c3hex.log > $O/${TAG}_bench_c3_hex8_fast.json &&
bash tools/profile.sh c2 --steps 5 --warmup 1 --no-cpu-baseline --no-hbm-roofline > $O/${TAG}_profile_c2.log 2>&1 &&
python3 tools/pmc_summary.py gpurun_out/prof_c2 --kernel "$K" --json $O/${TAG}_c2_fast_pmc.json > $O/${TAG}_c2_fast_summary.txt &&
cp gpurun_out/prof_c2/kt/kt_kernel_stats.csv $O/${TAG}_c2_fast_kernel_stats.csv && grep "^{\"metric" gpurun_out/prof_c2/bench_kt.log > $O/${TAG}_c2_bench_under_rocprof.json &&
bash tools/profile.sh c3 --config c3 --steps 2 --warmup 1 --no-cpu-baseline > $O/${TAG}_profile_c3.log 2>&1 &&
python3 tools/pmc_summary.py gpurun_out/prof_c3 --kernel "$K" --json $O/${TAG}_c3_fast_pmc.json > $O/${TAG}_c3_fast_summary.txt &&
cp gpurun_out/prof_c3/kt/kt_kernel_stats.csv $O/${TAG}_c3_fast_kernel_stats.csv && grep "^{\"metric" gpurun_out/prof_c3/bench_kt.log > $O/${TAG}_c3_bench_under_rocprof.json
rc=$?
rm -rf gpurun_out/prof_c2 gpurun_out/prof_c3
head -8 $O/${TAG}_c2_fast_summary.txt
head -8 $O/${TAG}_c3_fast_summary.txt
exit $rc
