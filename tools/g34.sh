#!/bin/bash
# hex8 evidence: rocprofv3 kernel trace + FETCH/WRITE PMC over the C2/C3 hex8 benches, PMC JSON named so
# bench.py's --traffic auto finds it, then the hex8 bench lines re-run so they carry the PMC traffic.
set -o pipefail
O=gpurun_out/hex
mkdir -p $O
K="k_keff_hex_tiles<true, false, 1,"
bash tools/profile.sh c2hex --element hex8 --steps 5 --warmup 1 --no-cpu-baseline > $O/profile_c2.log 2>&1 &&
python3 tools/pmc_summary.py gpurun_out/prof_c2hex --kernel "$K" --json $O/r01_c2_fast_hex8_pmc.json > $O/r01_c2_fast_hex8_summary.txt &&
cp gpurun_out/prof_c2hex/kt/kt_kernel_stats.csv $O/r01_c2_fast_hex8_kernel_stats.csv &&
bash tools/profile.sh c3hex --element hex8 --config c3 --steps 2 --warmup 1 --no-cpu-baseline > $O/profile_c3.log 2>&1 &&
python3 tools/pmc_summary.py gpurun_out/prof_c3hex --kernel "$K" --json $O/r01_c3_fast_hex8_pmc.json > $O/r01_c3_fast_hex8_summary.txt &&
cp gpurun_out/prof_c3hex/kt/kt_kernel_stats.csv $O/r01_c3_fast_hex8_kernel_stats.csv &&
cp $O/r01_c2_fast_hex8_pmc.json $O/r01_c3_fast_hex8_pmc.json profiles/ &&
timeout -k 10 300 python -u bench.py --element hex8 --no-cpu-baseline > $O/bench_c2hex.log 2>&1 && tail -1 $O/bench_c2hex.log > $O/r01_bench_c2_hex8_fast.json &&
timeout -k 10 300 python -u bench.py --element hex8 --config c3 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_c3hex.log 2>&1 && tail -1 $O/bench_c3hex.log > $O/r01_bench_c3_hex8_fast.json
rc=$?
rm -rf gpurun_out/prof_c2hex gpurun_out/prof_c3hex
head -6 $O/r01_c2_fast_hex8_summary.txt $O/r01_c3_fast_hex8_summary.txt
exit $rc
