set -o pipefail
O=gpurun_out/round; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py -v --timeout 600 --timeout-method thread --durations=0 > gpurun_out/tfull.log 2>&1; tail -12 gpurun_out/tfull.log
bash tools/profile.sh c2hex --element hex8 --steps 5 --warmup 1 --no-cpu-baseline > $O/r01_profile_c2hex.log 2>&1 &&
python3 tools/pmc_summary.py gpurun_out/prof_c2hex --kernel "k_keff_hex_tiles<true, false, 1," --json $O/r01_c2_fast_hex8_pmc.json > $O/r01_c2_fast_hex8_summary.txt &&
cp gpurun_out/prof_c2hex/kt/kt_kernel_stats.csv $O/r01_c2_fast_hex8_kernel_stats.csv && cp $O/r01_c2_fast_hex8_pmc.json profiles/ &&
timeout -k 10 300 python -u bench.py --element hex8 --no-cpu-baseline > $O/r01_bench_c2hex.log 2>&1 && tail -1 $O/r01_bench_c2hex.log > $O/r01_bench_c2_hex8_fast.json
rm -rf gpurun_out/prof_c2hex
head -6 $O/r01_c2_fast_hex8_summary.txt; cat $O/r01_bench_c2_hex8_fast.json | cut -c1-300
