set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && tail -3 gpurun_out/gpu_tests.log &&
timeout -k 10 300 python -u bench.py > gpurun_out/bench_c2.log 2>&1 && tail -1 gpurun_out/bench_c2.log &&
timeout -k 10 300 python -u bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c3.log 2>&1 && tail -1 gpurun_out/bench_c3.log &&
NO_PMC= bash tools/profile.sh c2 --steps 5 --warmup 1 --no-cpu-baseline && python tools/pmc_summary.py gpurun_out/prof_c2 --kernel keff_tiles --json gpurun_out/prof_c2/pmc.json > gpurun_out/prof_c2/summary.txt; cat gpurun_out/prof_c2/summary.txt
