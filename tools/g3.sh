source tools/ab.sh
bash tools/sq_profile.sh c2 && python3 tools/sq_summary.py gpurun_out/sq_c2 > gpurun_out/sq_c2.txt &&
bash tools/sq_profile.sh c3 --config c3 --steps 1 --warmup 1 --no-cpu-baseline && python3 tools/sq_summary.py gpurun_out/sq_c3 > gpurun_out/sq_c3.txt &&
NO_PMC=1 bash tools/profile.sh c2 && cp gpurun_out/prof_c2/kt/kt_kernel_stats.csv gpurun_out/c2_stats.csv && tail -1 gpurun_out/prof_c2/bench_kt.log > gpurun_out/c2_kt_bench.json
rm -rf gpurun_out/sq_c2 gpurun_out/sq_c3 gpurun_out/prof_c2
