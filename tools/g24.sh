source tools/ab.sh
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tall.log 2>&1; tail -3 gpurun_out/tall.log
run c2hex python bench.py --no-cpu-baseline --element hex8 &&
run c3hex python bench.py --no-cpu-baseline --element hex8 --config c3 --steps 3 --warmup 1
