source tools/ab.sh
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tall.log 2>&1; tail -1 gpurun_out/tall.log
run c2 python bench.py --no-cpu-baseline &&
run c3 python bench.py --no-cpu-baseline --config c3 --steps 3 --warmup 1
