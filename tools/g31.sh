source tools/ab.sh
timeout -k 10 300 python -u -m pytest tests/test_hex8.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/thex.log 2>&1; tail -3 gpurun_out/thex.log
run c2hex python bench.py --no-cpu-baseline --element hex8 &&
run c3hex python bench.py --no-cpu-baseline --element hex8 --config c3 --steps 3 --warmup 1
