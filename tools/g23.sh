timeout -k 10 300 python -u -m pytest tests/test_hex8.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/thex.log 2>&1; tail -25 gpurun_out/thex.log
