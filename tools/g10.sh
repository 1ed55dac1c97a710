timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/tall.log 2>&1; tail -25 gpurun_out/tall.log
