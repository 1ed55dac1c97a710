timeout -k 10 300 python -u -m pytest tests/test_gpu_renumber.py -x -v --timeout 120 --timeout-method thread > gpurun_out/tren.log 2>&1; tail -8 gpurun_out/tren.log
