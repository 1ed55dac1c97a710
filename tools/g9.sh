timeout -k 10 300 python -u -m pytest tests/test_gpu_post.py -x -v --timeout 120 --timeout-method thread > gpurun_out/tpost.log 2>&1; tail -15 gpurun_out/tpost.log
