source tools/ab.sh
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "fast" > gpurun_out/t.log 2>&1; tail -1 gpurun_out/t.log
timeout -k 10 200 python tools/ablate.py --config c3 --bits 0 128 > gpurun_out/abl_c3.log 2>&1; grep -v amdgpu.ids gpurun_out/abl_c3.log
run c2 CWF_X=1 python bench.py --no-cpu-baseline &&
run c3 CWF_X=1 python bench.py --no-cpu-baseline --config c3 --steps 3 --warmup 1
