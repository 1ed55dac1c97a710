source tools/ab.sh
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "fast or shard or scenario" > gpurun_out/t.log 2>&1; tail -1 gpurun_out/t.log
for nt in 128 256; do timeout -k 10 200 env CWF_PIPE_NT=$nt python tools/ablate.py --config c2 --bits 0 > gpurun_out/abl.log 2>&1; echo "nt=$nt $(grep abl gpurun_out/abl.log)"; done
for nt in 128 256; do timeout -k 10 200 env CWF_PIPE_NT=$nt python tools/ablate.py --config c3 --bits 0 > gpurun_out/abl.log 2>&1; echo "nt=$nt $(grep abl gpurun_out/abl.log)"; done
run c2_128 CWF_PIPE_NT=128 python bench.py --no-cpu-baseline &&
run c2_256 CWF_PIPE_NT=256 python bench.py --no-cpu-baseline &&
run c3_128 CWF_PIPE_NT=128 python bench.py --no-cpu-baseline --config c3 --steps 3 --warmup 1
