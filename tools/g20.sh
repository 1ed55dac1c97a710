source tools/ab.sh
timeout -k 10 300 env CWF_PACKED=1 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "fast or shard or scenario" > gpurun_out/t.log 2>&1; tail -1 gpurun_out/t.log
for f in 0 1; do for c in c2 c3; do timeout -k 10 200 env CWF_PACKED=$f python tools/ablate.py --config $c --bits 0 > gpurun_out/abl.log 2>&1; echo "packed=$f $(grep abl gpurun_out/abl.log | tr '\n' ' ')"; done; done
for f in 0 1; do for c in c2 c3; do timeout -k 10 200 env CWF_PACKED=$f CWF_PIPE_NT=256 python tools/ablate.py --config $c --bits 0 > gpurun_out/abl.log 2>&1; echo "nt256 packed=$f $(grep abl gpurun_out/abl.log | tr '\n' ' ')"; done; done
