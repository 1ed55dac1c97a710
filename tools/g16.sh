source tools/ab.sh
timeout -k 10 300 env CWF_PIPE_FOLD=acc python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "fast or shard or scenario" > gpurun_out/t.log 2>&1; tail -1 gpurun_out/t.log
for f in csr acc; do for c in c2 c3; do timeout -k 10 200 env CWF_PIPE_FOLD=$f python tools/ablate.py --config $c --bits 0 > gpurun_out/abl.log 2>&1; echo "fold=$f $(grep abl gpurun_out/abl.log)"; done; done
run c2_acc CWF_PIPE_FOLD=acc python bench.py --no-cpu-baseline &&
run c2_csr CWF_PIPE_FOLD=csr python bench.py --no-cpu-baseline &&
run c3_acc CWF_PIPE_FOLD=acc python bench.py --no-cpu-baseline --config c3 --steps 3 --warmup 1 &&
run c3_csr CWF_PIPE_FOLD=csr python bench.py --no-cpu-baseline --config c3 --steps 3 --warmup 1
