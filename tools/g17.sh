source tools/ab.sh
timeout -k 10 300 env CWF_TILE_ORDER=deg python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "fast or shard or scenario" > gpurun_out/t.log 2>&1; tail -1 gpurun_out/t.log
for f in id deg; do for c in c2 c3; do timeout -k 10 200 env CWF_TILE_ORDER=$f python tools/ablate.py --config $c --bits 0 128 > gpurun_out/abl.log 2>&1; echo "order=$f $(grep abl gpurun_out/abl.log | tr '\n' ' ')"; done; done
run c2_deg CWF_TILE_ORDER=deg python bench.py --no-cpu-baseline &&
run c3_deg CWF_TILE_ORDER=deg python bench.py --no-cpu-baseline --config c3 --steps 3 --warmup 1
