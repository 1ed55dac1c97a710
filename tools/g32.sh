source tools/ab.sh
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "fast or renumber" > gpurun_out/t.log 2>&1; tail -1 gpurun_out/t.log
for c in c2 c3; do timeout -k 10 200 python tools/ablate.py --config $c --bits 0 > gpurun_out/abl.log 2>&1; echo "$(grep abl gpurun_out/abl.log | tr '\n' ' ')"; done
run c2 python bench.py --no-cpu-baseline &&
run c3 python bench.py --no-cpu-baseline --config c3 --steps 3 --warmup 1
