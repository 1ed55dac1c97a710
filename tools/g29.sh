source tools/ab.sh
( while true; do date >> gpurun_out/heartbeat.log; sleep 20; done ) &
HB=$!
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/tall.log 2>&1; tail -3 gpurun_out/tall.log
run c4 python bench.py --no-cpu-baseline --config c4 --steps 3 --warmup 1 &&
run c3 python bench.py --no-cpu-baseline --config c3 --steps 3 --warmup 1 &&
run c2 python bench.py --no-cpu-baseline
kill $HB
