source tools/ab.sh
( while true; do date >> gpurun_out/heartbeat.log; sleep 20; done ) &
HB=$!
run c4_morton CWF_MORTON_NODES=1 python bench.py --no-cpu-baseline --config c4 --steps 3 --warmup 1 &&
run c3_morton CWF_MORTON_NODES=1 python bench.py --no-cpu-baseline --config c3 --steps 3 --warmup 1 &&
run c2_morton CWF_MORTON_NODES=1 python bench.py --no-cpu-baseline
kill $HB
