#!/bin/bash
# round-end check: smoke(), then the C4 / C5 single-GPU lines on the current build
set -o pipefail
O=gpurun_out/final
mkdir -p $O
( while true; do date >> $O/heartbeat.log; sleep 20; done ) &
HB=$!
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 &&
timeout -k 10 500 python -u bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_c4.log 2>&1 && tail -1 $O/bench_c4.log > $O/r01_bench_c4_fast.json &&
timeout -k 10 700 python -u bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_c5.log 2>&1 && tail -1 $O/bench_c5.log > $O/r01_bench_c5_fast.json
rc=$?
kill $HB
tail -1 $O/smoke.log
exit $rc
