set -o pipefail
( while true; do date >> gpurun_out/heartbeat.log; sleep 20; done ) &
HB=$!
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; tail -1 gpurun_out/smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench_default.log 2>&1; tail -1 gpurun_out/bench_default.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], d['pcg_iterations_per_sec'], r['frac'], r['measured_copy_gbs'], r['frac_of_measured_copy'], d['cpu_baseline']['value'])"
kill $HB
