set -o pipefail
O=gpurun_out/round; mkdir -p $O
( while true; do date >> gpurun_out/heartbeat.log; sleep 20; done ) &
HB=$!
timeout -k 10 400 python -u bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline > $O/r01_bench_c4.log 2>&1 && tail -1 $O/r01_bench_c4.log > $O/r01_bench_c4_fast.json &&
timeout -k 10 700 python -u bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline > $O/r01_bench_c5.log 2>&1 && tail -1 $O/r01_bench_c5.log > $O/r01_bench_c5_fast.json
rc=$?
kill $HB
for f in $O/r01_bench_c4_fast.json $O/r01_bench_c5_fast.json; do python3 -c "
import json; d=json.load(open('$f')); r=d['roofline']
print('$f', round(d['value']/1e9,2),'GDOF-it/s', round(d['pcg_iterations_per_sec']),'it/s', round(d['ms_per_step'],1),'ms/step keff', round(r['avg_launch_ms']*1e3,1),'frac', round(r['frac'],3), 'refequiv', round(r['reference_layout_equiv_gbs']))"; done
tail -3 $O/r01_bench_c5.log
exit $rc
