source tools/ab.sh
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "fast or shard or scenario" > gpurun_out/t.log 2>&1; tail -3 gpurun_out/t.log
run c2 CWF_X=1 python bench.py --no-cpu-baseline &&
run c3 CWF_X=1 python bench.py --no-cpu-baseline --config c3 --steps 3 --warmup 1 &&
NO_PMC=1 bash tools/profile.sh c3 --config c3 --steps 1 --warmup 1 --no-cpu-baseline >/dev/null 2>&1; python3 -c "
import csv
for r in list(csv.DictReader(open('gpurun_out/prof_c3/kt/kt_kernel_stats.csv')))[:3]:
    print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,1))
"; rm -rf gpurun_out/prof_c3
