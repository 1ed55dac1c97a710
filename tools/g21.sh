source tools/ab.sh
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tall.log 2>&1; tail -1 gpurun_out/tall.log
run c2 python bench.py --no-cpu-baseline &&
run c3 python bench.py --no-cpu-baseline --config c3 --steps 3 --warmup 1 &&
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3 -o c3 -- python bench.py --no-cpu-baseline --config c3 --steps 3 --warmup 1 > gpurun_out/prof_c3.log 2>&1; find gpurun_out/prof_c3 -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/c3_stats.csv; python3 -c "
import csv; r=list(csv.DictReader(open('gpurun_out/c3_stats.csv')))
for x in r[:8]: print(x['Name'][:60], x['Calls'], round(float(x['AverageNs'])/1e3,1), x['Percentage'])"
