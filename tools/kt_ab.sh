# Same-box rocprofv3 kernel-time comparison of the in-tree lib ("new") and lib_base on C3 (bench.py)
cd /tmp && export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT
for v in new base; do
  if [ $v = base ]; then export CWF_LIB_PATH=$R/civiwave-fem_amd/lib_base/libcwf_hip.so; else unset CWF_LIB_PATH; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/kt_$v -o kt -- python3 $R/bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/kt_$v.log 2>&1 || exit 1
  echo "== $v"; f=$(find $R/gpurun_out/kt_$v -name "*kernel_stats.csv" | head -1); python3 -c "
import csv,sys
for r in csv.DictReader(open('$f')):
    if float(r['Percentage'])>0.3: print('%-60s %6s %10.2f %6.2f'%(r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e3, float(r['Percentage'])))"
done
