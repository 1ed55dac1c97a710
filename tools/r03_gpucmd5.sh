#!/bin/bash
# round 3: PARITY speedups (staged folds, chunk dots, element-centric K_eff) -- bitwise tests, kernel-trace
# profiles of the C2 PARITY bench (element-centric and node-centric K_eff), then two default C2 bench lines
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
tag=${1:-r03f}
kstats() {
python3 - "$1" <<'PY'
import csv,glob,sys
f=glob.glob(f"gpurun_out/prof_{sys.argv[1]}/kt/*kernel_stats.csv")[0]
for r in csv.DictReader(open(f)):
    print("%-60s %7s %10.2f %6.2f" % (r["Name"][:60], r["Calls"], float(r["AverageNs"])/1e3, float(r["Percentage"])))
PY
}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_shard.py \
  tests/test_gpu_scenario.py "tests/test_gpu_configs.py::test_c1_parity_solve_bitwise_with_history" \
  "tests/test_gpu_configs.py::test_c1_parity_stepper_three_steps_bitwise" \
  "tests/test_gpu_configs.py::test_c4_small_harmonic_parity_steps_bitwise" -m gpu -x -q --timeout 300 \
  --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 &&
NO_PMC=1 bash tools/profile.sh ${tag}_c2_parity --mode parity --steps 2 --warmup 1 --no-cpu-baseline \
  --no-hbm-roofline > gpurun_out/${tag}_prof.log 2>&1 && kstats ${tag}_c2_parity > gpurun_out/${tag}_kstats.txt &&
CWF_PARITY_NODE=1 NO_PMC=1 bash tools/profile.sh ${tag}_c2_parity_node --mode parity --steps 2 --warmup 1 \
  --no-cpu-baseline --no-hbm-roofline > gpurun_out/${tag}_prof_node.log 2>&1 &&
kstats ${tag}_c2_parity_node > gpurun_out/${tag}_kstats_node.txt &&
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/${tag}_bench_c2_a.log 2>&1 &&
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/${tag}_bench_c2_b.log 2>&1
rc=$?
tail -3 gpurun_out/${tag}_tests.log; head -8 gpurun_out/${tag}_kstats.txt; head -4 gpurun_out/${tag}_kstats_node.txt
for f in gpurun_out/${tag}_bench_c2_a.log gpurun_out/${tag}_bench_c2_b.log; do python3 -c "
import json,sys; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); r=d['roofline']
print('it/s %.1f keff %.2f us frac %.3f hbm %.3f' % (d['pcg_iterations_per_sec'], r['avg_launch_ms']*1e3, r['frac'], (d['roofline_hbm'] or {}).get('frac',0)))"; done
exit $rc
