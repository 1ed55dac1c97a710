#!/bin/bash
# round 3: PARITY path speedups -- bitwise tests, then the C2 PARITY kernel-trace profile
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
tag=${1:-r03e}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_shard.py \
  tests/test_gpu_scenario.py "tests/test_gpu_configs.py::test_c1_parity_solve_bitwise_with_history" \
  "tests/test_gpu_configs.py::test_c1_parity_stepper_three_steps_bitwise" \
  "tests/test_gpu_configs.py::test_c4_small_harmonic_parity_steps_bitwise" -m gpu -x -q --timeout 300 \
  --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 &&
NO_PMC=1 bash tools/profile.sh ${tag}_c2_parity --mode parity --steps 2 --warmup 1 --no-cpu-baseline --no-hbm-roofline \
  > gpurun_out/${tag}_prof.log 2>&1 &&
python3 - <<'PY' > gpurun_out/${tag}_kstats.txt
import csv,glob,os
tag=os.environ.get("TAG","")
f=sorted(glob.glob("gpurun_out/prof_*_c2_parity/kt/*kernel_stats.csv"), key=os.path.getmtime)[-1]
for r in csv.DictReader(open(f)):
    print("%-60s %7s %10.2f %6.2f" % (r["Name"][:60], r["Calls"], float(r["AverageNs"])/1e3, float(r["Percentage"])))
PY
rc=$?
tail -3 gpurun_out/${tag}_tests.log; tail -2 gpurun_out/${tag}_prof.log | cut -c1-600; head -12 gpurun_out/${tag}_kstats.txt
exit $rc
