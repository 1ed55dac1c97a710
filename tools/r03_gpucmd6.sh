#!/bin/bash
# round 3: PARITY fused-dot tests + C2 parity profile
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
tag=${1:-r03g}
kstats() {
python3 - "$1" <<'PY'
import csv,glob,sys
f=glob.glob(f"gpurun_out/prof_{sys.argv[1]}/kt/*kernel_stats.csv")[0]
for r in csv.DictReader(open(f)):
    print("%-60s %7s %10.2f %6.2f" % (r["Name"][:60], r["Calls"], float(r["AverageNs"])/1e3, float(r["Percentage"])))
PY
}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_shard.py \
  "tests/test_gpu_configs.py::test_c1_parity_solve_bitwise_with_history" \
  "tests/test_gpu_configs.py::test_c1_parity_stepper_three_steps_bitwise" \
  "tests/test_gpu_configs.py::test_c4_small_harmonic_parity_steps_bitwise" -m gpu -x -q --timeout 300 \
  --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 &&
NO_PMC=1 bash tools/profile.sh ${tag}_c2_parity --mode parity --steps 2 --warmup 1 --no-cpu-baseline \
  --no-hbm-roofline > gpurun_out/${tag}_prof.log 2>&1 && kstats ${tag}_c2_parity > gpurun_out/${tag}_kstats.txt
rc=$?
tail -3 gpurun_out/${tag}_tests.log; head -12 gpurun_out/${tag}_kstats.txt; grep '"metric"' gpurun_out/${tag}_prof.log
exit $rc
