#!/bin/bash
# round 3: balanced fan-group tile count A/B (C2 two passes, C3 one) and the PARITY C2 profile
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
CWF_VERBOSE=1 timeout -k 10 120 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-hbm-roofline \
  > gpurun_out/verbose_c2.log 2>&1 && grep "fan groups" gpurun_out/verbose_c2.log | tail -2 &&
CONFIGS=c2 PASSES=2 bash tools/ab_env.sh "bal=CWF_GROUP_BALANCE=1" "nobal=CWF_GROUP_BALANCE=0" "r3=CWF_GROUP_ROUNDS=3" &&
CONFIGS=c3 PASSES=1 bash tools/ab_env.sh "bal=CWF_GROUP_BALANCE=1" &&
SQ_PMC=1 bash tools/profile.sh r03c_c2_parity --mode parity --steps 2 --warmup 1 --no-cpu-baseline --no-hbm-roofline &&
python3 tools/pmc_summary.py gpurun_out/prof_r03c_c2_parity --json gpurun_out/prof_r03c_c2_parity/pmc.json \
  > gpurun_out/prof_r03c_c2_parity/summary.txt &&
python3 tools/sq_summary.py gpurun_out/prof_r03c_c2_parity > gpurun_out/prof_r03c_c2_parity/sq_summary.txt
rc=$?
head -12 gpurun_out/prof_r03c_c2_parity/summary.txt
exit $rc
