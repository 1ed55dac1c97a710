#!/bin/bash
# lattice evidence: kernel-trace timelines (C3, C2), rocprofv3 kernel stats + FETCH / WRITE PMC passes of the C3 and
# C2 bench runs -> profiles/<TAG>_c{3,2}_fast_{summary.txt,pmc.json,kernel_stats.csv}
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=${1:-r03aa}
bash $R/tools/kt_timeline.sh || exit 1
for c in c3 c2; do
  NO_SQ=1 bash $R/tools/profile.sh ${TAG}_$c --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-hbm-roofline || exit 2
  python3 $R/tools/pmc_summary.py $R/gpurun_out/prof_${TAG}_$c --kernel k_keff_lattice --kernel k_pcg_update \
    --json $R/gpurun_out/prof_${TAG}_$c/pmc.json > $R/gpurun_out/prof_${TAG}_$c/summary.txt || exit 3
  cat $R/gpurun_out/prof_${TAG}_$c/summary.txt
done
