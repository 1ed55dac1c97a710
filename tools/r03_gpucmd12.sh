#!/bin/bash
# round 3 evidence B: rocprofv3 kernel trace + FETCH/WRITE PMC passes over the C2 and C3 FAST benches and the
# C2 PARITY bench, SQ passes over C3 FAST -> gpurun_out/round/${TAG}_*
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r03o}
O=gpurun_out/round
mkdir -p $O
K="k_keff_groups_pipe<true, false, 1,"
prof() {
  local name=$1 kern=$2; shift 2
  bash tools/profile.sh ${TAG}_$name "$@" > $O/${TAG}_profile_$name.log 2>&1 &&
  python3 tools/pmc_summary.py gpurun_out/prof_${TAG}_$name --kernel "$kern" --json $O/${TAG}_${name}_pmc.json \
    > $O/${TAG}_${name}_summary.txt &&
  cp gpurun_out/prof_${TAG}_$name/kt/kt_kernel_stats.csv $O/${TAG}_${name}_kernel_stats.csv &&
  grep '^{"metric"' gpurun_out/prof_${TAG}_$name/bench_kt.log > $O/${TAG}_${name}_bench_under_rocprof.json &&
  head -6 $O/${TAG}_${name}_summary.txt
}
prof c2_fast "$K" --steps 5 --warmup 1 --no-cpu-baseline --no-hbm-roofline &&
prof c3_fast "$K" --config c3 --steps 2 --warmup 1 --no-cpu-baseline &&
prof c2_parity "k_keff_parity" --mode parity --steps 2 --warmup 1 --no-cpu-baseline --no-hbm-roofline &&
bash tools/sq_profile.sh ${TAG}_c3 --config c3 --steps 1 --warmup 1 --no-cpu-baseline --no-hbm-roofline \
  > $O/${TAG}_sq_c3.log 2>&1 &&
python3 tools/sq_summary.py gpurun_out/sq_${TAG}_c3 --kernel k_keff_groups_pipe --kernel k_pcg_update_tiles \
  > $O/${TAG}_c3_fast_sq_summary.txt
rc=$?
rm -rf gpurun_out/prof_${TAG}_* gpurun_out/sq_${TAG}_*  # raw traces: > 64 MiB, the summaries above keep what counts
head -30 $O/${TAG}_c3_fast_sq_summary.txt
exit $rc
