#!/bin/bash
# Same-box A/B of the per-iteration time of one structured-block solve (tools/block_iter_time.py) between the in-tree
# library and civiwave-fem_amd/lib_VARIANT/libcwf_hip.so, PASSES (default 3) alternating passes.
#   bash tools/ab_iter.sh VARIANT NX NY NZ [ITERATIONS] [SCHEDULES]
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
V=$1; NX=$2; NY=$3; NZ=$4; IT=${5:-300}; export BLK_SCHEDULES=${6:-resident}
for pass in $(seq 1 ${PASSES:-3}); do
  timeout -k 10 120 python -u tools/block_iter_time.py $NX $NY $NZ $IT 2>/dev/null | sed "s/^/new  p$pass /" || exit 1
  CWF_LIB_PATH=$R/civiwave-fem_amd/lib_$V/libcwf_hip.so timeout -k 10 120 python -u tools/block_iter_time.py $NX $NY $NZ $IT 2>/dev/null | sed "s/^/$V p$pass /" || exit 1
done
