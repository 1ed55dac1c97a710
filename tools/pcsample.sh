#!/bin/bash
# rocprofv3 stochastic PC sampling of one bench config (where the waves of the hot kernels stall).
# usage: bash tools/pcsample.sh TAG [bench args]; lists the box's PC-sampling configurations first.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=${1:-pcs}; shift
ARGS=${@:-"--config c3 --steps 1 --warmup 1 --no-cpu-baseline --no-hbm-roofline"}
cd /tmp && export TMPDIR=/tmp
OUT=$R/gpurun_out/pcs_$TAG
mkdir -p $OUT
timeout -k 10 60 rocprofv3 -L > $OUT/list.txt 2>&1
grep -i -A12 "pc.sampl\|PC Sampling" $OUT/list.txt | head -40
timeout -k 10 400 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles \
  --pc-sampling-interval ${PCS_INTERVAL:-65536} --output-format csv -d $OUT/pcs -o pcs -- python3 $R/bench.py $ARGS \
  > $OUT/bench.log 2>&1
rc=$?
tail -3 $OUT/bench.log
find $OUT -name "*.csv" | head
exit $rc
