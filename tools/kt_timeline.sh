#!/bin/bash
# rocprofv3 kernel trace of a short bench run per config, then the per-kernel averages and launch gaps
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp
for c in ${CFGS:-c3 c2}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/kt_$c -o kt -- python3 $R/bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-hbm-roofline > $R/gpurun_out/kt_$c.log 2>&1 || exit 1
  echo "== $c"; python3 $R/tools/kt_gaps.py $R/gpurun_out/kt_$c --last ${LAST:-600} || exit 1
done
