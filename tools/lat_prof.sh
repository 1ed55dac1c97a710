#!/bin/bash
# lattice kernel on one config: spmv_bench timing (lattice and fan groups), rocprofv3 kernel stats and two SQ passes
# usage: tools/lat_prof.sh TAG [config]
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=${1:-lat}; CFG=${2:-c3}
OUT=$R/gpurun_out/latprof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 python3 $R/tools/spmv_bench.py --config $CFG --iters 100 > $OUT/spmv_lat.json 2>$OUT/spmv_lat.err && cat $OUT/spmv_lat.json &&
CWF_LATTICE=0 timeout -k 10 200 python3 $R/tools/spmv_bench.py --config $CFG --iters 100 > $OUT/spmv_grp.json 2>$OUT/spmv_grp.err && cat $OUT/spmv_grp.json &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 $R/tools/spmv_bench.py --config $CFG --iters 100 > $OUT/kt.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAVES --output-format csv -d $OUT/p1 -o p1 -- python3 $R/tools/spmv_bench.py --config $CFG --iters 100 > $OUT/p1.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM SQ_BUSY_CYCLES --output-format csv -d $OUT/p2 -o p2 -- python3 $R/tools/spmv_bench.py --config $CFG --iters 100 > $OUT/p2.log 2>&1 &&
python3 $R/tools/sq_summary.py $OUT --kernel k_keff_lattice --kernel k_pcg_update
rc=$?
find $OUT/kt -name "*kernel_stats.csv" -exec head -8 {} \;
exit $rc
