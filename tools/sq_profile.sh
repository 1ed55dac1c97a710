#!/bin/bash
# SQ counter passes (one rocprofv3 run per pass) over bench.py: where the waves of each kernel spend
# their cycles. Usage: tools/sq_profile.sh TAG [bench args]
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=${1:-run}; shift
ARGS=${@:-"--steps 2 --warmup 1 --no-cpu-baseline"}
cd /tmp && export TMPDIR=/tmp
OUT=$R/gpurun_out/sq_$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAVES --output-format csv -d $OUT/p1 -o p1 -- python3 $R/bench.py $ARGS > $OUT/p1.log 2>&1 || { echo "sq pass 1 failed"; tail -20 $OUT/p1.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES --output-format csv -d $OUT/p2 -o p2 -- python3 $R/bench.py $ARGS > $OUT/p2.log 2>&1 || { echo "sq pass 2 failed"; tail -20 $OUT/p2.log; exit 2; }
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum --output-format csv -d $OUT/p3 -o p3 -- python3 $R/bench.py $ARGS > $OUT/p3.log 2>&1 || { echo "tcc pass failed"; tail -20 $OUT/p3.log; exit 3; }
echo "sq passes done: $OUT"
