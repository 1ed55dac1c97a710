#!/bin/bash
# rocprofv3 passes over the bench command: kernel trace + stats, then separate PMC passes
# (FETCH_SIZE and WRITE_SIZE cannot share one pass on gfx950). Usage: tools/profile.sh TAG [bench args]
# SCRIPT=tools/spmv_bench.py profiles that script instead of bench.py (args likewise).
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=${1:-run}; shift
ARGS=${@:-"--steps 3 --warmup 1 --no-cpu-baseline"}
SCRIPT=$R/${SCRIPT:-bench.py}
cd /tmp && export TMPDIR=/tmp
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 $SCRIPT $ARGS > $OUT/bench_kt.log 2>&1 || { echo "kt pass failed"; tail -20 $OUT/bench_kt.log; exit 1; }
tail -1 $OUT/bench_kt.log
if [ -n "$NO_PMC" ]; then exit 0; fi
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o fetch -- python3 $SCRIPT $ARGS > $OUT/bench_fetch.log 2>&1 || { echo "fetch pass failed"; tail -20 $OUT/bench_fetch.log; exit 2; }
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o write -- python3 $SCRIPT $ARGS > $OUT/bench_write.log 2>&1 || { echo "write pass failed"; tail -20 $OUT/bench_write.log; exit 3; }
if [ -n "$SQ_PMC" ]; then
  timeout -k 10 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM --output-format csv -d $OUT/sq -o sq -- python3 $SCRIPT $ARGS > $OUT/bench_sq.log 2>&1 || { echo "sq pass failed"; tail -20 $OUT/bench_sq.log; exit 4; }
fi
find $OUT -name "*.csv" | head -20
