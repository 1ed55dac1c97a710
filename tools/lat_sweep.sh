#!/bin/bash
# lattice kernel: PCG-loop K_eff time on C3 for several planes-per-work-item (CWF_LAT_L), then SQ counters
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd $R
CFG=${1:-c3}
for L in ${LS:-3 6 10 20}; do
  CWF_LAT_L=$L timeout -k 10 200 python tools/spmv_bench.py --config $CFG --iters 100 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('L=$L', 'keff_pcg_us', round(d['keff_pcg_us'],1), 'it/s', round(d['pcg_it_per_s']))" || exit 1
done
[ -n "$NO_SQ" ] && exit 0
OUT=$R/gpurun_out/latsq_$CFG; mkdir -p $OUT; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAVES --output-format csv -d $OUT/p1 -o p1 -- python3 $R/tools/spmv_bench.py --config $CFG --iters 100 > $OUT/p1.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM SQ_BUSY_CYCLES --output-format csv -d $OUT/p2 -o p2 -- python3 $R/tools/spmv_bench.py --config $CFG --iters 100 > $OUT/p2.log 2>&1 &&
python3 $R/tools/sq_summary.py $OUT --kernel "k_keff_lattice<1"
