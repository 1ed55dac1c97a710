#!/bin/bash
# LDS instruction / bank-conflict counters of the PCG-mode fan-group kernel (CFG, default c3) (timed loop of tools/ablate.py)
# with phases ablated (bits: 64 = no element math/push, 128 = no fold). usage: bash tools/lds_ablate.sh [bits..]
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp
for b in ${@:-0 128 64}; do
  OUT=$R/gpurun_out/lds_$b
  mkdir -p $OUT
  timeout -k 10 240 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES --output-format csv -d $OUT -o p -- python3 $R/tools/ablate.py --config ${CFG:-c3} --bits $b > $OUT/run.log 2>&1 || { echo "pass $b failed"; tail -5 $OUT/run.log; exit 1; }
  python3 - $OUT $b <<'PY'
import csv, glob, sys, collections
out, b = sys.argv[1], sys.argv[2]
f = glob.glob(out + '/**/*counter_collection*.csv', recursive=True)
acc = collections.defaultdict(float); n = collections.Counter()
for path in f:
    for row in csv.DictReader(open(path)):
        if 'k_keff_groups_pipe<true, false, 1' not in row.get('Kernel_Name', ''):
            continue
        acc[row['Counter_Name']] += float(row['Counter_Value'])
        n[row['Counter_Name']] += 1
print('ablate', b, {k: round(v / max(1, n[k]) * 1.0) for k, v in sorted(acc.items())})
PY
done
