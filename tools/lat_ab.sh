#!/bin/bash
# A/B of lattice builds (CWF_LIB_PATH) and the fan groups (CWF_LATTICE=0) on C2 and C3: spmv_bench K_eff and it/s
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd $R
for pass in 1 2; do
for cfg in c2 c3; do
  for lib in ${LIBS:-libcwf_hip.so}; do
    CWF_LIB_PATH=$R/civiwave-fem_amd/lib/$lib timeout -k 10 200 python tools/spmv_bench.py --config $cfg --iters 200 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$pass $cfg $lib', 'keff', round(d['keff_pcg_us'],1), 'it/s', round(d['pcg_it_per_s']), 'apply', round(d['apply_keff_us'],1))" || exit 1
  done
  [ -n "$NO_GROUPS" ] || CWF_LATTICE=0 timeout -k 10 200 python tools/spmv_bench.py --config $cfg --iters 200 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$pass $cfg groups', 'keff', round(d['keff_pcg_us'],1), 'it/s', round(d['pcg_it_per_s']))" || exit 1
done
done
