# A/B runs of bench.py variants on the GPU box; each line: label, env, args
set -o pipefail
mkdir -p gpurun_out
run() { local tag=$1; shift; timeout -k 10 240 env "$@" > gpurun_out/ab_$tag.log 2>&1 || { echo "FAIL $tag"; tail -5 gpurun_out/ab_$tag.log; exit 1; }; python3 -c "
import json,sys; d=json.loads(open('gpurun_out/ab_$tag.log').read().strip().splitlines()[-1]); r=d['roofline']
print('%-14s it/s %8.1f  ms/step %7.2f  keff %.2f us  frac %.3f  refequiv %.0f GB/s' % ('$tag', d['pcg_iterations_per_sec'], d['ms_per_step'], r['avg_launch_ms']*1e3, r['frac'] or 0, r['reference_layout_equiv_gbs'] or 0))"; }
