#!/bin/bash
# round 3: the driver's N>1 bench flow rehearsed on one GPU: 2 ranks under torch.distributed.run, the RCCL code
# path over the host-staged test transport (numbers are not performance figures: the transport is host memory)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export CWF_RCCL_LIB=$PWD/tests/transport/libcwf_host_nccl.so
run() {
  local name=$1; shift
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port $((29500 + RANDOM % 1000)) bench.py --gpus 2 --no-cpu-baseline "$@" > gpurun_out/n2_${name}.log 2>&1
  local rc=$?
  grep '"metric"' gpurun_out/n2_${name}.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.readline())
print('$name', d['n_gpus'], d['scaling'], d['config']['parallelism'], 'it', d['pcg_iterations'], 'conv', d.get('steps_converged'), [ (r['owned_dofs'], r['halo_nodes']) for r in d['ranks']])" || tail -20 gpurun_out/n2_${name}.log
  return $rc
}
run c2_weak --steps 2 --warmup 1 &&
run c3_strong --config c3 --scaling strong --steps 1 --warmup 0 &&
run c4_rcb --config c4 --steps 1 --warmup 0 &&
run c2_hex8 --element hex8 --steps 1 --warmup 0
