#!/bin/bash
# 1-GPU rehearsal of the multi-rank bench path: 2 ranks under torch.distributed.run share cuda:0
# (slab shards, RCCL communicator, halo + scalar all-gathers, max-over-ranks timing).
set -o pipefail
mkdir -p gpurun_out/mr
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 > gpurun_out/mr/bench_n2.log 2>&1
rc=$?
tail -30 gpurun_out/mr/bench_n2.log
exit $rc
