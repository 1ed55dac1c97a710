#!/bin/bash
# The driver's N > 1 bench flow rehearsed on one GPU (processes share the device, so the rates are protocol figures,
# not xGMI ones): 4 ranks of C1 weak (middle ranks with two neighbours) and 2 ranks of C2 hex8 strong, both through
# --comm auto (PEER after the trial solve; the resident solve on every rank, schedule 3). Outputs gpurun_out/r06t/.
set -o pipefail
mkdir -p gpurun_out/r06t
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 4 --config c1 --steps 5 --warmup 1 > gpurun_out/r06t/n4_c1.log 2>&1 && \
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29521 bench.py --gpus 2 --config c2 --scaling strong --element hex8 --steps 5 --warmup 1 > gpurun_out/r06t/n2_c2hex_strong.log 2>&1
