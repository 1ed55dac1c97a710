#!/bin/bash
# GPU-box entry point for the maintained runs (each GPU step under its own time limit, stop at the first
# failure). usage: bash tools/gpu.sh SUBCOMMAND [args]
#   tests [pytest -k expr]     the GPU suite (-m gpu), log in gpurun_out/tests.log
#   bench CFG [bench args]     one bench.py line for config CFG (c2 c3 c4 c5), JSON in gpurun_out/bench_CFG.json
#   ab VARIANT...              GPU suite, then same-box A/B: in-tree lib vs civiwave-fem_amd/lib_VARIANT (tools/ab_lib.sh)
#   configs                    smoke(), then the C4 / C5 single-GPU lines
#   multirank N                N ranks of bench.py under torch.distributed.run sharing cuda:0 (RCCL refuses
#                              duplicate GPUs past communicator init; rehearses sharding + systems only)
#   round TAG                  the full evidence pass (tools/gpu_round.sh)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
cmd=$1; shift
case "$cmd" in
  tests)
    timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${1:+-k "$1"} \
      > gpurun_out/tests.log 2>&1; rc=$?
    tail -3 gpurun_out/tests.log
    [ $rc -eq 0 ] || grep -E "FAILED|Error|assert" gpurun_out/tests.log | head -20
    exit $rc ;;
  bench)
    cfg=${1:-c2}; shift
    timeout -k 10 700 python -u bench.py --config "$cfg" "$@" > gpurun_out/bench_$cfg.log 2>&1 &&
      tail -1 gpurun_out/bench_$cfg.log | tee gpurun_out/bench_$cfg.json ;;
  ab)
    bash "$0" tests || exit $?
    bash tools/ab_lib.sh "$@" ;;
  configs)
    timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
      tail -1 gpurun_out/smoke.log &&
      bash "$0" bench c4 --steps 3 --warmup 1 --no-cpu-baseline &&
      bash "$0" bench c5 --steps 2 --warmup 1 --no-cpu-baseline ;;
  multirank)
    n=${1:-2}
    timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$n" --master-addr 127.0.0.1 \
      --master-port 29533 bench.py --gpus "$n" --steps 3 --warmup 1 > gpurun_out/bench_n$n.log 2>&1; rc=$?
    tail -30 gpurun_out/bench_n$n.log
    exit $rc ;;
  round)
    bash tools/gpu_round.sh "$@" ;;
  *)
    sed -n 2,12p "$0"; exit 2 ;;
esac
