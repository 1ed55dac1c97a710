#!/bin/bash
# One parameterised GPU-box runner (replaces the per-round one-off command scripts). Every step runs under its own
# time limit and the steps are chained: the first failure ends the call. Outputs go to gpurun_out/<TAG>_*.
#
#   bash tools/gpu_run.sh TAG STEP [STEP ...]
#
# STEP is one of
#   tests[:FILE,FILE..[:KEXPR]]  pytest -m gpu -s over tests/ (or the listed test files; KEXPR: a -k expression,
#                           commas for spaces; no '::' node ids, ':' splits the step)
#   smoke                   __graft_entry__.smoke()
#   bench:NAME[:ARGS]       one bench.py line (ARGS: bench.py arguments, commas for spaces) -> <TAG>_bench_NAME.json
#   ab:NAME:ENV[:ARGS]      the same bench twice per pass, in-tree default vs ENV (commas for spaces: several
#                           VAR=VALUE), PASSES (default 2) alternating passes -> one summary line per run
#   ablib:NAME:VARIANT[:ARGS]  the same against civiwave-fem_amd/lib_VARIANT/libcwf_hip.so
#   prof:NAME[:ARGS]        rocprofv3 kernel trace + FETCH_SIZE / WRITE_SIZE passes (tools/profile.sh) and the
#                           K_eff kernel's summary (tools/pmc_summary.py) -> <TAG>_NAME_{summary.txt,pmc.json,...}
#   sq:NAME[:ARGS]          the SQ counter pass of the same (tools/profile.sh SQ_PMC=1)
#   calib                   FETCH_SIZE / WRITE_SIZE against known byte counts (tools/pmc_calib, built in-tree
#                           beforehand) -> <TAG>_calib.json
#   n2:NAME[:ARGS]          bench.py --gpus 2 under torch.distributed.run, both ranks on this GPU (a rehearsal of the
#                           driver's N>1 flow: the PEER communicator maps the other process's mailbox on the same
#                           device) -> <TAG>_n2_NAME.json
#   peer                    the PEER communicator's tests with their exchange-latency prints (2 / 3 processes on
#                           this GPU) -> <TAG>/peer.log
# e.g. bash tools/gpu_run.sh r04c tests:tests/test_gpu_lattice.py bench:c2 bench:c3:--config,c3,--steps,3 \
#        ab:c2cg:CWF_LAT_CG=0 prof:c3:--config,c3,--steps,2,--warmup,1,--no-cpu-baseline
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
sp() { echo "${1//,/ }"; }
line() {  # summary of one bench log
  python3 -c "
import json, sys
d = [json.loads(l) for l in open('$1') if l.startswith('{\"metric\"')][0]; r = d['roofline']
g = d.get('general') or {}
print('%-22s %9.0f it/s %7.2f G DOF-it/s  %7.2f ms/step  keff %7.2f us  frac %.3f  conv %s/%s  %s%s' % ('$2',
      d['pcg_iterations_per_sec'], d['value'] / 1e9, d['ms_per_step'], r['avg_launch_ms'] * 1e3, r['frac'] or 0,
      d['steps_converged'], d['steps'], r['kernel'],
      ('  general %.0f it/s' % g['pcg_iterations_per_sec']) if g else ''))"
}
bench() {  # NAME ENV ARGS
  local name=$1 envs=$2; shift 2
  timeout -k 10 400 env $envs python -u bench.py "$@" > $O/${name}.log 2>&1 || { echo "FAIL $name"; tail -20 $O/${name}.log; return 1; }
  grep '^{"metric"' $O/${name}.log > $O/${name}.json && line $O/${name}.log $name
}
for step in "$@"; do
  IFS=: read -r kind a b c <<< "$step"
  case $kind in
    tests)
      files=$(sp "${a:-tests}")
      kx=(); [ -n "$b" ] && kx=(-k "$(sp "$b")")
      timeout -k 10 900 python -u -m pytest $files "${kx[@]}" -m gpu -v -s --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
      rc=$?; tail -1 $O/gpu_tests.log
      [ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $O/gpu_tests.log | head -30; exit $rc; } ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
      tail -1 $O/smoke.log ;;
    bench)
      bench bench_$a "" $(sp "$b") || exit 2 ;;
    ab|ablib)
      for pass in $(seq 1 ${PASSES:-2}); do
        bench ${a}_new_p$pass "" --no-cpu-baseline --no-hbm-roofline --no-general-roofline --no-general $(sp "$c") || exit 2
        if [ $kind = ab ]; then other=$(sp "$b"); else other="CWF_LIB_PATH=$R/civiwave-fem_amd/lib_$b/libcwf_hip.so"; fi
        bench ${a}_alt_p$pass "$other" --no-cpu-baseline --no-hbm-roofline --no-general-roofline --no-general $(sp "$c") || exit 2
      done ;;
    prof|sq)
      args=$(sp "${b:---steps,3,--warmup,1,--no-cpu-baseline}")
      if [ $kind = sq ]; then export SQ_PMC=1; fi
      bash tools/profile.sh ${TAG}_$a $args > $O/prof_$a.log 2>&1 || { tail -20 $O/prof_$a.log; exit 3; }
      K=$(grep -h '^{"metric"' gpurun_out/prof_${TAG}_$a/bench_kt.log | python3 -c "import json,sys; print(json.loads(sys.stdin.read())['roofline']['kernel'])")
      python3 tools/pmc_summary.py gpurun_out/prof_${TAG}_$a --kernel "$K" --json $O/${a}_pmc.json > $O/${a}_summary.txt || exit 3
      cp gpurun_out/prof_${TAG}_$a/kt/kt_kernel_stats.csv $O/${a}_kernel_stats.csv
      grep '^{"metric"' gpurun_out/prof_${TAG}_$a/bench_kt.log > $O/${a}_bench_under_rocprof.json
      if [ $kind = sq ]; then python3 tools/sq_summary.py gpurun_out/prof_${TAG}_$a --kernel "$K" > $O/${a}_sq_summary.txt; unset SQ_PMC; fi
      rm -rf gpurun_out/prof_${TAG}_$a
      head -6 $O/${a}_summary.txt ;;
    calib)
      C=$R/gpurun_out/calib_$TAG; mkdir -p $C
      (cd /tmp && export TMPDIR=/tmp &&
       timeout -k 10 120 $R/tools/pmc_calib > $C/known.json &&
       timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $C/fetch -o fetch -- $R/tools/pmc_calib > /dev/null &&
       timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $C/write -o write -- $R/tools/pmc_calib > /dev/null) || exit 4
      python3 tools/pmc_calib.py $C > $O/calib.txt && cp $C/calib.json $O/calib.json && cat $O/calib.txt || exit 4
      rm -rf $C ;;
    peer)
      timeout -k 10 300 python -u -m pytest tests/test_gpu_peer.py -m gpu -s -q --timeout 280 --timeout-method thread \
        > $O/peer.log 2>&1 || { tail -30 $O/peer.log; exit 5; }
      grep -E "PEER exchange|passed|failed" $O/peer.log ;;
    n2)
      timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port 29517 bench.py --gpus 2 $(sp "$b") > $O/n2_$a.log 2>&1 || { echo "FAIL n2_$a"; tail -20 $O/n2_$a.log; exit 2; }
      grep '^{"metric"' $O/n2_$a.log > $O/n2_$a.json && line $O/n2_$a.log n2_$a ;;
    *) echo "unknown step $step"; exit 64 ;;
  esac
done
