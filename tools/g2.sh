source tools/ab.sh
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "fast or shard" > gpurun_out/t.log 2>&1 && tail -1 gpurun_out/t.log &&
run direct   CWF_X=1 python bench.py --no-cpu-baseline &&
run kfold    CWF_FOLD=kernel python bench.py --no-cpu-baseline &&
run notime   CWF_X=1 python bench.py --no-cpu-baseline --keff-sample 100000 &&
run t1       CWF_X=1 python bench.py --no-cpu-baseline --keff-sample 1 &&
run c3       CWF_X=1 python bench.py --no-cpu-baseline --config c3 --steps 3 --warmup 1
