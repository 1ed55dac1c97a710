cd $GRAFT_REPO_ROOT
for cap in 2048 1024 512; do for c in c2 c3; do
CWF_UPD_CAP=$cap timeout -k 10 200 python tools/spmv_bench.py --config $c --iters 200 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('cap $cap $c', 'keff', round(d['keff_pcg_us'],1), 'it/s', round(d['pcg_it_per_s']))" || exit 1
done; done
