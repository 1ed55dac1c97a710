# Same-box A/B of the native hex8 path: in-tree lib vs civiwave-fem_amd/lib_base (C2, C3; PASSES, default 2)
source tools/ab.sh
B=$PWD/civiwave-fem_amd/lib_base/libcwf_hip.so
for pass in $(seq 1 ${PASSES:-2}); do
  run c2h_new_$pass X=1 python bench.py --element hex8 --no-cpu-baseline || exit 1
  run c2h_base_$pass CWF_LIB_PATH=$B python bench.py --element hex8 --no-cpu-baseline || exit 1
  run c3h_new_$pass X=1 python bench.py --element hex8 --config c3 --steps 3 --warmup 1 --no-cpu-baseline || exit 1
  run c3h_base_$pass CWF_LIB_PATH=$B python bench.py --element hex8 --config c3 --steps 3 --warmup 1 --no-cpu-baseline || exit 1
done
