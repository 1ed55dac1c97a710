# A/B of the in-tree library against civiwave-fem_amd/lib_base/libcwf_hip.so (CWF_LIB_PATH), same box
source tools/ab.sh
B=CWF_LIB_PATH=$PWD/civiwave-fem_amd/lib_base/libcwf_hip.so
run c2_base $B python bench.py --no-cpu-baseline &&
run c2_new X=1 python bench.py --no-cpu-baseline &&
run c3_base $B python bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline &&
run c3_new X=1 python bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline &&
run c2_base2 $B python bench.py --no-cpu-baseline &&
run c2_new2 X=1 python bench.py --no-cpu-baseline &&
run hex_base $B python bench.py --element hex8 --no-cpu-baseline &&
run hex_new X=1 python bench.py --element hex8 --no-cpu-baseline
