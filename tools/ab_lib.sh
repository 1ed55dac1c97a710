# Same-box A/B of library builds: the in-tree lib ("new") against civiwave-fem_amd/lib_<v>/libcwf_hip.so for
# each variant v given on the command line (CWF_LIB_PATH). usage: bash tools/ab_lib.sh base [noslp ...]
# CONFIGS (default "c2 c3") and PASSES (default 2) override the sweep.
source tools/ab.sh
for pass in $(seq 1 ${PASSES:-2}); do
  for cfg in ${CONFIGS:-c2 c3}; do
    extra="--config $cfg"; [ $cfg = c3 ] && extra="--config c3 --steps 3 --warmup 1"
    run ${cfg}_new_$pass X=1 python bench.py --no-cpu-baseline $extra || exit 1
    for v in "$@"; do
      run ${cfg}_${v}_$pass CWF_LIB_PATH=$PWD/civiwave-fem_amd/lib_$v/libcwf_hip.so python bench.py --no-cpu-baseline $extra || exit 1
    done
  done
done
