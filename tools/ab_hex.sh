# Same-box A/B of the hex8 bench: the in-tree lib against civiwave-fem_amd/lib_<v> (usage: bash tools/ab_hex.sh base)
source tools/ab.sh
for pass in 1 2; do
  run hex_new_$pass X=1 python bench.py --element hex8 --no-cpu-baseline || exit 1
  for v in "$@"; do
    run hex_${v}_$pass CWF_LIB_PATH=$PWD/civiwave-fem_amd/lib_$v/libcwf_hip.so python bench.py --element hex8 --no-cpu-baseline || exit 1
  done
done
