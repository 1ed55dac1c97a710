# Same-box A/B of environment switches on the in-tree lib (and optional saved libs):
# usage: bash tools/ab_env.sh "LABEL=ENV ..." ... ; CONFIGS (default "c2 c3"), PASSES (default 2)
source tools/ab.sh
for pass in $(seq 1 ${PASSES:-2}); do
  for cfg in ${CONFIGS:-c2 c3}; do
    extra="--config $cfg"; [ $cfg = c3 ] && extra="--config c3 --steps 3 --warmup 1"
    for spec in "$@"; do
      label=${spec%%=*}; envs=${spec#*=}
      run ${cfg}_${label}_$pass $envs python bench.py --no-cpu-baseline $extra || exit 1
    done
  done
done
