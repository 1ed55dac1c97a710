set -o pipefail
for c in c2 c3; do timeout -k 10 300 python tools/ablate.py --config $c --bits 0 2048 4096 6144 || exit 1; done
