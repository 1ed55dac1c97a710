#!/bin/bash
# round 3: C3 fan-group tile width A/B (256 vs 128 lanes), same box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
CONFIGS=c3 PASSES=2 bash tools/ab_env.sh "nt256=CWF_GROUP_NT=256" "nt128=CWF_GROUP_NT=128"
