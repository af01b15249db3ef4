#!/bin/bash
# Round 4i: cfg3 PMC at the split row-tile kernels: stall / LDS / MFMA diag pass, then HBM bytes.
set -o pipefail
TAG=${1:-r04i}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash scripts/gpu_diag.sh $TAG cfg3 || exit $?
bash scripts/gpu_counters.sh $TAG cfg3 || exit $?
