#!/bin/bash
# Round-4 evidence, call B: cfg3 and cfg4.
set -o pipefail
TAG=${1:-r04z}
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash $R/scripts/gpu_r04_evidence.sh $TAG cfg3 20 && bash $R/scripts/gpu_r04_evidence.sh $TAG cfg4 50
