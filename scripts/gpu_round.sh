#!/bin/bash
# One GPU-box evidence pass: GPU suite, smoke, cfg2 bench + rocprofv3 kernel stats (+ the counter list).
# Usage: bash scripts/gpu_round.sh TAG [suite|nosuite]
set -o pipefail
TAG=${1:-r02}; SUITE=${2:-suite}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
if [ "$SUITE" = suite ]; then
  timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu $R/tests > $O/gpu_all_$TAG.log 2>&1 || exit $?
  timeout -k 10 120 python -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke()" > $O/smoke_$TAG.log 2>&1 || exit $?
fi
bash $R/scripts/gpu_bench_prof.sh $TAG cfg2 || exit $?
