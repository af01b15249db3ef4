#!/bin/bash
# Round-4 evidence, call A: GPU suite, smoke, cfg2 evidence.
set -o pipefail
TAG=${1:-r04z}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export MQ_PARITY_DIR=$O/parity_${TAG}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu $R/tests > $O/gpu_all_$TAG.log 2>&1 || { tail -20 $O/gpu_all_$TAG.log; exit 1; }
tail -2 $O/gpu_all_$TAG.log
timeout -k 10 200 python -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke()" > $O/smoke_$TAG.log 2>&1 || { tail -5 $O/smoke_$TAG.log; exit 1; }
bash $R/scripts/gpu_r04_evidence.sh $TAG cfg2 50
