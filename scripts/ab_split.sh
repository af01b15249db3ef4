#!/bin/bash
# Parity + A/B of a fused-BPTT variant: bash scripts/ab_split.sh VAR
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
V=${1:-1792}
mkdir -p $R/gpurun_out
MQ_BWD_VAR=$V timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu $R/tests/test_gpu_parity.py -k "teacher_forced and not unfused" > $R/gpurun_out/ab_parity_$V.log 2>&1 || exit $?
bash $R/scripts/ab_env.sh MQ_BWD_VAR=$V || exit $?
