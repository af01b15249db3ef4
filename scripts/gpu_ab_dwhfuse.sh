#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu $R/tests/test_gpu_parity.py -k "dwh or teacher_forced and (cfg2_qmix or tiny)" > $R/gpurun_out/dwhfuse_tests.log 2>&1 || exit $?
bash $R/scripts/ab_env.sh MQ_DWH_UNFUSED=1 || exit $?
