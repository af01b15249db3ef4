#!/bin/bash
# Round 4a: the data-parallel contract tests (global sample, pre-sharded rejection, COMA chain-fault rollback on
# every rank), then the cfg5 exit-crash reproduction under rocprofv3 with the process mappings dumped.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_dp.py \
  > $O/r04a_dp_tests.log 2>&1 || { echo "dp tests failed"; tail -30 $O/r04a_dp_tests.log; exit 1; }
tail -12 $O/r04a_dp_tests.log
bash scripts/gpu_r04_segv.sh r04a
tail -40 $O/prof_r04a_cfg5.log
