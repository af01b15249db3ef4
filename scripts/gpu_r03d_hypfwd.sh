#!/bin/bash
# QMIX hypernet workgroups appended to the fused forward's grid (default) against hyper_ws_kernel after the forward
# (MQ_HYP_IN_FWD=0): bitwise test, the parity cases, then three interleaved cfg2 rounds and two cfg4 rounds.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "hyper_in_forward or cfg2_trajectory or tiny_full or teacher or wide" > $O/r03d_hypfwd_parity.log 2>&1 || exit $?
echo "parity: $(tail -1 $O/r03d_hypfwd_parity.log)"
for k in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > $O/r03d_hypfwd_on_$k.json 2> $O/r03d_hypfwd_on_$k.err || exit $?
  MQ_HYP_IN_FWD=0 timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > $O/r03d_hypfwd_off_$k.json 2> $O/r03d_hypfwd_off_$k.err || exit $?
  echo "cfg2 round $k done"
done
for k in 1 2; do
  timeout -k 10 200 python bench.py --config cfg4 --steps 100 --warmup 10 --no-cpu-baseline > $O/r03d_hypfwd4_on_$k.json 2> $O/r03d_hypfwd4_on_$k.err || exit $?
  MQ_HYP_IN_FWD=0 timeout -k 10 200 python bench.py --config cfg4 --steps 100 --warmup 10 --no-cpu-baseline > $O/r03d_hypfwd4_off_$k.json 2> $O/r03d_hypfwd4_off_$k.err || exit $?
  echo "cfg4 round $k done"
done
