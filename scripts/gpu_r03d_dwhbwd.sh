#!/bin/bash
# dW_hyper tiles appended to the fused BPTT's grid (default for R > CUs) against dW_hyper in the reduction's launch
# (MQ_DWH_IN_BWD=0): bitwise test and parity cases, then interleaved cfg4 rounds and a forced-on cfg2 pair.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "dwh or hyper_in_forward or cfg2_trajectory or tiny_full or teacher or wide" > $O/r03d_dwhbwd_parity.log 2>&1 || exit $?
echo "parity: $(tail -1 $O/r03d_dwhbwd_parity.log)"
for k in 1 2 3; do
  timeout -k 10 200 python bench.py --config cfg4 --steps 100 --warmup 10 --no-cpu-baseline > $O/r03d_dwhbwd4_on_$k.json 2> $O/r03d_dwhbwd4_on_$k.err || exit $?
  MQ_DWH_IN_BWD=0 timeout -k 10 200 python bench.py --config cfg4 --steps 100 --warmup 10 --no-cpu-baseline > $O/r03d_dwhbwd4_off_$k.json 2> $O/r03d_dwhbwd4_off_$k.err || exit $?
  echo "cfg4 round $k done"
done
for k in 1 2; do
  MQ_DWH_IN_BWD=1 timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > $O/r03d_dwhbwd2_on_$k.json 2> $O/r03d_dwhbwd2_on_$k.err || exit $?
  timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > $O/r03d_dwhbwd2_off_$k.json 2> $O/r03d_dwhbwd2_off_$k.err || exit $?
  echo "cfg2 round $k done"
done
