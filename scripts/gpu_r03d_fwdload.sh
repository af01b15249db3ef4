#!/bin/bash
# Fused BPTT prologue: one 16-byte W_hh^T load per row and lane (default) against one dword per weight
# (MQ_BWD_VAR=344832 = production 82688 + 262144), three interleaved cfg2 rounds, after the parity cases.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "cfg2_trajectory or tiny_full or wide_batch" > $O/r03d_fwdload_parity.log 2>&1 || exit $?
echo "parity: $(tail -1 $O/r03d_fwdload_parity.log)"
for k in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --phases > $O/r03d_fwdload_x4_$k.json 2> $O/r03d_fwdload_x4_$k.err || exit $?
  MQ_BWD_VAR=344832 timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --phases > $O/r03d_fwdload_dw_$k.json 2> $O/r03d_fwdload_dw_$k.err || exit $?
  echo "round $k done"
done
