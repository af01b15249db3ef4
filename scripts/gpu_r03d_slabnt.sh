#!/bin/bash
# Fused BPTT slab stores: non-temporal (default) against plain (MQ_BWD_VAR=606976 = production 82688 + 524288),
# three interleaved cfg2 rounds, after the parity cases.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "cfg2_trajectory or tiny_full or teacher" > $O/r03d_slabnt_parity.log 2>&1 || exit $?
echo "parity: $(tail -1 $O/r03d_slabnt_parity.log)"
for k in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --phases > $O/r03d_slabnt_nt_$k.json 2> $O/r03d_slabnt_nt_$k.err || exit $?
  MQ_BWD_VAR=606976 timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --phases > $O/r03d_slabnt_plain_$k.json 2> $O/r03d_slabnt_plain_$k.err || exit $?
  echo "round $k done"
done
