#!/bin/bash
# cfg4 (R = 320): fused forward (640 row-nets, two per CU: two waves) against the unfused forward
# (fc1 / GI GEMMs + gru_fwd<1> + fc2), interleaved.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
for k in 1 2; do
  timeout -k 10 200 python bench.py --config cfg4 --steps 50 --warmup 5 --no-cpu-baseline --phases > $O/r03d_cfg4fwd_fused_$k.json 2> $O/r03d_cfg4fwd_fused_$k.err || exit $?
  MQ_UNFUSED_FWD=1 timeout -k 10 200 python bench.py --config cfg4 --steps 50 --warmup 5 --no-cpu-baseline --phases > $O/r03d_cfg4fwd_unfused_$k.json 2> $O/r03d_cfg4fwd_unfused_$k.err || exit $?
  echo "round $k done"
done
