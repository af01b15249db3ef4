#!/bin/bash
# Reduction pass 2 fused with RMSprop (mq_train_step): bitwise test against the two-launch path and the parity
# cases it touches, then interleaved cfg2 A/B benches (MQ_FUSED_APPLY=0 is the two-launch path).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "fused_pass2_apply or tiny_full or cfg2_trajectory" > $O/r03d_apply_parity.log 2>&1 || exit $?
echo "parity: $(tail -1 $O/r03d_apply_parity.log)"
for k in 1 2; do
  timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --phases > $O/r03d_apply_fused_$k.json 2> $O/r03d_apply_fused_$k.err || exit $?
  MQ_FUSED_APPLY=0 timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --phases > $O/r03d_apply_twolaunch_$k.json 2> $O/r03d_apply_twolaunch_$k.err || exit $?
  echo "round $k done"
done
