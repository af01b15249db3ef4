#!/bin/bash
# cfg4 (configs[3] per-GPU shard, R = 320) on the fused BPTT: parity of the cfg4 cases, then interleaved A/B benches
# of the fused BPTT (default) against the round-2 cut-over (MQ_FUSED_BWD_RMAX=256: gru_bwd<2> + dX1 + dW1).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "cfg4" > $O/r03d_cfg4_parity.log 2>&1 || exit $?
echo "cfg4 parity: $(tail -1 $O/r03d_cfg4_parity.log)"
for k in 1 2; do
  timeout -k 10 200 python bench.py --config cfg4 --steps 50 --warmup 5 --no-cpu-baseline --phases > $O/r03d_cfg4_fused_$k.json 2> $O/r03d_cfg4_fused_$k.err || exit $?
  MQ_FUSED_BWD_RMAX=256 timeout -k 10 200 python bench.py --config cfg4 --steps 50 --warmup 5 --no-cpu-baseline --phases > $O/r03d_cfg4_unfused_$k.json 2> $O/r03d_cfg4_unfused_$k.err || exit $?
  echo "round $k done"
done
