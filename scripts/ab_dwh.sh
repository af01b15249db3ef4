#!/bin/bash
# A/B of dW_hyper on the side stream beside the fused BPTT (MQ_DWH_OVERLAP=1) vs in stream order (default), cfg2,
# interleaved rounds.
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
for round in 1 2 3; do
  for v in 1 0; do
    MQ_DWH_OVERLAP=$v timeout -k 10 200 python $R/bench.py --steps 100 --warmup 5 --no-cpu-baseline --phases \
      > $R/gpurun_out/abd_${v}_${round}.json 2> $R/gpurun_out/abd_${v}_${round}.err || exit $?
  done
done
