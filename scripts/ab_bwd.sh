#!/bin/bash
# A/B of the fused-BPTT schedule variants in the real cfg2 pipeline (MQ_BWD_VAR), interleaved rounds.
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
for round in 1 2; do
  for v in ${VARS:-0 128 256 384}; do
    MQ_BWD_VAR=$v timeout -k 10 200 python $R/bench.py --steps 50 --warmup 5 --no-cpu-baseline --phases \
      > $R/gpurun_out/abb_${v}_${round}.json 2> $R/gpurun_out/abb_${v}_${round}.err || exit $?
  done
done
