#!/bin/bash
# Timing-only A/B of MQ_BWD_VAR values (diagnostic variants allowed): bash scripts/ab_vars.sh "772 1796"
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
for round in 1 2; do
  for v in $1; do
    MQ_BWD_VAR=$v timeout -k 10 200 python $R/bench.py --steps 50 --warmup 5 --no-cpu-baseline --phases \
      > $R/gpurun_out/abv_${v}_${round}.json 2> $R/gpurun_out/abv_${v}_${round}.err || exit $?
  done
done
for f in $R/gpurun_out/abv_*_1.err; do echo $(basename $f) $(grep -o '"gru_bwd": [0-9.]*' $f); done
for f in $R/gpurun_out/abv_*_2.err; do echo $(basename $f) $(grep -o '"gru_bwd": [0-9.]*' $f); done
