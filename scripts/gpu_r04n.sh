#!/bin/bash
# Round 4n: where hymix_kernel's time goes: cfg2 with the hypernet part only (exp1) / the mixer part only (exp2).
set -o pipefail
TAG=${1:-r04n}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
for v in 1 2; do
  MQ_LEARNER_LIB=$R/exp/libmq_exp$v.so MQ_HYMIX=1 timeout -k 10 300 python bench.py --config cfg2 --steps 30 --warmup 5 --phases --no-cpu-baseline > $O/bench_${TAG}_exp$v.json 2> $O/bench_${TAG}_exp$v.err || { tail -5 $O/bench_${TAG}_exp$v.err; exit 1; }
  tail -1 $O/bench_${TAG}_exp$v.err
done
