#!/bin/bash
# Round 4r: s_setprio A/B on the row-tile kernels (exp2/libmq_prio{A,B}.so: A = the recurrence / chain roles at
# priority 2, B = the projection / weight-gradient roles at priority 1), cfg3, against the production build.
set -o pipefail
TAG=${1:-r04r}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
for v in base A B base; do
  if [ $v = base ]; then L=$R/pymarl_amd/lib/libmq_learner.so; else L=$R/exp2/libmq_prio$v.so; fi
  MQ_LEARNER_LIB=$L timeout -k 10 300 python bench.py --config cfg3 --steps 20 --warmup 3 --phases --no-cpu-baseline > $O/bench_${TAG}_$v.json 2> $O/bench_${TAG}_$v.err || { tail -5 $O/bench_${TAG}_$v.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_${TAG}_$v.json'));print('$v', d['ms_per_step'])"
  tail -1 $O/bench_${TAG}_$v.err
done
