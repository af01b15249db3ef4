#!/bin/bash
# Round 4t: s_setprio A/B on the fused BPTT (cfg2): A = chain waves at priority 2, B = producer waves at priority 1.
set -o pipefail
TAG=${1:-r04t}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
for v in base A B base A B; do
  if [ $v = base ]; then L=$R/pymarl_amd/lib/libmq_learner.so; else L=$R/exp2/libmq_bprio$v.so; fi
  MQ_LEARNER_LIB=$L timeout -k 10 300 python bench.py --config cfg2 --steps 100 --warmup 5 --phases --no-cpu-baseline > $O/bench_${TAG}_$v.json 2> $O/bench_${TAG}_$v.err || { tail -5 $O/bench_${TAG}_$v.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_${TAG}_$v.json'));print('$v', d['ms_per_step'], d['roofline']['launch_ms'])"
done
