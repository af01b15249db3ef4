#!/bin/bash
# A/B two builds of libmq_learner.so on the cfg2 bench: bash scripts/ab_bench.sh libA.so libB.so [config]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
A=$1; B=$2; CFG=${3:-cfg2}
mkdir -p $R/gpurun_out
for i in 1 2; do
  for L in $A $B; do
    MQ_LEARNER_LIB=$R/pymarl_amd/lib/$L timeout -k 10 200 python $R/bench.py --config $CFG --steps 100 --warmup 5 --phases --no-cpu-baseline > $R/gpurun_out/ab_${L%.so}_$i.json 2> $R/gpurun_out/ab_${L%.so}_$i.err || exit $?
  done
done
for f in $R/gpurun_out/ab_*.json; do python -c "import json,sys;d=json.load(open('$f'));print('$(basename $f)', round(d['ms_per_step'],4), d['roofline']['kernel'], round(d['roofline']['launch_ms'],4))"; done
for f in $R/gpurun_out/ab_*_1.err; do echo $(basename $f); grep phase $f; done
