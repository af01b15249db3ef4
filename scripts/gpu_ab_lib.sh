#!/bin/bash
# Same-box A/B of the current library against another build of it (pymarl_amd/lib/libmq_learner_base.so, e.g. the
# round's starting sources): rocprof kernel averages of each, then interleaved 100-step cfg2 bench lines.
# Usage: bash scripts/gpu_ab_lib.sh TAG [config]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; T=${1:-ab}; C=${2:-cfg2}
BASE=$R/pymarl_amd/lib/libmq_learner_base.so
for v in new base; do
  E=""; [ $v = base ] && E="MQ_LEARNER_LIB=$BASE"
  (cd /tmp && export TMPDIR=/tmp && env $E timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_${T}_$v -o run -- python $R/bench.py --config $C --steps 30 --warmup 3 --no-cpu-baseline > $O/prof_${T}_$v.log 2>&1) || exit 1
  echo "== $v"; python -c "
import csv
for r in csv.DictReader(open('$O/prof_${T}_$v/run_kernel_stats.csv')):
    if int(r['Calls']) >= 30: print('  ', r['Name'][:48], r['Calls'], round(float(r['AverageNs'])/1000, 2))
" || exit 1
done
for i in 1 2; do
  for v in new base; do
    E=""; [ $v = base ] && E="MQ_LEARNER_LIB=$BASE"
    env $E timeout -k 10 200 python bench.py --config $C --steps 100 --warmup 10 --no-cpu-baseline > $O/${T}_bench_${v}_$i.json 2> $O/${T}_bench_${v}_$i.err || exit 1
    python -c "import json;d=json.load(open('$O/${T}_bench_${v}_$i.json'));print('  bench $v $i', round(d['ms_per_step'],4))"
  done
done
