#!/bin/bash
# rocprof kernel averages and 100-step cfg2 bench lines for each MQ_PLAN value given (round 6 sweeps).
# Usage: bash scripts/gpu_plan_sweep.sh TAG PLAN...   (PLAN "-" = the default plan)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; T=$1; shift
for p in "$@"; do
  v=$p; [ "$p" = "-" ] && p=""
  (cd /tmp && export TMPDIR=/tmp && MQ_PLAN=$p timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_${T}_$v -o run -- python $R/bench.py --steps 30 --warmup 3 --no-cpu-baseline > $O/prof_${T}_$v.log 2>&1) || exit 1
  echo "== $v"; python -c "
import csv
for r in csv.DictReader(open('$O/prof_${T}_$v/run_kernel_stats.csv')):
    if int(r['Calls']) >= 30: print('  ', r['Name'][:48], r['Calls'], round(float(r['AverageNs'])/1000, 2))
" || exit 1
  MQ_PLAN=$p timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > $O/${T}_bench_$v.json 2> $O/${T}_bench_$v.err || exit 1
  python -c "import json;d=json.load(open('$O/${T}_bench_$v.json'));print('  bench', round(d['ms_per_step'],4))"
done
