#!/bin/bash
# Row-pair forward at cfg2 (round 6): stamps of the default schedule, then the kernel's rocprof average for each
# in-loop hypernet schedule given (MQ_DIAG hyp_sched=<hex>). Usage: bash scripts/gpu_hyp_sweep.sh TAG SCHED...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; T=$1; shift
rm -f $O/${T}_stamps.bin
MQ_DIAG=pair_stamp=$O/${T}_stamps.bin timeout -k 10 200 python bench.py --steps 3 --warmup 2 --no-cpu-baseline > /dev/null 2> $O/${T}_stamps.err || exit 1
python scripts/pair_stamps.py $O/${T}_stamps.bin 121 || exit 1
for h in "$@"; do
  (cd /tmp && export TMPDIR=/tmp && MQ_DIAG=hyp_sched=$h timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_${T}_$h -o run -- python $R/bench.py --steps 30 --warmup 3 --no-cpu-baseline > $O/prof_${T}_$h.log 2>&1) || exit 1
  python -c "
import csv
for r in csv.DictReader(open('$O/prof_${T}_$h/run_kernel_stats.csv')):
    if 'pair' in r['Name']: print('$h', r['Name'][:40], r['Calls'], round(float(r['AverageNs'])/1000, 2))
" || exit 1
done
