#!/bin/bash
# Sweep of the in-forward hypernet's tile schedule (MQ_DIAG hyp_sched=<hex>, gru_fwd_pair.hpp hyp_tiles_by) at cfg2: the pair
# kernel's rocprof average per schedule, then stamps and the bench line of the first. Args: tag sched...
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; T=$1; shift
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "pair_hyper" > $O/${T}_tests.log 2>&1; rc=$?; tail -2 $O/${T}_tests.log; [ $rc = 0 ] || exit 1
for h in "$@"; do
  (cd /tmp && export TMPDIR=/tmp && MQ_DIAG=hyp_sched=$h timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_${T}_$h -o run -- python $R/bench.py --steps 30 --warmup 3 --no-cpu-baseline > $O/prof_${T}_$h.log 2>&1) || exit 1
  python -c "
import csv
for r in csv.DictReader(open('$O/prof_${T}_$h/run_kernel_stats.csv')):
    if 'pair' in r['Name']: print('$h', r['Name'][:40], r['Calls'], round(float(r['AverageNs'])/1000, 2))
" || exit 1
done
rm -f $O/${T}_stamps.bin
MQ_DIAG=hyp_sched=$1,pair_stamp=$O/${T}_stamps.bin timeout -k 10 200 python bench.py --steps 3 --warmup 2 --no-cpu-baseline > /dev/null 2> $O/${T}_stamps.err || exit 1
python scripts/pair_stamps.py $O/${T}_stamps.bin 121 || exit 1
MQ_DIAG=hyp_sched=$1 timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > $O/${T}_bench.json 2> $O/${T}_bench.err || exit 1
python -c "import json;d=json.load(open('$O/${T}_bench.json'));print('bench', '$1', d['ms_per_step'])"
