#!/bin/bash
# Quick check of the row-pair forward at cfg2 (round 6): its parity tests, stamps (scripts/pair_stamps.py), rocprof
# kernel averages and a 100-step bench line. Usage: bash scripts/gpu_pair_quick.sh TAG [MQ_DIAG items, e.g. hyp_sched=10642]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; T=${1:-pq}; X=${2:-}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "pair_switch or pair_hyper or test_tiny_full or cfg2_trajectory or teacher_forced_steps" > $O/${T}_tests.log 2>&1; rc=$?; tail -2 $O/${T}_tests.log; [ $rc = 0 ] || { tail -40 $O/${T}_tests.log; exit 1; }
rm -f $O/${T}_stamps.bin
MQ_DIAG=pair_stamp=$O/${T}_stamps.bin${X:+,$X} timeout -k 10 200 python bench.py --steps 3 --warmup 2 --no-cpu-baseline > /dev/null 2> $O/${T}_stamps.err || exit 1
python scripts/pair_stamps.py $O/${T}_stamps.bin 121 || exit 1
(cd /tmp && export TMPDIR=/tmp && MQ_DIAG=$X timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_${T} -o run -- python $R/bench.py --steps 30 --warmup 3 --no-cpu-baseline > $O/prof_${T}.log 2>&1) || exit 1
python -c "
import csv
for r in csv.DictReader(open('$O/prof_${T}/run_kernel_stats.csv')):
    if int(r['Calls']) >= 30: print('  ', r['Name'][:48], r['Calls'], round(float(r['AverageNs'])/1000, 2))
" || exit 1
MQ_DIAG=$X timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > $O/${T}_bench.json 2> $O/${T}_bench.err || exit 1
python -c "import json;d=json.load(open('$O/${T}_bench.json'));print('  bench', d['ms_per_step'])"
