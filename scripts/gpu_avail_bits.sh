#!/bin/bash
# A/B of the mixer reading the replay buffer's avail bitmask (default) vs avail_actions (MQ_AVAIL_BITS=0): parity
# tests, then rocprof kernel averages and the bench line of configs[2] (cfg3) and cfg2 for each. Arg: tag.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; T=${1:-r05v}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "avail_bits or mix_stream or tiny_full or huber" > $O/${T}_tests.log 2>&1; rc=$?; tail -3 $O/${T}_tests.log; [ $rc = 0 ] || exit 1
for cfg in cfg3 cfg2; do
  for v in bits int; do
    case $v in bits) E="MQ_AVAIL_BITS=1" ;; int) E="MQ_AVAIL_BITS=0" ;; esac
    (cd /tmp && export TMPDIR=/tmp && env $E timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_${T}_${cfg}_$v -o run -- python $R/bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline > $O/prof_${T}_${cfg}_$v.log 2>&1) || exit 1
    echo "== $cfg $v"; python -c "
import csv
for r in csv.DictReader(open('$O/prof_${T}_${cfg}_$v/run_kernel_stats.csv')):
    if 'mix' in r['Name']: print('  ', r['Name'][:48], r['Calls'], round(float(r['AverageNs'])/1000, 2))
" || exit 1
    env $E timeout -k 10 300 python bench.py --config $cfg --steps 30 --warmup 3 --no-cpu-baseline > $O/${T}_bench_${cfg}_$v.json 2> $O/${T}_bench_${cfg}_$v.err || exit 1
    python -c "import json;d=json.load(open('$O/${T}_bench_${cfg}_$v.json'));print('  bench', d['ms_per_step'])"
  done
done
