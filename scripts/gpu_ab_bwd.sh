#!/bin/bash
# A/B of the one-chain-wave BPTT (MQ_BWD_PAIR=1, gru_bwd_pair.hpp) against the fused BPTT at cfg2: its parity tests,
# then rocprof kernel averages and the bench line of each. Arg: tag.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; T=${1:-r05y}
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "bwd_pair" > $O/${T}_tests.log 2>&1; rc=$?; tail -3 $O/${T}_tests.log; [ $rc = 0 ] || { grep -E "Error|assert" $O/${T}_tests.log | head -20; exit 1; }
for v in new old; do
  case $v in new) E="MQ_BWD_PAIR=1" ;; old) E="MQ_BWD_PAIR=0" ;; esac
  (cd /tmp && export TMPDIR=/tmp && env $E timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_${T}_$v -o run -- python $R/bench.py --steps 30 --warmup 3 --no-cpu-baseline > $O/prof_${T}_$v.log 2>&1) || exit 1
  echo "== $v"; python -c "
import csv
for r in csv.DictReader(open('$O/prof_${T}_$v/run_kernel_stats.csv')):
    if int(r['Calls']) >= 30: print('  ', r['Name'][:48], r['Calls'], round(float(r['AverageNs'])/1000, 2))
" || exit 1
  env $E timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > $O/${T}_bench_$v.json 2> $O/${T}_bench_$v.err || exit 1
  python -c "import json;d=json.load(open('$O/${T}_bench_$v.json'));print('  bench', d['ms_per_step'])"
done
for v in new old; do
  case $v in new) E="MQ_BWD_PAIR=1" ;; old) E="MQ_BWD_PAIR=0" ;; esac
  env $E timeout -k 10 300 python bench.py --config cfg4 --steps 50 --warmup 5 --no-cpu-baseline --phases > $O/${T}_cfg4_$v.json 2> $O/${T}_cfg4_$v.err || exit 1
  python -c "import json;d=json.load(open('$O/${T}_cfg4_$v.json'));print('  cfg4 $v', d['ms_per_step'], d['roofline']['plan'].get('fused_bwd'))"
done
