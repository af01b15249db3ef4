#!/bin/bash
# Round-5 A/B of the agent forward at cfg2: parity tests of the pair kernel, its stamps (scripts/pair_stamps.py), then
# rocprof kernel durations of the row-pair kernel with the hypernet on waves 4 / 5 (default), as its epilogue and of the one-row-net kernel
# (MQ_PLAN=fwd_pair=0), and the bench line of each.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; T=${1:-r05k}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "pair_switch or pair_hyper or test_tiny_full or cfg2_trajectory" > $O/${T}_tests.log 2>&1; rc=$?; tail -3 $O/${T}_tests.log; [ $rc = 0 ] || exit 1
rm -f $O/${T}_stamps.bin
MQ_DIAG=pair_stamp=$O/${T}_stamps.bin timeout -k 10 200 python bench.py --steps 3 --warmup 2 --no-cpu-baseline > /dev/null 2> $O/${T}_stamps.err || exit 1
python scripts/pair_stamps.py $O/${T}_stamps.bin 121 || exit 1
for v in pair epi old; do
  case $v in pair) E="" ;; epi) E="MQ_PLAN=pair_hyp_epi" ;; old) E="MQ_PLAN=fwd_pair=0" ;; esac
  (cd /tmp && export TMPDIR=/tmp && env $E timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_${T}_$v -o run -- python $R/bench.py --steps 30 --warmup 3 --no-cpu-baseline > $O/prof_${T}_$v.log 2>&1) || exit 1
  echo "== $v"; python -c "
import csv
for r in csv.DictReader(open('$O/prof_${T}_$v/run_kernel_stats.csv')):
    if int(r['Calls']) >= 30: print('  ', r['Name'][:48], r['Calls'], round(float(r['AverageNs'])/1000, 2))
" || exit 1
  env $E timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > $O/${T}_bench_$v.json 2> $O/${T}_bench_$v.err || exit 1
  python -c "import json;d=json.load(open('$O/${T}_bench_$v.json'));print('  bench', d['ms_per_step'])"
done
