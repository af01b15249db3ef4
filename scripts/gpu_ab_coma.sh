#!/bin/bash
# Same-box A/B of the COMA critic chain at cfg5: the current library against pymarl_amd/lib/libmq_learner_base.so.
# The COMA GPU tests on the current library, then per library: the chain's phase spans (MQ_DIAG coma_trace), rocprof
# kernel averages, and two interleaved bench lines. Usage: bash scripts/gpu_ab_coma.sh TAG [skip-tests]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; T=${1:-abc}
cd $R
if [ "$2" != skip-tests ]; then
  timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_coma.py > $O/${T}_coma_tests.log 2>&1; rc=$?
  tail -3 $O/${T}_coma_tests.log; [ $rc = 0 ] || exit 1
fi
BASE=$R/pymarl_amd/lib/libmq_learner_base.so
BT=$R/pymarl_amd/lib/libmq_learner_btrace.so   # built with -DMQ_COMA_BTRACE (phase B split into its parts)
if [ -f $BT ]; then
  MQ_LEARNER_LIB=$BT MQ_DIAG=coma_trace timeout -k 10 200 python bench.py --config cfg5 --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2> $O/${T}_btrace.err || exit 1
  echo "== phase B split (labels: B = H1 fan-in, bar2 = H2, C = Q + TD, bar3 = dH2, D = dH1, next = rest of the step)"
  grep "coma_chain ns" $O/${T}_btrace.err | tail -2
fi
CT=$R/pymarl_amd/lib/libmq_learner_ctrace.so   # built with -DMQ_COMA_CTRACE (phase C split into its parts)
if [ -f $CT ]; then
  MQ_LEARNER_LIB=$CT MQ_DIAG=coma_trace timeout -k 10 200 python bench.py --config cfg5 --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2> $O/${T}_ctrace.err || exit 1
  echo "== phase C split (labels: B = B + B->C wait, bar2 = dH1 staged, C = dW1, bar3 = drain barrier, D = granule + X staging, next = D + rest)"
  grep "coma_chain ns" $O/${T}_ctrace.err | tail -2
fi
ALT=$R/pymarl_amd/lib/libmq_learner_alt.so   # optional third library (e.g. the previous step of a series)
VS="new base"; [ -f $ALT ] && VS="new alt base"
for v in $VS; do
  E=""; [ $v = base ] && E="MQ_LEARNER_LIB=$BASE"; [ $v = alt ] && E="MQ_LEARNER_LIB=$ALT"
  env $E MQ_DIAG=coma_trace timeout -k 10 200 python bench.py --config cfg5 --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2> $O/${T}_trace_$v.err || exit 1
  echo "== $v"; grep "coma_chain ns" $O/${T}_trace_$v.err | tail -2
  (cd /tmp && export TMPDIR=/tmp && env $E timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_${T}_$v -o run -- python $R/bench.py --config cfg5 --steps 10 --warmup 2 --no-cpu-baseline > $O/prof_${T}_$v.log 2>&1) || exit 1
  python -c "
import csv
for r in csv.DictReader(open('$O/prof_${T}_$v/run_kernel_stats.csv')):
    if 'chain_kernel' in r['Name']: print('  ', r['Name'][:48], r['Calls'], round(float(r['AverageNs'])/1000, 2))
" || exit 1
done
for i in 1 2; do
  for v in $VS; do
    E=""; [ $v = base ] && E="MQ_LEARNER_LIB=$BASE"; [ $v = alt ] && E="MQ_LEARNER_LIB=$ALT"
    env $E timeout -k 10 200 python bench.py --config cfg5 --steps 10 --warmup 2 --no-cpu-baseline > $O/${T}_bench_${v}_$i.json 2> $O/${T}_bench_${v}_$i.err || exit 1
    python -c "import json;d=json.load(open('$O/${T}_bench_${v}_$i.json'));print('  bench $v $i', round(d['ms_per_step'],4), d['roofline'].get('phases_ms'))"
  done
done
