#!/bin/bash
# Round 4s: fc2 on the recurrence waves (tree build) against fc2 on the projection waves (exp2/libmq_noC.so), cfg3;
# row-tile tests on the tree build.
set -o pipefail
TAG=${1:-r04s}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "row_tiles or wide_batch" > $O/t_${TAG}.log 2>&1
rc=$?
tail -2 $O/t_${TAG}.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $O/t_${TAG}.log | head; exit $rc; }
for v in C noC C noC; do
  if [ $v = C ]; then L=$R/pymarl_amd/lib/libmq_learner.so; else L=$R/exp2/libmq_$v.so; fi
  MQ_LEARNER_LIB=$L timeout -k 10 300 python bench.py --config cfg3 --steps 20 --warmup 3 --phases --no-cpu-baseline > $O/bench_${TAG}_$v.json 2> $O/bench_${TAG}_$v.err || { tail -5 $O/bench_${TAG}_$v.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_${TAG}_$v.json'));print('$v', d['ms_per_step'])"
  tail -1 $O/bench_${TAG}_$v.err
done
