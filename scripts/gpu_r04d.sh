#!/bin/bash
# Round 4d: row-tile and hymix parity tests, then cfg3 and cfg2 benches with phases.
set -o pipefail
TAG=${1:-r04d}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
export MQ_PARITY_DIR=$O/parity_${TAG}
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "row_tiles or wide_batch or row_batched or hymix or hyper_in_forward or dwh_in_bptt" > $O/t_${TAG}.log 2>&1
rc=$?
tail -4 $O/t_${TAG}.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/t_${TAG}.log | head; exit $rc; }
for c in cfg3 cfg2; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 3 --phases --no-cpu-baseline > $O/bench_${TAG}_$c.json 2> $O/bench_${TAG}_$c.err || { tail -5 $O/bench_${TAG}_$c.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_${TAG}_$c.json'));print('$c', d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'])"
  tail -1 $O/bench_${TAG}_$c.err
done
