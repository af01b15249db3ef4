#!/bin/bash
# Round 4k: full GPU suite (LDS b128 alignment in every kernel, row-tile BPTT row order), cfg2 / cfg3 benches,
# cfg3 diag pass.
set -o pipefail
TAG=${1:-r04k}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
export MQ_PARITY_DIR=$O/parity_${TAG}
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/gpu_all_${TAG}.log 2>&1
rc=$?
tail -3 $O/gpu_all_${TAG}.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $O/gpu_all_${TAG}.log | head; exit $rc; }
for c in cfg2 cfg3; do
  timeout -k 10 300 python bench.py --config $c --steps 50 --warmup 5 --phases --no-cpu-baseline > $O/bench_${TAG}_$c.json 2> $O/bench_${TAG}_$c.err || { tail -5 $O/bench_${TAG}_$c.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_${TAG}_$c.json'));print('$c', d['ms_per_step'])"
  tail -1 $O/bench_${TAG}_$c.err
done
bash scripts/gpu_diag.sh $TAG cfg3 | grep gru_
