#!/bin/bash
# Round 4j: row-tile tests, cfg3 bench with phases, diag PMC pass (LDS conflicts / stalls).
set -o pipefail
TAG=${1:-r04j}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "row_tiles or wide_batch" > $O/t_${TAG}.log 2>&1
rc=$?
tail -2 $O/t_${TAG}.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $O/t_${TAG}.log | head; exit $rc; }
timeout -k 10 300 python bench.py --config cfg3 --steps 20 --warmup 3 --phases --no-cpu-baseline > $O/bench_${TAG}_cfg3.json 2> $O/bench_${TAG}_cfg3.err || { tail -5 $O/bench_${TAG}_cfg3.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_${TAG}_cfg3.json'));print('cfg3', d['ms_per_step'])"
tail -1 $O/bench_${TAG}_cfg3.err
bash scripts/gpu_diag.sh $TAG cfg3 | grep gru_
