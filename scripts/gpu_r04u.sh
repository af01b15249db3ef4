#!/bin/bash
# Round 4u: row-tile tests and cfg3 bench after removing the per-step 64-bit address VALU (buffer descriptors,
# readfirstlane'd loop counters) and the GI register copies across the forward's back edge.
set -o pipefail
TAG=${1:-r04u}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "row_tiles or wide_batch or cfg3_vdn_b128" > $O/t_${TAG}.log 2>&1
rc=$?
tail -2 $O/t_${TAG}.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $O/t_${TAG}.log | head; exit $rc; }
for k in 1 2; do
  timeout -k 10 300 python bench.py --config cfg3 --steps 20 --warmup 3 --phases --no-cpu-baseline > $O/bench_${TAG}_cfg3_$k.json 2> $O/bench_${TAG}_cfg3_$k.err || { tail -5 $O/bench_${TAG}_cfg3_$k.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_${TAG}_cfg3_$k.json'));print('cfg3', d['ms_per_step'])"
  tail -1 $O/bench_${TAG}_cfg3_$k.err
done
