#!/bin/bash
# Round 4c: the row-tile MFMA forward / BPTT (gru_tiles.hpp): parity tests, then the cfg3 bench with phases.
set -o pipefail
TAG=${1:-r04c}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
export MQ_PARITY_DIR=$O/parity_${TAG}
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "row_tiles or wide_batch or row_batched" > $O/tiles_${TAG}.log 2>&1
rc=$?
tail -25 $O/tiles_${TAG}.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config cfg3 --steps 10 --warmup 3 --phases --no-cpu-baseline > $O/bench_${TAG}_cfg3.json 2> $O/bench_${TAG}_cfg3.err || { tail -5 $O/bench_${TAG}_cfg3.err; exit 1; }
cat $O/bench_${TAG}_cfg3.json
tail -2 $O/bench_${TAG}_cfg3.err
