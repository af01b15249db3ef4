#!/bin/bash
# Round 4h: hymix + row-tile tests (both BPTT variants), cfg2 hymix A/B, cfg3 BPTT A/B.
set -o pipefail
TAG=${1:-r04h}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "hymix or row_tiles" > $O/t_${TAG}.log 2>&1
rc=$?
tail -2 $O/t_${TAG}.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $O/t_${TAG}.log | head; exit $rc; }
MQ_BWD_SPLIT=1 timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "row_tiles" > $O/t_${TAG}_split.log 2>&1
rc=$?
tail -2 $O/t_${TAG}_split.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $O/t_${TAG}_split.log | head; exit $rc; }
for hm in 1 0; do
  MQ_HYMIX=$hm timeout -k 10 300 python bench.py --config cfg2 --steps 50 --warmup 5 --phases --no-cpu-baseline > $O/bench_${TAG}_cfg2_hm$hm.json 2> $O/bench_${TAG}_cfg2_hm$hm.err || { tail -5 $O/bench_${TAG}_cfg2_hm$hm.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_${TAG}_cfg2_hm$hm.json'));print('cfg2 hymix=$hm', d['ms_per_step'])"
  tail -1 $O/bench_${TAG}_cfg2_hm$hm.err
done
for sp in 0 1; do
  MQ_BWD_SPLIT=$sp timeout -k 10 300 python bench.py --config cfg3 --steps 20 --warmup 3 --phases --no-cpu-baseline > $O/bench_${TAG}_cfg3_sp$sp.json 2> $O/bench_${TAG}_cfg3_sp$sp.err || { tail -5 $O/bench_${TAG}_cfg3_sp$sp.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_${TAG}_cfg3_sp$sp.json'));print('cfg3 split=$sp', d['ms_per_step'])"
  tail -1 $O/bench_${TAG}_cfg3_sp$sp.err
done
