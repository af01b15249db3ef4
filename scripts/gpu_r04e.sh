#!/bin/bash
# Round 4e: hymix bitwise tests, then cfg2 with and without the fused hypernet+mixer kernel.
set -o pipefail
TAG=${1:-r04e}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "hymix" > $O/t_${TAG}.log 2>&1
rc=$?
tail -3 $O/t_${TAG}.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/t_${TAG}.log | head; exit $rc; }
for hm in 1 0; do
  MQ_HYMIX=$hm timeout -k 10 300 python bench.py --config cfg2 --steps 50 --warmup 5 --phases --no-cpu-baseline > $O/bench_${TAG}_hm$hm.json 2> $O/bench_${TAG}_hm$hm.err || { tail -5 $O/bench_${TAG}_hm$hm.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_${TAG}_hm$hm.json'));print('hymix=$hm', d['ms_per_step'])"
  tail -1 $O/bench_${TAG}_hm$hm.err
done
