#!/bin/bash
# Round 4g: hymix bitwise tests, cfg2 hymix A/B.
set -o pipefail
TAG=${1:-r04g}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "hymix" > $O/t_${TAG}.log 2>&1
rc=$?
tail -2 $O/t_${TAG}.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $O/t_${TAG}.log | head; exit $rc; }
for hm in 1 0; do
  MQ_HYMIX=$hm timeout -k 10 300 python bench.py --config cfg2 --steps 50 --warmup 5 --phases --no-cpu-baseline > $O/bench_${TAG}_cfg2_hm$hm.json 2> $O/bench_${TAG}_cfg2_hm$hm.err || { tail -5 $O/bench_${TAG}_cfg2_hm$hm.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_${TAG}_cfg2_hm$hm.json'));print('cfg2 hymix=$hm', d['ms_per_step'])"
  tail -1 $O/bench_${TAG}_cfg2_hm$hm.err
done
