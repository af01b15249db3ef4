#!/bin/bash
# configs[3] shard (R = 320): hypernet beside the two-wave fused forward (default) against in order
# (MQ_HYP_OVERLAP=0): bitwise test and the cfg4 / cfg2 parity cases, then three interleaved cfg4 rounds and one
# cfg2 round (where the overlap does not apply: R = 256).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "hyper_beside or cfg4 or cfg2_qmix or tiny_qmix" > $O/r03d_hypov_parity.log 2>&1 || exit $?
echo "parity: $(tail -1 $O/r03d_hypov_parity.log)"
for k in 1 2 3; do
  timeout -k 10 200 python bench.py --config cfg4 --steps 100 --warmup 10 --no-cpu-baseline > $O/r03d_hypov_on_$k.json 2> $O/r03d_hypov_on_$k.err || exit $?
  MQ_HYP_OVERLAP=0 timeout -k 10 200 python bench.py --config cfg4 --steps 100 --warmup 10 --no-cpu-baseline > $O/r03d_hypov_off_$k.json 2> $O/r03d_hypov_off_$k.err || exit $?
  echo "round $k done"
done
timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > $O/r03d_hypov_cfg2.json 2> $O/r03d_hypov_cfg2.err || exit $?
echo "cfg2 done"
