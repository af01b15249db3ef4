#!/bin/bash
# mix_fast_kernel<16, 8> for n <= 8 (default) against <16, 16> (MQ_MIX_MN16=1): bitwise test, parity cases, then
# three interleaved cfg2 rounds.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "mix_mn8 or cfg2_trajectory or tiny_full or teacher" > $O/r03d_mixmn_parity.log 2>&1 || exit $?
echo "parity: $(tail -1 $O/r03d_mixmn_parity.log)"
for k in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --phases > $O/r03d_mixmn_8_$k.json 2> $O/r03d_mixmn_8_$k.err || exit $?
  MQ_MIX_MN16=1 timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --phases > $O/r03d_mixmn_16_$k.json 2> $O/r03d_mixmn_16_$k.err || exit $?
  echo "round $k done"
done
