#!/bin/bash
# Round-5 A/B of the cfg2 agent forward: the row-pair kernel with split SIMD roles (default), the row-pair kernel with
# shared SIMDs (MQ_PAIR_SPLIT=0) and the one-row-net kernel (MQ_FWD_PAIR=0), after the parity tests that cover them.
set -o pipefail
O=gpurun_out; mkdir -p $O; T=${1:-r05c}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "pair_switch or test_tiny_full or cfg2_trajectory" > $O/${T}_tests.log 2>&1; rc=$?; tail -3 $O/${T}_tests.log; [ $rc = 0 ] || exit 1
for rnd in 1 2; do for v in split shared old; do
  case $v in split) E="" ;; shared) E="MQ_PAIR_SPLIT=0" ;; old) E="MQ_FWD_PAIR=0" ;; esac
  env $E timeout -k 10 200 python bench.py --steps 100 --warmup 10 --phases --no-cpu-baseline > $O/${T}_bench_$v$rnd.json 2> $O/${T}_bench_$v$rnd.err || exit 1
  python -c "import json;d=json.load(open('$O/${T}_bench_$v$rnd.json'));print('$v', d['ms_per_step'])"; grep phase $O/${T}_bench_$v$rnd.err | tail -1 | cut -c1-120
done; done
