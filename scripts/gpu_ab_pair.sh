#!/bin/bash
# Round-5 A/B of the agent forward: the row-pair kernel (default where the rows fit the CUs) against the one-row-net
# kernel (MQ_FWD_PAIR=0) at cfg2, and forced (MQ_FWD_PAIR=1) at cfg4's two-wave shard, after the parity tests that
# cover both; then the pair kernel's stamps.
set -o pipefail
O=gpurun_out; mkdir -p $O; T=${1:-r05e}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "pair_switch or pair_hyper or test_tiny_full or cfg2_trajectory" > $O/${T}_tests.log 2>&1; rc=$?; tail -3 $O/${T}_tests.log; [ $rc = 0 ] || exit 1
for rnd in 1 2; do for v in pair old; do
  case $v in pair) E="" ;; old) E="MQ_FWD_PAIR=0" ;; esac
  env $E timeout -k 10 200 python bench.py --steps 100 --warmup 10 --phases --no-cpu-baseline > $O/${T}_bench_$v$rnd.json 2> $O/${T}_bench_$v$rnd.err || exit 1
  python -c "import json;d=json.load(open('$O/${T}_bench_$v$rnd.json'));print('$v', d['ms_per_step'])"; grep phase $O/${T}_bench_$v$rnd.err | tail -1 | cut -c1-120
done; done
rm -f $O/${T}_stamps.bin
MQ_PAIR_STAMP=$O/${T}_stamps.bin timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2> $O/${T}_stamps.err || exit 1
python scripts/pair_stamps.py $O/${T}_stamps.bin 121
for v in pair1 default; do
  case $v in pair1) E="MQ_FWD_PAIR=1" ;; default) E="" ;; esac
  env $E timeout -k 10 200 python bench.py --config cfg4 --steps 50 --warmup 5 --phases --no-cpu-baseline > $O/${T}_cfg4_$v.json 2> $O/${T}_cfg4_$v.err || exit 1
  python -c "import json;d=json.load(open('$O/${T}_cfg4_$v.json'));print('cfg4 $v', d['ms_per_step'])"; grep phase $O/${T}_cfg4_$v.err | tail -1 | cut -c1-160
done
