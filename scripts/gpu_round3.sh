#!/bin/bash
# Round-3 evidence on one MI355X at the final sources. Usage: bash scripts/gpu_round3.sh TAG PART
#   PART a: GPU suite (parity records -> gpurun_out/parity_TAG), smoke, cfg2 bench + rocprof stats + PMC
#   PART b: cfg3 / cfg4 / cfg5 benches, cfg3 + cfg5 PMC and rocprof stats, gloo two-rank rehearsals
#   PART c: the cfg5 profile / PMC and the gloo rehearsals alone
set -o pipefail
TAG=${1:-r03}; PART=${2:-a}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
if [ "$PART" = a ]; then
  MQ_PARITY_DIR=$O/parity_$TAG timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu $R/tests > $O/gpu_all_$TAG.log 2>&1 || exit $?
  echo "suite: $(tail -1 $O/gpu_all_$TAG.log)"
  timeout -k 10 120 python -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke()" > $O/smoke_$TAG.log 2>&1 || exit $?
  echo "smoke ok"
  bash $R/scripts/gpu_bench_prof.sh $TAG cfg2 || exit $?
  echo "cfg2 bench + prof done"
  bash $R/scripts/gpu_counters.sh $TAG cfg2 || exit $?
  echo "cfg2 counters done"
  cd $R && timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_${TAG}_driver_cmd.json 2> $O/bench_${TAG}_driver_cmd.err || exit $?
  echo "driver cmd done"
elif [ "$PART" = c ]; then
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_${TAG}_cfg5 -o run -- python $R/bench.py --config cfg5 --steps 5 --warmup 2 --no-cpu-baseline > $O/prof_${TAG}_cfg5.log 2>&1) || exit $?
  bash $R/scripts/gpu_counters.sh $TAG cfg5 || exit $?
  echo "cfg5 prof + counters done"
  cd $R
  MQ_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 20 --warmup 3 > $O/bench_${TAG}_gloo2_cfg2.json 2> $O/bench_${TAG}_gloo2_cfg2.err || exit $?
  MQ_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29532 bench.py --config cfg5 --gpus 2 --steps 3 --warmup 1 > $O/bench_${TAG}_gloo2_cfg5.json 2> $O/bench_${TAG}_gloo2_cfg5.err || exit $?
  echo "gloo rehearsals done"
else
  for C in cfg3 cfg4; do
    timeout -k 10 300 python $R/bench.py --config $C --steps 20 --warmup 3 --no-cpu-baseline --phases > $O/bench_${TAG}_$C.json 2> $O/bench_${TAG}_$C.err || exit $?
    echo "$C bench done"
  done
  bash $R/scripts/gpu_counters.sh $TAG cfg3 || exit $?
  echo "cfg3 counters done"
  timeout -k 10 300 python $R/bench.py --config cfg5 --steps 20 --warmup 3 > $O/bench_${TAG}_cfg5.json 2> $O/bench_${TAG}_cfg5.err || exit $?
  echo "cfg5 bench done"
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_${TAG}_cfg5 -o run -- python $R/bench.py --config cfg5 --steps 5 --warmup 2 --no-cpu-baseline > $O/prof_${TAG}_cfg5.log 2>&1) || exit $?
  bash $R/scripts/gpu_counters.sh $TAG cfg5 || exit $?
  echo "cfg5 prof + counters done"
  cd $R
  MQ_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 20 --warmup 3 > $O/bench_${TAG}_gloo2_cfg2.json 2> $O/bench_${TAG}_gloo2_cfg2.err || exit $?
  MQ_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29532 bench.py --config cfg5 --gpus 2 --steps 3 --warmup 1 > $O/bench_${TAG}_gloo2_cfg5.json 2> $O/bench_${TAG}_gloo2_cfg5.err || exit $?
  echo "gloo rehearsals done"
fi
