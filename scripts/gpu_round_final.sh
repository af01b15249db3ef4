#!/bin/bash
# Round-end evidence on one MI355X: GPU suite, smoke, cfg2 bench + rocprof stats + PMC traffic, cfg5 COMA bench,
# and the N>1 control flow of both benches rehearsed with gloo (2 ranks sharing the GPU). Usage: TAG
set -o pipefail
TAG=${1:-r01}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu $R/tests > $O/gpu_all_$TAG.log 2>&1 || exit $?
timeout -k 10 120 python -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke()" > $O/smoke_$TAG.log 2>&1 || exit $?
bash $R/scripts/gpu_bench_prof.sh $TAG cfg2 || exit $?
bash $R/scripts/gpu_pmc.sh $TAG cfg2 || exit $?
timeout -k 10 300 python $R/bench.py --config cfg5 --steps 20 --warmup 3 > $O/bench_${TAG}_cfg5.json 2> $O/bench_${TAG}_cfg5.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_${TAG}_cfg5 -o run -- python $R/bench.py --config cfg5 --steps 5 --warmup 2 --no-cpu-baseline > $O/prof_${TAG}_cfg5.log 2>&1 || exit $?
cd $R
MQ_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 20 --warmup 3 > $O/bench_${TAG}_gloo2_cfg2.json 2> $O/bench_${TAG}_gloo2_cfg2.err || exit $?
MQ_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29532 bench.py --config cfg5 --gpus 2 --steps 3 --warmup 1 > $O/bench_${TAG}_gloo2_cfg5.json 2> $O/bench_${TAG}_gloo2_cfg5.err || exit $?
