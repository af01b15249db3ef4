#!/bin/bash
# Round-4 evidence, call C: cfg5 (COMA) and the gloo N = 2 rehearsals of both benches.
set -o pipefail
TAG=${1:-r04z}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
bash $R/scripts/gpu_r04_evidence.sh $TAG cfg5 20 || exit $?
cd $R
MQ_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 20 --warmup 3 > $O/bench_${TAG}_gloo2_cfg2.json 2> $O/bench_${TAG}_gloo2_cfg2.err || exit $?
MQ_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29532 bench.py --config cfg5 --gpus 2 --steps 3 --warmup 1 > $O/bench_${TAG}_gloo2_cfg5.json 2> $O/bench_${TAG}_gloo2_cfg5.err || exit $?
echo "gloo rehearsals done"
