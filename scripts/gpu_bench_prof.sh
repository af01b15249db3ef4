#!/bin/bash
# Bench + rocprofv3 kernel-trace stats on the GPU box. Usage: bash scripts/gpu_bench_prof.sh TAG [config]
set -o pipefail
TAG=${1:-r01}; CFG=${2:-cfg2}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
timeout -k 10 400 python $R/bench.py --config $CFG --steps 50 --warmup 5 --phases > $R/gpurun_out/bench_${TAG}_${CFG}.json 2> $R/gpurun_out/bench_${TAG}_${CFG}.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_${TAG}_${CFG} -o run -- python $R/bench.py --config $CFG --steps 20 --warmup 3 --no-cpu-baseline > $R/gpurun_out/prof_${TAG}_${CFG}.log 2>&1 || exit $?
