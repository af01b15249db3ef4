#!/bin/bash
# HBM traffic counters for the bench workload (separate --pmc passes; no trace domains beside kernel-trace).
# Usage: bash scripts/gpu_pmc.sh TAG [config]
set -o pipefail
TAG=${1:-r01}; CFG=${2:-cfg2}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d $R/gpurun_out/pmc_${TAG}_${CFG}_$C -o run -- python $R/bench.py --config $CFG --steps 5 --warmup 2 --no-cpu-baseline > $R/gpurun_out/pmc_${TAG}_${CFG}_$C.log 2>&1 || exit $?
done
