#!/bin/bash
# SQ occupancy / stall counters per kernel for the bench workload (one --pmc pass, kernel-trace only).
# Usage: bash scripts/gpu_sq.sh TAG [config]
set -o pipefail
TAG=${1:-r01}; CFG=${2:-cfg2}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/sq_${TAG}_${CFG} -o run -- python $R/bench.py --config $CFG --steps 5 --warmup 2 --no-cpu-baseline > $R/gpurun_out/sq_${TAG}_${CFG}.log 2>&1
