#!/bin/bash
# One diagnostic rocprofv3 --pmc pass (stall / LDS / MFMA counters) over a short bench run. Usage:
# bash scripts/gpu_diag.sh TAG CONFIG
set -o pipefail
TAG=${1:-diag}; CFG=${2:-cfg3}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
BENCH="python $R/bench.py --config $CFG --steps 3 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --output-format csv -d $O/diag_${TAG}_${CFG} -o run -- $BENCH > $O/diag_${TAG}_${CFG}.log 2>&1 || exit $?
python $R/scripts/diag_summary.py $O/diag_${TAG}_${CFG} > $O/diag_${TAG}_${CFG}.txt
cat $O/diag_${TAG}_${CFG}.txt
