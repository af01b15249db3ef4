#!/bin/bash
# PMC evidence for the bench workload, one rocprofv3 --pmc pass per counter group (no trace domains beside the
# kernel dispatch records): HBM bytes (FETCH_SIZE, WRITE_SIZE) and SQ utilisation (MFMA busy, VALU busy, ...).
# Records the kernel-source hash of the tree it measured. Usage: bash scripts/gpu_counters.sh TAG [config]
set -o pipefail
TAG=${1:-r02}; CFG=${2:-cfg2}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
python -c "import sys; sys.path.insert(0, '$R'); import bench; print(bench.kernel_source_hash())" > $O/src_hash_${TAG}_${CFG}.txt || exit $?
cd /tmp && export TMPDIR=/tmp
BENCH="python $R/bench.py --config $CFG --steps 5 --warmup 2 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_${TAG}_${CFG}_FETCH_SIZE -o run -- $BENCH > $O/pmc_${TAG}_${CFG}_FETCH_SIZE.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_${TAG}_${CFG}_WRITE_SIZE -o run -- $BENCH > $O/pmc_${TAG}_${CFG}_WRITE_SIZE.log 2>&1 || exit $?
# 8 SQ counters + 1 GRBM (gfx950 per-pass limits: 8 SQ, 2 GRBM)
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_COEXEC_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_${TAG}_${CFG}_SQ -o run -- $BENCH > $O/pmc_${TAG}_${CFG}_SQ.log 2>&1 || exit $?
