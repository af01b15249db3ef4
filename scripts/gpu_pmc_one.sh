#!/bin/bash
# One PMC pass of scripts/gpu_counters.sh (its groups: FETCH_SIZE | WRITE_SIZE | SQ), for workloads whose process
# crashes in exit-time teardown under rocprofv3 after the profiler has written its results (cfg5): each pass is then
# its own gpurun call. Usage: bash scripts/gpu_pmc_one.sh TAG CFG GROUP
set -o pipefail
TAG=$1; CFG=$2; GRP=$3
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
python -c "import sys; sys.path.insert(0, '$R'); import bench; print(bench.kernel_source_hash())" > $O/src_hash_${TAG}_${CFG}.txt || exit $?
cd /tmp && export TMPDIR=/tmp
BENCH="python $R/bench.py --config $CFG --steps 5 --warmup 2 --no-cpu-baseline"
case $GRP in
  FETCH_SIZE|WRITE_SIZE) CTR=$GRP ;;
  SQ) CTR="SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_COEXEC_CYCLES GRBM_GUI_ACTIVE" ;;
  *) echo "unknown group $GRP"; exit 2 ;;
esac
timeout -k 10 300 rocprofv3 --pmc $CTR --output-format csv -d $O/pmc_${TAG}_${CFG}_${GRP} -o run -- $BENCH > $O/pmc_${TAG}_${CFG}_${GRP}.log 2>&1
rc=$?
ls $O/pmc_${TAG}_${CFG}_${GRP}/ 2>/dev/null
exit $rc
