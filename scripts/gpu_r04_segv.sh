#!/bin/bash
# Round 4: reproduce the cfg5 exit-time crash under rocprofv3 once, with the process's mappings dumped as Python
# exits (bench.py MQ_DUMP_MAPS), so the crash frames resolve to library + offset. Usage: bash scripts/gpu_r04_segv.sh TAG
set -o pipefail
TAG=${1:-r04a}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
MQ_DUMP_MAPS=$O/maps_${TAG}_cfg5.txt timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv \
  -d $O/prof_${TAG}_cfg5 -o run -- python $R/bench.py --config cfg5 --steps 5 --warmup 2 --no-cpu-baseline \
  > $O/prof_${TAG}_cfg5.log 2>&1
rc=$?
echo "rocprofv3 exit $rc" >> $O/prof_${TAG}_cfg5.log
exit 0
