#!/bin/bash
# Round 4o: COMA chain phase spans (workgroup 0, MQ_COMA_CHAIN_TRACE=1) at the current sources.
set -o pipefail
TAG=${1:-r04o}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
MQ_COMA_CHAIN_TRACE=1 timeout -k 10 300 python bench.py --config cfg5 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_${TAG}_cfg5.json 2> $O/trace_${TAG}_cfg5.txt || { tail -5 $O/trace_${TAG}_cfg5.txt; exit 1; }
grep -v amdgpu.ids $O/trace_${TAG}_cfg5.txt | tail -6
