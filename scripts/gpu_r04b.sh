#!/bin/bash
# Round 4b: full GPU suite at the pruned sources, smoke, cfg2 bench, and the cfg5 rocprof run that crashed at exit
# before the chain moved to a plain launch. Usage: bash scripts/gpu_r04b.sh TAG
set -o pipefail
TAG=${1:-r04b}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/gpu_all_${TAG}.log 2>&1
rc=$?
tail -5 $O/gpu_all_${TAG}.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $O/gpu_all_${TAG}.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_${TAG}.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --phases > $O/bench_${TAG}_cfg2.json 2> $O/bench_${TAG}_cfg2.err || exit $?
cat $O/bench_${TAG}_cfg2.json
bash scripts/gpu_r04_segv.sh $TAG
tail -3 $O/prof_${TAG}_cfg5.log
