#!/bin/bash
# One GPU-box evidence pass. Usage: bash scripts/gpu_round.sh TAG [steps...]
#   steps: suite smoke bench counters gloo2 cfg5 cfg3   (default: suite smoke bench)
set -o pipefail
TAG=${1:-r02}; shift
STEPS=${@:-suite smoke bench}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export MQ_PARITY_DIR=$O/parity_$TAG
for S in $STEPS; do
  echo "== $S $(date +%T)"
  case $S in
    suite) timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu $R/tests > $O/gpu_all_$TAG.log 2>&1 || exit $? ;;
    smoke) timeout -k 10 120 python -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke()" > $O/smoke_$TAG.log 2>&1 || exit $? ;;
    bench) bash $R/scripts/gpu_bench_prof.sh $TAG cfg2 || exit $? ;;
    counters) bash $R/scripts/gpu_counters.sh $TAG cfg2 || exit $? ;;
    gloo2) MQ_BENCH_BACKEND=gloo timeout -k 10 300 python $R/bench.py --gpus 2 --steps 20 --warmup 3 > $O/bench_${TAG}_gloo2_cfg2.json 2> $O/bench_${TAG}_gloo2_cfg2.err || exit $? ;;
    cfg5) timeout -k 10 300 python $R/bench.py --config cfg5 --steps 20 --warmup 3 > $O/bench_${TAG}_cfg5.json 2> $O/bench_${TAG}_cfg5.err || exit $? ;;
    cfg3) timeout -k 10 300 python $R/bench.py --config cfg3 --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_${TAG}_cfg3.json 2> $O/bench_${TAG}_cfg3.err || exit $? ;;
    *) echo "unknown step $S"; exit 1 ;;
  esac
done
echo "== done $(date +%T)"
