#!/bin/bash
# Round-4 evidence for one config at the current sources: bench (with cpu_baseline and phases), the driver's own
# command line (cfg2), rocprofv3 kernel-trace stats of the same bench, and the three PMC passes (FETCH_SIZE,
# WRITE_SIZE, SQ) stamped with the kernel-source hash. Usage: TAG CONFIG [STEPS]
set -o pipefail
TAG=${1:-r04z}; CFG=${2:-cfg2}; STEPS=${3:-50}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 400 python bench.py --config $CFG --steps $STEPS --warmup 5 --phases > $O/bench_${TAG}_${CFG}.json 2> $O/bench_${TAG}_${CFG}.err || { tail -5 $O/bench_${TAG}_${CFG}.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_${TAG}_${CFG}.json'));print('$CFG', d['ms_per_step'], d['value'], d['roofline']['kernel'], d['roofline']['frac'], (d.get('cpu_baseline') or {}).get('value'))"
if [ "$CFG" = cfg2 ]; then
  timeout -k 10 300 python bench.py > $O/bench_${TAG}_driver_cmd.json 2> $O/bench_${TAG}_driver_cmd.err || exit 1
fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_${TAG}_${CFG} -o run -- python $R/bench.py --config $CFG --steps 20 --warmup 3 --no-cpu-baseline > $O/prof_${TAG}_${CFG}.log 2>&1 || exit $?
cd $R
bash scripts/gpu_counters.sh $TAG $CFG || exit $?
echo "evidence $CFG done"
