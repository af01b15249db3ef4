#!/bin/bash
# Bench lines at the r04x sources with the PMC summaries committed, so `roofline.traffic` is filled: the driver's
# default command line (cfg2) and one short run per other config.
set -o pipefail
TAG=${1:-r04x}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python bench.py > $O/bench_${TAG}_traffic_cfg2.json 2> $O/bench_${TAG}_traffic_cfg2.err || exit 1
for c in cfg3 cfg4 cfg5; do
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 3 > $O/bench_${TAG}_traffic_$c.json 2> $O/bench_${TAG}_traffic_$c.err || exit 1
done
for c in cfg2 cfg3 cfg4 cfg5; do
  python -c "import json;d=json.load(open('$O/bench_${TAG}_traffic_$c.json'));r=d['roofline'];print('$c', d['ms_per_step'], r['frac'], r['traffic'])"
done
