#!/bin/bash
# Round 4l: cfg4 / cfg5 benches at the aligned-LDS sources, cfg2 hymix A/B again.
set -o pipefail
TAG=${1:-r04l}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
for c in cfg4 cfg5; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 3 --phases --no-cpu-baseline > $O/bench_${TAG}_$c.json 2> $O/bench_${TAG}_$c.err || { tail -5 $O/bench_${TAG}_$c.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_${TAG}_$c.json'));print('$c', d['ms_per_step'])"
  tail -1 $O/bench_${TAG}_$c.err
done
for hm in 1 0; do
  MQ_HYMIX=$hm timeout -k 10 300 python bench.py --config cfg2 --steps 50 --warmup 5 --phases --no-cpu-baseline > $O/bench_${TAG}_cfg2_hm$hm.json 2> $O/bench_${TAG}_cfg2_hm$hm.err || { tail -5 $O/bench_${TAG}_cfg2_hm$hm.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_${TAG}_cfg2_hm$hm.json'));print('cfg2 hymix=$hm', d['ms_per_step'])"
  tail -1 $O/bench_${TAG}_cfg2_hm$hm.err
done
