#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
for i in 1 2; do
  for v in 8 16 24; do
    MQ_DWH_SPLIT=$v timeout -k 10 200 python $R/bench.py --steps 100 --warmup 5 --phases --no-cpu-baseline > $R/gpurun_out/abs_${v}_$i.json 2> $R/gpurun_out/abs_${v}_$i.err || exit $?
  done
done
for f in $R/gpurun_out/abs_*.json; do python -c "import json;d=json.load(open('$f'));print('$(basename $f)', round(d['ms_per_step'],4))"; done
for f in $R/gpurun_out/abs_*_1.err; do echo $(basename $f) $(grep -o '"dwh": [0-9.]*, "reduce": [0-9.]*' $f); done
