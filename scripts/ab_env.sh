#!/bin/bash
# A/B one env switch on the cfg2 bench: bash scripts/ab_env.sh VAR=VALUE [config]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
KV=$1; CFG=${2:-cfg2}
mkdir -p $R/gpurun_out
for i in 1 2; do
  timeout -k 10 200 python $R/bench.py --config $CFG --steps 100 --warmup 5 --phases --no-cpu-baseline > $R/gpurun_out/abe_base_$i.json 2> $R/gpurun_out/abe_base_$i.err || exit $?
  env $KV timeout -k 10 200 python $R/bench.py --config $CFG --steps 100 --warmup 5 --phases --no-cpu-baseline > $R/gpurun_out/abe_var_$i.json 2> $R/gpurun_out/abe_var_$i.err || exit $?
done
for f in $R/gpurun_out/abe_*.json; do python -c "import json;d=json.load(open('$f'));print('$(basename $f)', round(d['ms_per_step'],4))"; done
for f in $R/gpurun_out/abe_*_1.err; do echo $(basename $f); grep phase $f; done
