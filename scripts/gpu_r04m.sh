#!/bin/bash
# Round 4m: mixer kernels with a wave-uniform row index: tail tests, cfg2 and cfg3 kernel times.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "hymix or cfg2 or cfg3 or tiny or teacher or mix or wide" > $O/t_mixu.log 2>&1 || { tail -20 $O/t_mixu.log; exit 1; }
tail -1 $O/t_mixu.log
cd /tmp && export TMPDIR=/tmp
for c in cfg2 cfg3; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_mixu_$c -o run -- python $R/bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline > $O/prof_mixu_$c.log 2>&1 || exit $?
python - <<PY
import csv
for r in list(csv.DictReader(open("$O/prof_mixu_$c/run_kernel_stats.csv")))[:7]:
    print("$c %-50s %8.1f" % (r["Name"][:50], float(r["AverageNs"]) / 1000))
PY
done
