#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "hymix or cfg2 or tiny or teacher or mix" > $O/t_mixu.log 2>&1 || { tail -20 $O/t_mixu.log; exit 1; }
tail -1 $O/t_mixu.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_mixu -o run -- python $R/bench.py --steps 30 --warmup 3 --no-cpu-baseline > $O/prof_mixu.log 2>&1 || exit $?
python - <<PY
import csv
for r in list(csv.DictReader(open("$O/prof_mixu/run_kernel_stats.csv")))[:7]:
    print("%-50s %8.1f" % (r["Name"][:50], float(r["AverageNs"]) / 1000))
PY
