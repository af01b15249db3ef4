#!/bin/bash
# Round 4q: COMA chain with LDS-only barriers inside the workgroup: COMA tests, cfg5 bench, phase spans, phase-B split.
set -o pipefail
TAG=${1:-r04q}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_coma.py tests/test_gpu_dp.py > $O/t_${TAG}.log 2>&1
rc=$?
tail -2 $O/t_${TAG}.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $O/t_${TAG}.log | head; exit $rc; }
timeout -k 10 300 python bench.py --config cfg5 --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_${TAG}_cfg5.json 2> $O/bench_${TAG}_cfg5.err || { tail -5 $O/bench_${TAG}_cfg5.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_${TAG}_cfg5.json'));print('cfg5', d['ms_per_step'], d['roofline'].get('phases_ms'))"
MQ_COMA_CHAIN_TRACE=1 timeout -k 10 300 python bench.py --config cfg5 --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2> $O/trace_${TAG}_cfg5.txt || exit 1
grep coma_chain $O/trace_${TAG}_cfg5.txt | tail -2
MQ_LEARNER_LIB=$R/exp2/libmq_btrace.so MQ_COMA_CHAIN_TRACE=1 timeout -k 10 300 python bench.py --config cfg5 --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2> $O/btrace_${TAG}_cfg5.txt || exit 1
grep coma_chain $O/btrace_${TAG}_cfg5.txt | tail -2
