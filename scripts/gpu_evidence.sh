#!/bin/bash
# Evidence on one MI355X at the current sources, one gpurun call. Usage: bash scripts/gpu_evidence.sh TAG PART...
#   suite    the GPU test suite (parity records -> gpurun_out/parity_TAG)
#   smoke    __graft_entry__.smoke()
#   cfgN     bench.py --config cfgN with cpu_baseline and phases, the driver's own command line (cfg2), rocprofv3
#            kernel-trace stats of the same bench, and the PMC passes stamped with the kernel-source hash
#            (scripts/gpu_counters.sh); cfgN:bench runs only the bench line, cfgN:prof bench + rocprof (no PMC)
#   gloo2    the N = 2 control flow of the cfg2 and cfg5 benches (gloo, two ranks sharing the GPU)
#   traffic  bench lines of every config after the PMC summaries are committed (roofline.traffic filled)
# Every step runs under its own time limit and the first failure ends the call.
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
summ() { python -c "import json;d=json.load(open('$1'));r=d['roofline'];print('$2', round(d['ms_per_step'],4), d['value'], r['kernel'], r['frac'], r.get('traffic'), (d.get('cpu_baseline') or {}).get('value'))"; }
for P in "$@"; do
  case $P in
    suite)
      MQ_PARITY_DIR=$O/parity_$TAG timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu $R/tests > $O/gpu_all_$TAG.log 2>&1 || { tail -30 $O/gpu_all_$TAG.log; exit 1; }
      tail -2 $O/gpu_all_$TAG.log ;;
    smoke)
      timeout -k 10 200 python -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke()" > $O/smoke_$TAG.log 2>&1 || { tail -5 $O/smoke_$TAG.log; exit 1; }
      tail -1 $O/smoke_$TAG.log ;;
    cfg*)
      CFG=${P%%:*}; MODE=${P#*:}; [ "$MODE" = "$P" ] && MODE=full
      case $CFG in cfg3|cfg5) STEPS=20 ;; *) STEPS=50 ;; esac
      timeout -k 10 400 python bench.py --config $CFG --steps $STEPS --warmup 5 --phases > $O/bench_${TAG}_${CFG}.json 2> $O/bench_${TAG}_${CFG}.err || { tail -5 $O/bench_${TAG}_${CFG}.err; exit 1; }
      summ $O/bench_${TAG}_${CFG}.json $CFG || exit 1
      grep phase $O/bench_${TAG}_${CFG}.err | tail -3
      [ "$MODE" = bench ] && continue
      if [ "$CFG" = cfg2 ]; then
        timeout -k 10 300 python bench.py > $O/bench_${TAG}_driver_cmd.json 2> $O/bench_${TAG}_driver_cmd.err || exit 1
        summ $O/bench_${TAG}_driver_cmd.json driver_cmd || exit 1
      fi
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_${TAG}_${CFG} -o run -- python $R/bench.py --config $CFG --steps 20 --warmup 3 --no-cpu-baseline > $O/prof_${TAG}_${CFG}.log 2>&1) || exit 1
      [ "$MODE" = prof ] && continue
      bash scripts/gpu_counters.sh $TAG $CFG || exit 1 ;;
    gloo2)
      MQ_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 20 --warmup 3 > $O/bench_${TAG}_gloo2_cfg2.json 2> $O/bench_${TAG}_gloo2_cfg2.err || exit 1
      MQ_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29532 bench.py --config cfg5 --gpus 2 --steps 3 --warmup 1 > $O/bench_${TAG}_gloo2_cfg5.json 2> $O/bench_${TAG}_gloo2_cfg5.err || exit 1
      echo "gloo rehearsals done" ;;
    traffic)
      timeout -k 10 300 python bench.py > $O/bench_${TAG}_traffic_cfg2.json 2> $O/bench_${TAG}_traffic_cfg2.err || exit 1
      for c in cfg3 cfg4 cfg5; do
        timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 3 > $O/bench_${TAG}_traffic_$c.json 2> $O/bench_${TAG}_traffic_$c.err || exit 1
      done
      for c in cfg2 cfg3 cfg4 cfg5; do summ $O/bench_${TAG}_traffic_$c.json $c; done ;;
    *) echo "unknown part $P"; exit 2 ;;
  esac
done
echo "evidence $TAG done"
