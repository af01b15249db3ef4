#!/bin/bash
# Stamps of the row-pair forward at cfg2 (scripts/pair_stamps.py).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; T=${1:-r05q}
rm -f $O/${T}_stamps.bin
MQ_PAIR_STAMP=$O/${T}_stamps.bin timeout -k 10 200 python bench.py --steps 3 --warmup 2 --no-cpu-baseline > /dev/null 2> $O/${T}_stamps.err || exit 1
python scripts/pair_stamps.py $O/${T}_stamps.bin 121
