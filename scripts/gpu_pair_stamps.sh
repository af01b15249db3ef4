#!/bin/bash
# Step stamps of the row-pair forward at cfg2 (split and shared roles).
set -o pipefail
O=gpurun_out; mkdir -p $O
for v in 1 0; do rm -f $O/stamps_$v.bin
  MQ_PAIR_SPLIT=$v MQ_PAIR_STAMP=$O/stamps_$v.bin timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2> $O/stamps_$v.err || exit 1
  echo "split=$v"; python scripts/pair_stamps.py $O/stamps_$v.bin 121 || exit 1
done
