#!/bin/bash
# Round 4: the strong split's per-GPU shapes (8192 x 65536 by N = 1, 2, 4, 8 rows) through the one-rank
# RCCL row-shard path on one GPU -- the per-GPU part of the N > 1 value line
set -o pipefail
OUT=gpurun_out/r04_split
mkdir -p $OUT
for M in 8192 4096 2048 1024; do
  timeout -k 10 240 python bench.py --m $M --n-per-gpu 65536 --comm --shard rows --no-cpu \
      > $OUT/rows_m${M}_n65536.json 2> $OUT/rows_m${M}.err || exit $?
done
