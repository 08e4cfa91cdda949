#!/bin/bash
# Infinity-Cache reuse at the strong-scaling per-GPU shapes (VERDICT r02 "next" 3): the one-pass
# row iteration through the one-rank RCCL leg (fold + graph-captured all-reduce included) at
# m = 1024 / 2048 rows x 65536 columns (the N = 8 / 4 shards of the 8192 x 65536 matrix: 256 /
# 512 MiB of A, against the 256 MiB Infinity Cache), sweeping "onepass_cache_permille" -- the
# share of each row group read with cache-allocating loads; launches alternate the row direction,
# so the next launch starts on those rows.  Usage (GPU box): tools/strong_cache_sweep.sh
set -o pipefail
OUT=gpurun_out/strong_cache
mkdir -p $OUT
for m in 1024 2048; do
  for c in 0 250 500 750 900 1000; do
    timeout -k 10 120 python3 bench.py --no-cpu --steps 256 --warmup 100 --windows 3 --comm --shard rows \
      --m $m --n-per-gpu 65536 --onepass-cache $c > $OUT/m${m}_c${c}.json 2> $OUT/m${m}_c${c}.err || exit 1
  done
done
