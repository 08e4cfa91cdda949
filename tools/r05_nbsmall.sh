#!/bin/bash
# A 12-row ring (LAG 8) against 16 on the small strong row shards (N = 8 / 4 / 2: 1024 / 2048 / 4096 rows).
set -o pipefail
OUT=${1:-gpurun_out/r05_nbsmall}
mkdir -p $OUT
B="python3 bench.py --no-cpu --no-side-legs --comm --shard rows --n-per-gpu 65536 --steps 256 --warmup 100 --windows 5"
for r in 1 2; do
  for v in base nb12; do
    for m in 1024 2048 4096; do
      BPGL_LIB=build_ab/$v.so timeout -k 10 200 $B --m $m > $OUT/m${m}_${v}_$r.json 2> $OUT/m${m}_${v}_$r.err || exit $?
    done
  done
done
