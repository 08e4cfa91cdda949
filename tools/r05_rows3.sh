#!/bin/bash
# Interleaved (1) against consecutive (0) row groups with the final library (the consecutive form compiled
# without the runtime stride): configs[1], the N = 4 and N = 2 strong shards.
set -o pipefail
OUT=${1:-gpurun_out/r05_rows3}
mkdir -p $OUT
B="python3 bench.py --no-cpu --no-side-legs --steps 256 --warmup 100 --windows 5"
for r in 1 2; do
  for v in 0 1; do
    timeout -k 10 200 $B --onepass-rows $v > $OUT/c1_r${v}_$r.json 2> $OUT/c1_r${v}_$r.err || exit $?
    for m in 2048 4096; do
      timeout -k 10 200 $B --comm --shard rows --m $m --n-per-gpu 65536 --onepass-rows $v > $OUT/m${m}_r${v}_$r.json 2> $OUT/m${m}_r${v}_$r.err || exit $?
    done
  done
done
