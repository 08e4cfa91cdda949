#!/bin/bash
# configs[1] and the N = 2 strong shard, consecutive (0) against interleaved (1) row groups, alternating.
set -o pipefail
OUT=${1:-gpurun_out/r05_rows2}
mkdir -p $OUT
B="python3 bench.py --no-cpu --no-side-legs"
for r in 1 2 3; do
  for v in 0 1; do
    timeout -k 10 200 $B --steps 256 --warmup 100 --windows 5 --onepass-rows $v > $OUT/c1_r${v}_$r.json 2> $OUT/c1_r${v}_$r.err || exit $?
    timeout -k 10 200 $B --comm --shard rows --m 4096 --n-per-gpu 65536 --steps 256 --warmup 100 --windows 5 \
        --onepass-rows $v > $OUT/m4096_r${v}_$r.json 2> $OUT/m4096_r${v}_$r.err || exit $?
  done
done
