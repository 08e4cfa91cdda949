#!/bin/bash
# configs[1] with interleaved row groups: share of each group's rows read cache-allocating (permille).
set -o pipefail
OUT=${1:-gpurun_out/r05_cache}
mkdir -p $OUT
B="python3 bench.py --no-cpu --no-side-legs --steps 256 --warmup 100 --windows 5"
for r in 1 2; do
  for v in 0 50 100 150; do
    timeout -k 10 200 $B --onepass-cache $v > $OUT/c1_p${v}_$r.json 2> $OUT/c1_p${v}_$r.err || exit $?
  done
done
