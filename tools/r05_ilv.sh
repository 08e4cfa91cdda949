#!/bin/bash
# configs[4] pass-2 / pass-1 mainloop variants (interleave 0-2) with pass 2's stage-major tiles.
set -o pipefail
OUT=${1:-gpurun_out/r05_ilv}
mkdir -p $OUT
B="python3 bench.py --config 4 --no-cpu --steps 256 --warmup 200"
for r in 1 2; do
  for v in 2 1 0; do
    timeout -k 10 200 $B --interleave2 $v > $OUT/c4_i2_${v}_$r.json 2> $OUT/c4_i2_${v}_$r.err || exit $?
  done
  for v in 1 0; do
    timeout -k 10 200 $B --interleave1 $v > $OUT/c4_i1_${v}_$r.json 2> $OUT/c4_i1_${v}_$r.err || exit $?
  done
done
