#!/bin/bash
# configs[4] split-K chunks with pass 2's stage-major tiles.
set -o pipefail
OUT=${1:-gpurun_out/r05_kc}
mkdir -p $OUT
for r in 1 2; do
  for kc in 8 4 16; do
    timeout -k 10 200 python3 bench.py --config 4 --no-cpu --steps 256 --warmup 200 --kchunks $kc > $OUT/c4_kc${kc}_$r.json 2> $OUT/c4_kc${kc}_$r.err || exit $?
  done
done
