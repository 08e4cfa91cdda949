#!/bin/bash
# Round 4: pass-2 mainloop default check (interleave2 1 vs 2) at k = 128 / 64 / 32, alternating
set -o pipefail
OUT=gpurun_out/r04_ilv2
mkdir -p $OUT
for K in 128 64 32; do
  for R in 1 2; do
    for I in 1 2; do
      timeout -k 10 200 python bench.py --rhs $K --interleave2 $I --windows 3 --no-cpu \
          > $OUT/bench_k${K}_i${I}_$R.json 2> $OUT/bench_k${K}_i${I}_$R.err || exit $?
    done
  done
done
