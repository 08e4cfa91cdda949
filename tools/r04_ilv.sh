#!/bin/bash
# Round 4: mainloop variants per pass at the final configs[4] defaults (interleave1 / interleave2 0-3)
set -o pipefail
OUT=gpurun_out/r04_ilv
mkdir -p $OUT
for V in "2 1" "0 1" "1 1" "3 1" "2 0" "2 2" "2 3" "2 1"; do
  set -- $V
  timeout -k 10 200 python bench.py --config 4 --interleave1 $1 --interleave2 $2 --windows 3 \
      > $OUT/bench_i$1_$2_$RANDOM.json 2> $OUT/bench_i$1_$2.err || exit $?
done
