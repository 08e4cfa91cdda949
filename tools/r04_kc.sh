#!/bin/bash
# Round 4: configs[4] split-K chunks and the pass-1 mainloop at the final defaults
set -o pipefail
OUT=gpurun_out/r04_kc
mkdir -p $OUT
for V in "--kchunks 8" "--kchunks 4" "--kchunks 16" "--interleave1 3" "--kchunks 8"; do
  timeout -k 10 200 python bench.py --config 4 --windows 3 --no-cpu $V \
      > $OUT/bench_$(echo $V | tr ' ' '_' | tr -d '-')_$RANDOM.json 2> $OUT/bench.err || exit $?
done
