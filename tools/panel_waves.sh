#!/bin/bash
# configs[4] panel: 8 vs 16 waves per block, each pass and each mainloop variant (GPU box).
set -o pipefail
OUT=gpurun_out/panel_waves
mkdir -p $OUT
for w1 in 0 4; do for w2 in 0 4; do
  timeout -k 10 200 python3 bench.py --config 4 --steps 64 --warmup 100 --windows 3 --waves1 $w1 --waves2 $w2 \
      > $OUT/w${w1}_${w2}.json 2> $OUT/w${w1}_${w2}.err || exit 1
done; done
for i in 0 1 2; do
  timeout -k 10 200 python3 bench.py --config 4 --steps 64 --warmup 100 --windows 3 --waves1 4 --waves2 4 --interleave $i \
      > $OUT/w4_4_ilv$i.json 2> $OUT/w4_4_ilv$i.err || exit 1
done
