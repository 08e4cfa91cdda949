#!/bin/bash
# Round 4: the N = 8 strong shard (1024 x 65536) under the one-pass variants, the fp32 exchange and
# the in-kernel fold, through the one-rank RCCL row-shard path
set -o pipefail
OUT=gpurun_out/r04_split2
mkdir -p $OUT
run() {
  timeout -k 10 240 python bench.py --m 1024 --n-per-gpu 65536 --comm --shard rows --no-cpu "$@" \
      > $OUT/m1024_$(echo "$@" | tr ' ' '_' | tr -d '-').json 2> $OUT/m1024.err || exit $?
}
run --onepass-variant 1
run --onepass-variant 2
run --onepass-variant 3
run --exchange-fp32 1
run --onepass-fold 1
run --tail-row-blocks 0
