#!/bin/bash
# Two-granule (SB > 64) one-pass shapes: the N = 8 weak per-GPU row shard and configs[2] on one GPU.
set -o pipefail
OUT=gpurun_out/gpl2
mkdir -p $OUT
run() {
    local name=$1; shift
    timeout -k 10 150 python3 bench.py --no-cpu --steps 256 --warmup 100 --windows 3 "$@" > $OUT/$name.json 2> $OUT/$name.err || exit 1
}
run rows_m1024_n524288 --comm --shard rows --m 1024 --n-per-gpu 524288
run rows_m2048_n262144 --comm --shard rows --m 2048 --n-per-gpu 262144
run config2_n1 --config 2 --steps 64 --warmup 40
