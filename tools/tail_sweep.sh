#!/bin/bash
# Row-shard per-GPU shapes through the one-rank RCCL leg (the k_onepass_tail change of round 3:
# pipelined column tiles, up to 2048 blocks).  Usage (GPU box): tools/tail_sweep.sh
set -o pipefail
OUT=gpurun_out/tail_sweep
mkdir -p $OUT
run() {
    local name=$1; shift
    timeout -k 10 150 python3 bench.py --no-cpu --steps 256 --warmup 100 --windows 3 "$@" > $OUT/$name.json 2> $OUT/$name.err || exit 1
}
run rows_m1024_n524288 --comm --shard rows --m 1024 --n-per-gpu 524288
run rows_m2048_n262144 --comm --shard rows --m 2048 --n-per-gpu 262144
run rows_m1024_n65536 --comm --shard rows --m 1024 --n-per-gpu 65536
run rows_m8192_n65536 --comm --shard rows --m 8192 --n-per-gpu 65536
