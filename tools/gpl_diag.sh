#!/bin/bash
# One-pass shapes by hand-off width: SB = 16 (configs[1]), SB = 64 (N = 4 weak shard), SB = 128 (N = 8
# weak shard, two granules per lane) and configs[2] on one GPU (SB = 128).  Usage (GPU box): tools/gpl_diag.sh
set -o pipefail
OUT=gpurun_out/gpl_diag
mkdir -p $OUT
run() {
    local name=$1; shift
    timeout -k 10 150 python3 bench.py --no-cpu --steps 256 --warmup 100 --windows 3 "$@" > $OUT/$name.json 2> $OUT/$name.err || exit 1
}
run sb16 --m 8192 --n-per-gpu 65536
run sb64 --comm --shard rows --m 2048 --n-per-gpu 262144
run sb128 --comm --shard rows --m 1024 --n-per-gpu 524288
run config2_n1 --config 2 --steps 64 --warmup 40
