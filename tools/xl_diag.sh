#!/bin/bash
# configs[1] (SB = 16, 16 row groups) with each row group's blocks on one XCD (default) or spread
# over all XCDs (BPGL_ONEPASS_XL=0, diagnostic), against the SB = 64 shape (4 groups, always spread).
set -o pipefail
OUT=gpurun_out/xl_diag
mkdir -p $OUT
run() {
    local name=$1; shift
    timeout -k 10 150 python3 bench.py --no-cpu --steps 256 --warmup 100 --windows 3 "$@" > $OUT/$name.json 2> $OUT/$name.err || exit 1
}
run sb16_xl1 --m 8192 --n-per-gpu 65536
BPGL_ONEPASS_XL=0 run sb16_xl0 --m 8192 --n-per-gpu 65536
run sb16_xl1_b --m 8192 --n-per-gpu 65536
BPGL_ONEPASS_XL=0 run sb16_xl0_b --m 8192 --n-per-gpu 65536
run sb128 --comm --shard rows --m 1024 --n-per-gpu 524288
