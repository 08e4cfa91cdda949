#!/bin/bash
# onepass_wide A/B (round 3): rows of 8 loads per lane against 4, per ring variant, on the per-GPU
# shapes of the row split (one-rank RCCL leg, as tools/split_model.sh) and on configs[1].
# Usage (GPU box, repo root): tools/wide_sweep.sh -> gpurun_out/wide_sweep/*.json
set -o pipefail
OUT=gpurun_out/wide_sweep
mkdir -p $OUT
run() {   # name, bench args...
    local name=$1; shift
    echo "$name" >&2
    timeout -k 10 240 python3 bench.py --no-cpu --steps 256 --warmup 100 --windows 3 "$@" > $OUT/$name.json 2> $OUT/$name.err || return 1
}
R8="--comm --shard rows --m 1024 --n-per-gpu 524288"
run m1024_n524288_w0 $R8 --onepass-wide 0 &&
run m1024_n524288_w1_v0 $R8 --onepass-wide 1 --onepass-variant 0 &&
run m1024_n524288_w1_v1 $R8 --onepass-wide 1 --onepass-variant 1 &&
run m1024_n524288_w1_v2 $R8 --onepass-wide 1 --onepass-variant 2 &&
run m1024_n524288_w1_v3 $R8 --onepass-wide 1 --onepass-variant 3 &&
run m2048_n262144_w0 --comm --shard rows --m 2048 --n-per-gpu 262144 --onepass-wide 0 &&
run m2048_n262144_w1 --comm --shard rows --m 2048 --n-per-gpu 262144 --onepass-wide 1 &&
run m1024_n65536_w0 --comm --shard rows --m 1024 --n-per-gpu 65536 --onepass-wide 0 &&
run m1024_n65536_w1 --comm --shard rows --m 1024 --n-per-gpu 65536 --onepass-wide 1 &&
run one_m8192_n65536_w0 --m 8192 --n-per-gpu 65536 --onepass-wide 0 &&
run one_m8192_n65536_w1 --m 8192 --n-per-gpu 65536 --onepass-wide 1 &&
run one_m8192_n65536_w1_v3 --m 8192 --n-per-gpu 65536 --onepass-wide 1 --onepass-variant 3 &&
run m1024_n524288_w0_again $R8 --onepass-wide 0 &&
run m1024_n524288_w1_again $R8 --onepass-wide 1
