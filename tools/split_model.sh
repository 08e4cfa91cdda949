#!/bin/bash
# Per-GPU iteration time of every shape the N = 2 / 4 / 8 runs give one GPU, for both splits,
# measured on one GPU (DESIGN.md section 6 cost model).  Row shards run through the one-rank
# RCCL leg (--comm: fold + graph-captured all-reduce of a one-rank communicator, i.e. everything
# but the cross-GPU transfer); column shards run the two-pass kernels on their (m, n/N) shard.
# Usage (GPU box, repo root): tools/split_model.sh  -> gpurun_out/split_model/*.json
set -o pipefail
OUT=gpurun_out/split_model
mkdir -p $OUT
run() {   # name, bench args...
    local name=$1; shift
    timeout -k 10 240 python3 bench.py --no-cpu --no-side-legs --steps 256 --warmup 100 --windows 3 "$@" > $OUT/$name.json 2> $OUT/$name.err || return 1
}
run rows_m8192_n65536   --comm --shard rows --m 8192 --n-per-gpu 65536 &&
run rows_m4096_n65536   --comm --shard rows --m 4096 --n-per-gpu 65536 &&
run rows_m2048_n65536   --comm --shard rows --m 2048 --n-per-gpu 65536 &&
run rows_m1024_n65536   --comm --shard rows --m 1024 --n-per-gpu 65536 &&
run rows_m4096_n131072  --comm --shard rows --m 4096 --n-per-gpu 131072 &&
run rows_m2048_n262144  --comm --shard rows --m 2048 --n-per-gpu 262144 &&
run rows_m1024_n524288  --comm --shard rows --m 1024 --n-per-gpu 524288 &&
run cols_m8192_n65536   --onepass 0 --m 8192 --n-per-gpu 65536 &&
run cols_m8192_n32768   --onepass 0 --m 8192 --n-per-gpu 32768 &&
run cols_m8192_n16384   --onepass 0 --m 8192 --n-per-gpu 16384 &&
run cols_m8192_n8192    --onepass 0 --m 8192 --n-per-gpu 8192 &&
run one_m8192_n65536    --m 8192 --n-per-gpu 65536
