#!/bin/bash
# Every single-GPU BASELINE config through bench.py (one JSON line each) into
# gpurun_out/bench_all/; run on the GPU box from the repo root.
set -e
OUT=gpurun_out/bench_all
mkdir -p $OUT
timeout -k 10 300 python bench.py --config 1 > $OUT/config1.json 2> $OUT/config1.err
timeout -k 10 300 python bench.py --config 3 --no-cpu > $OUT/config3.json 2> $OUT/config3.err
timeout -k 10 300 python bench.py --config 4 --no-cpu --steps 100 > $OUT/config4.json 2> $OUT/config4.err
timeout -k 10 300 python bench.py --config 1 --type double --no-cpu --steps 100 > $OUT/config1_f64.json 2> $OUT/config1_f64.err
timeout -k 10 300 python bench.py --config 1 --type bf16 --no-cpu > $OUT/config1_bf16.json 2> $OUT/config1_bf16.err
timeout -k 10 300 python bench.py --config 1 --block 4 --no-cpu > $OUT/config1_b4.json 2> $OUT/config1_b4.err
# BLOCK = 2: the reference's own benchmark setting (cpu_vs_gpu.py:101, b_exp = 1)
timeout -k 10 300 python bench.py --config 1 --block 2 --no-cpu > $OUT/config1_b2.json 2> $OUT/config1_b2.err
# one-rank RCCL row-shard path (the multi-GPU code path on one GPU)
timeout -k 10 300 python bench.py --config 1 --comm --shard rows --no-cpu > $OUT/config1_rows_comm.json 2> $OUT/config1_rows_comm.err
# the same single-block workloads on the two-pass iteration (one-pass off)
timeout -k 10 300 python bench.py --config 3 --no-cpu --onepass 0 > $OUT/config3_twopass.json 2> $OUT/config3_twopass.err
timeout -k 10 300 python bench.py --config 1 --type double --no-cpu --steps 100 --onepass 0 > $OUT/config1_f64_twopass.json 2> $OUT/config1_f64_twopass.err
timeout -k 10 300 python bench.py --config 1 --type bf16 --no-cpu --onepass 0 > $OUT/config1_bf16_twopass.json 2> $OUT/config1_bf16_twopass.err
