#!/bin/bash
# Round 5, first GPU call: the driver's N = 1 command with the new side legs (config3 / config4 /
# config2_one_gpu), then the N = 2 line launched by bench.py itself (no torchrun wrapper) on one
# GPU's two CU partitions (VERDICT r04 "Next round" 1 and 2).
set -o pipefail
OUT=gpurun_out/r05_bench
mkdir -p $OUT
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/n1.json 2> $OUT/n1.err || exit $?
BPGL_BENCH_DEVICE=0 BPGL_BENCH_CU_PARTITION=1 timeout -k 10 400 python3 bench.py --gpus 2 --steps 20 --warmup 5 \
  > $OUT/n2.json 2> $OUT/n2.err || exit $?
