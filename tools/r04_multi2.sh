#!/bin/bash
# Round 4 closing: the N = 2 and N = 4 bench rehearsals (CU partitions on one GPU) with the final code
set -o pipefail
OUT=gpurun_out/r04_multi2
mkdir -p $OUT
for N in 2 4; do
  BPGL_BENCH_DEVICE=0 BPGL_BENCH_CU_PARTITION=1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node $N --master-addr 127.0.0.1 --master-port $((29700 + N)) bench.py --gpus $N \
    --steps 32 --warmup 16 --ramp 32 --windows 3 --cpu-seconds 3 > $OUT/n$N.json 2> $OUT/n$N.err || exit $?
done
