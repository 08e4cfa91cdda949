#!/bin/bash
# Round 4: the 8-rank paths on one GPU (CU partitions of 32 CUs, 4 per XCD) before the driver's
# 8-GPU run: the CU-mask probe for 8 partitions, the world = 8 RCCL tests, and the N = 8 and
# N = 2 bench rehearsals with the round-4 line (value = strong iters/s on 8192 x 65536).
set -o pipefail
OUT=gpurun_out/r04_multi
mkdir -p $OUT
# rehearsals: every leg of the N > 1 line on CU partitions (short windows: the code path and the
# JSON fields, not N-GPU rates -- the ranks share one GPU's HBM and RCCL runs over loopback sockets)
for N in 8 2; do
  BPGL_BENCH_DEVICE=0 BPGL_BENCH_CU_PARTITION=1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node $N --master-addr 127.0.0.1 --master-port $((29700 + N)) bench.py --gpus $N \
    --steps 32 --warmup 16 --ramp 32 --windows 3 --cpu-seconds 3 > $OUT/n$N.json 2> $OUT/n$N.err || exit $?
done
