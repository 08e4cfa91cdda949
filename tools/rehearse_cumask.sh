#!/bin/bash
# The driver's N > 1 bench command line rehearsed on ONE GPU with N ranks (2 or 4), every rank's
# solver stream on its own XCD-symmetric CU partition, so the default N > 1
# iteration -- one-pass row shards + RCCL -- runs as designed.  Every leg of the N > 1 line runs
# (strong, rows_exchange_fp32, columns, columns.strong, n1_same_run); rates are those of N ranks
# sharing one GPU's HBM with RCCL over loopback sockets, not of N GPUs.
# Usage (GPU box, repo root): tools/rehearse_cumask.sh N [bench args...]
set -o pipefail
N=${1:-2}; shift
OUT=gpurun_out/rehearse_cumask
mkdir -p $OUT
BPGL_BENCH_DEVICE=0 BPGL_BENCH_CU_PARTITION=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node $N --master-addr 127.0.0.1 --master-port $((29700 + N)) bench.py --gpus $N "$@" \
    > $OUT/n$N.json 2> $OUT/n$N.err
