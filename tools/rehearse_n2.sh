#!/bin/bash
# Rehearsal of bench.py's N > 1 path on a one-GPU box: two ranks under torch.distributed.run,
# both on device 0 (BPGL_BENCH_DEVICE=0).  Throughput numbers are meaningless; the run checks
# that the multi-rank code path (gloo side channel, RCCL communicator, row shards, strong leg,
# JSON line) works end to end.  Default split: columns -- without CU partitions the row split's
# k_onepass cannot keep all of its blocks co-resident beside another rank's (it then falls back to
# the two-pass row iteration by design).  tools/rehearse_cumask.sh gives every rank its own CUs and
# runs the default row split as designed (round 3).
# Usage (GPU box): [NPROC=N] tools/rehearse_n2.sh [extra bench args]
set -o pipefail
mkdir -p gpurun_out/rehearse
BPGL_BENCH_DEVICE=0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node ${NPROC:-2} \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus ${NPROC:-2} --steps 16 --warmup 4 --no-cpu --shard columns "$@" \
    > gpurun_out/rehearse/bench_n${NPROC:-2}.json 2> gpurun_out/rehearse/bench_n${NPROC:-2}.err
