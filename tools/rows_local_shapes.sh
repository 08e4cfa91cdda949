#!/bin/bash
# Per-GPU shapes of the row-sharded multi-GPU bench, run on ONE GPU through the RCCL row
# path with a one-rank communicator (everything but the cross-GPU all-reduce itself):
#   weak (configs[2] family, m=8192 n=65536*N): N=2 4096x131072, N=4 2048x262144, N=8 1024x524288
#   strong (8192x65536 split N ways): 4096 / 2048 / 1024 rows x 65536
# and the column-sharded equivalent at N=1 for reference.  Usage: tools/rows_local_shapes.sh OUTDIR
set -e
OUT=${1:-gpurun_out/rows_local}
mkdir -p $OUT
for s in "8192 65536" "4096 131072" "2048 262144" "1024 524288" "4096 65536" "2048 65536" "1024 65536"; do
    set -- $s
    timeout -k 10 240 python -u bench.py --no-cpu --comm --shard rows --m $1 --n-per-gpu $2 \
        > $OUT/rows_m$1_n$2.json 2> $OUT/rows_m$1_n$2.err
done
timeout -k 10 240 python -u bench.py --no-cpu --comm --shard columns > $OUT/cols_m8192_n65536.json 2> $OUT/cols_m8192_n65536.err
