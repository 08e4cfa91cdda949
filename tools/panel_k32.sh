#!/bin/bash
# configs[4] panel pass 1: 32-deep stages with a deeper A ring (interleave1 7: 6 A slots, 8: 7 A
# slots) against the default 64-deep pipelined form (interleave1 2) -> gpurun_out/panel_k32/
set -o pipefail
OUT=gpurun_out/panel_k32
mkdir -p $OUT
run() { local n=$1; shift; timeout -k 10 200 python3 bench.py --config 4 --steps 64 --warmup 100 --windows 3 "$@" > $OUT/$n.json 2> $OUT/$n.err || exit 1; }
run base
run i1_7 --interleave1 7
run i1_8 --interleave1 8
run base_again
run i1_7_again --interleave1 7
