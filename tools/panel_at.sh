#!/bin/bash
# configs[4] panel: pass 1 reading a transposed copy of A vs transposing LDS reads (GPU box)
set -o pipefail
OUT=gpurun_out/panel_at
mkdir -p $OUT
run() { local n=$1; shift; timeout -k 10 200 python3 bench.py --config 4 --steps 64 --warmup 100 --windows 3 "$@" > $OUT/$n.json 2> $OUT/$n.err || exit 1; }
run base
run at --transposed 1
run at_i1 --transposed 1 --interleave1 1
run at_i3 --transposed 1 --interleave1 3
run at_i0 --transposed 1 --interleave1 0
run base2
