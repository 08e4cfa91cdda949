#!/bin/bash
# configs[4] panel: pass 2 on 512-row tiles (kchunks 16) vs 256-row tiles (GPU box)
set -o pipefail
OUT=gpurun_out/panel_rows2
mkdir -p $OUT
run() { local n=$1; shift; timeout -k 10 200 python3 bench.py --config 4 --steps 64 --warmup 100 --windows 3 "$@" > $OUT/$n.json 2> $OUT/$n.err || exit 1; }
run base
run r512_k16 --rows2 512 --kchunks 16
run r256_k16 --kchunks 16
run r512_k16_t --rows2 512 --kchunks 16 --transposed 1
run base2
