#!/bin/bash
# configs[4] panel pass 2 on 512-row tiles (interleave2 4, kchunks 16 for 256 blocks) against the
# default 256-row form (interleave2 1, kchunks 8) -> gpurun_out/panel_wide2/
set -o pipefail
OUT=gpurun_out/panel_wide2
mkdir -p $OUT
run() { local n=$1; shift; timeout -k 10 200 python3 bench.py --config 4 --steps 64 --warmup 100 --windows 3 "$@" > $OUT/$n.json 2> $OUT/$n.err || exit 1; }
run base
run w16 --interleave2 4 --kchunks 16
run base_k16 --kchunks 16
run w8 --interleave2 4 --kchunks 8
run base_again
run w16_again --interleave2 4 --kchunks 16
