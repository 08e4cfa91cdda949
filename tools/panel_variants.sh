#!/bin/bash
# configs[4] panel: mainloop variants per pass (GPU box) -> gpurun_out/panel_variants/*.json
set -o pipefail
OUT=gpurun_out/panel_variants
mkdir -p $OUT
run() { local n=$1; shift; timeout -k 10 200 python3 bench.py --config 4 --steps 64 --warmup 100 --windows 3 "$@" > $OUT/$n.json 2> $OUT/$n.err || exit 1; }
run base
run i1_3 --interleave1 3
run i2_3 --interleave2 3
run i33 --interleave 3
run base_again
