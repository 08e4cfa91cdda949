#!/bin/bash
# configs[4] panel pass 2 with loader and MFMA waves split (interleave2 4) against the default
# (interleave2 1) -> gpurun_out/panel_roles/
set -o pipefail
OUT=gpurun_out/panel_roles
mkdir -p $OUT
run() { local n=$1; shift; timeout -k 10 200 python3 bench.py --config 4 --steps 64 --warmup 100 --windows 3 "$@" > $OUT/$n.json 2> $OUT/$n.err || exit 1; }
run base
run i2_4 --interleave2 4
run base_again
run i2_4_again --interleave2 4
