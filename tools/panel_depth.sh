#!/bin/bash
# configs[4] panel: stream depths per pass -- interleave 4 / 5 / 6 (operand two stages ahead, A one)
# against the defaults (pass 1: 2, pass 2: 1) and their plain forms (1) -> gpurun_out/panel_depth/
set -o pipefail
OUT=gpurun_out/panel_depth
mkdir -p $OUT
run() { local n=$1; shift; timeout -k 10 200 python3 bench.py --config 4 --steps 64 --warmup 100 --windows 3 "$@" > $OUT/$n.json 2> $OUT/$n.err || exit 1; }
run base
run i1_1 --interleave1 1
run i1_5 --interleave1 5
run i1_4 --interleave1 4
run i2_5 --interleave2 5
run i2_4 --interleave2 4
run i55 --interleave 5
run i1_6 --interleave1 6
run i2_6 --interleave2 6
run i66 --interleave 6
run base_again
