#!/bin/bash
# configs[4] iteration rate against the iteration count: 64-iteration windows from a short and a long warmup.
set -o pipefail
OUT=${1:-gpurun_out/r05_c4trend}
mkdir -p $OUT
B="python3 bench.py --config 4 --no-cpu"
timeout -k 10 200 $B --steps 64 --warmup 5 --windows 12 > $OUT/w5.json 2> $OUT/w5.err || exit $?
timeout -k 10 200 $B --steps 64 --warmup 1500 --windows 6 > $OUT/w1500.json 2> $OUT/w1500.err || exit $?
timeout -k 10 200 $B --steps 64 --warmup 5 --windows 12 --defer-x 0 > $OUT/w5_nodefer.json 2> $OUT/w5_nodefer.err || exit $?
