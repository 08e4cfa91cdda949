#!/bin/bash
# configs[4] panel: per-pass time against the number of right-hand sides k (operand bytes per block
# scale with k, A bytes per block do not) and the direction encoding -> gpurun_out/panel_ksweep/
set -o pipefail
OUT=gpurun_out/panel_ksweep
mkdir -p $OUT
run() { local n=$1; shift; timeout -k 10 200 python3 bench.py --steps 64 --warmup 100 --windows 3 --no-cpu "$@" > $OUT/$n.json 2> $OUT/$n.err || exit 1; }
run k128 --rhs 128
run k64 --rhs 64
run k32 --rhs 32
run k16 --rhs 16
run k128_ds1 --rhs 128 --d-split 1
run k64_ds1 --rhs 64 --d-split 1
python3 tools/summarize_bench.py $OUT/*.json
