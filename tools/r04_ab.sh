#!/bin/bash
# A/B of two library builds on one box: configs[4] benches alternating (BPGL_LIB), kernel averages
set -o pipefail
OUT=gpurun_out/${OUT_DIR:-r04_ab}
mkdir -p $OUT
for R in 1 2; do
  for V in a b; do
    L=convex_optimization_amd/_lib/libbpgl.so; [ $V = b ] && L=$LIB_B
    BPGL_LIB=$L timeout -k 10 240 python bench.py --config 4 $BENCH_ARGS > $OUT/bench_${V}_$R.json 2> $OUT/bench_${V}_$R.err || exit $?
  done
done
