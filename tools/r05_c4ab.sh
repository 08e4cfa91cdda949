#!/bin/bash
# configs[4] early / late in the solve for libbpgl variants (build_ab/NAME.so): 12 windows of 64 iterations
# from iteration 517 and 6 from iteration 2012.  usage: VARIANTS="base xnt" tools/r05_c4ab.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/r05_c4ab}
mkdir -p $OUT
B="python3 bench.py --config 4 --no-cpu --steps 64"
for r in $(seq 1 ${ROUNDS:-1}); do
  for v in $VARIANTS; do
    BPGL_LIB=build_ab/$v.so timeout -k 10 200 $B --warmup 5 --windows 12 > $OUT/early_${v}_$r.json 2> $OUT/early_${v}_$r.err || exit $?
    BPGL_LIB=build_ab/$v.so timeout -k 10 200 $B --warmup 1500 --windows 6 > $OUT/late_${v}_$r.json 2> $OUT/late_${v}_$r.err || exit $?
  done
done
