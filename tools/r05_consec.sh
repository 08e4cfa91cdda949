#!/bin/bash
# The runtime row-stride arithmetic of interleaved row groups against a build with consecutive rows only
# (compile-time), on the consecutive shapes (configs[3], the N = 8 strong and the weak row shards) and on
# configs[1] with rows forced consecutive.
set -o pipefail
OUT=${1:-gpurun_out/r05_consec}
mkdir -p $OUT
B="python3 bench.py --no-cpu --no-side-legs"
for r in 1 2; do
  for v in base consec; do
    BPGL_LIB=build_ab/$v.so timeout -k 10 200 $B --steps 256 --warmup 100 --windows 5 --onepass-rows 0 > $OUT/c1r0_${v}_$r.json 2> $OUT/c1r0_${v}_$r.err || exit $?
    BPGL_LIB=build_ab/$v.so timeout -k 10 200 $B --config 3 --steps 64 --warmup 20 --windows 3 > $OUT/c3_${v}_$r.json 2> $OUT/c3_${v}_$r.err || exit $?
    BPGL_LIB=build_ab/$v.so timeout -k 10 200 $B --comm --shard rows --m 1024 --n-per-gpu 65536 --steps 256 --warmup 100 --windows 5 > $OUT/m1024_${v}_$r.json 2> $OUT/m1024_${v}_$r.err || exit $?
    BPGL_LIB=build_ab/$v.so timeout -k 10 200 $B --comm --shard rows --m 1024 --n-per-gpu 524288 --steps 256 --warmup 50 --windows 3 > $OUT/m1024w_${v}_$r.json 2> $OUT/m1024w_${v}_$r.err || exit $?
  done
done
