#!/bin/bash
# Round 5: the fused panel reduce + update -- its parity tests, then configs[4] with the knob on and
# off on the same box (alternating).  usage: tools/r05_panel_ab.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/r05_panel_ab}
mkdir -p $OUT
[ -n "$NOTEST" ] || timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_panel.py \
    -k "fused or interleave or carried" > $OUT/pytest_panel.txt 2>&1 || exit $?
B="python3 bench.py --no-cpu --no-side-legs --config 4 --steps 256 --warmup 200 --windows 5"
for r in 1 2; do
  # LIB@G: LIB = "tree" (the in-tree library) or a build_ab/LIB.so; G = 0: two kernels, else the fused
  # launch on a grid of G blocks
  for f in ${FORMS:-"tree@0 tree@256"}; do
    lib=${f%@*}; g=${f#*@}
    if [ "$g" = 0 ]; then a="--fuse-update 0"; else a="--fuse-update 1 --fuse-grid $g"; fi
    if [ "$lib" = tree ]; then env=""; else env="BPGL_LIB=build_ab/$lib.so"; fi
    env $env timeout -k 10 200 $B $a > $OUT/c4_${lib}_g${g}_$r.json 2> $OUT/c4_${lib}_g${g}_$r.err || exit $?
  done
done
