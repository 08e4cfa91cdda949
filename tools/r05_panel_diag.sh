#!/bin/bash
# Round 5: configs[4] pass times with one LDS-DMA stream dropped (timing-only builds, results wrong:
# build_ab/diag1 = no A pieces after stage 0, diag2 = no k-wide operand pieces, diag3 = neither)
# beside the real library, then the panel tests on the in-tree library.  usage: tools/r05_panel_diag.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/r05_panel_diag}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_panel.py \
    > $OUT/pytest_panel.txt 2>&1 || exit $?
B="python3 bench.py --no-cpu --no-side-legs --config 4 --steps 256 --warmup 100 --windows 3"
for v in head diag1 diag2 diag3; do
  BPGL_LIB=build_ab/$v.so timeout -k 10 200 $B > $OUT/c4_$v.json 2> $OUT/c4_$v.err || exit $?
done
timeout -k 10 200 $B > $OUT/c4_tree.json 2> $OUT/c4_tree.err || exit $?
