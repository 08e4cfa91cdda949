#!/bin/bash
# Same-box A/B of two stream-layout variants against the working tree's default (build_ab/base.so):
# cm (pass-2 tiles stage-major) on configs[4]; rilv (k_onepass row groups interleaved) on the one-pass
# configs and row shards.  Each variant's own GPU tests run first.
set -o pipefail
OUT=${1:-gpurun_out/r05_layout}
mkdir -p $OUT
T="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu"
BPGL_LIB=build_ab/cm.so timeout -k 10 400 $T tests/test_panel.py > $OUT/pytest_cm.txt 2>&1 || exit $?
BPGL_LIB=build_ab/rilv.so timeout -k 10 400 $T tests/test_onepass.py tests/test_rowshard.py > $OUT/pytest_rilv.txt 2>&1 || exit $?
VARIANTS="base cm" ROUNDS=2 tools/r05_c4ab.sh $OUT/c4 || exit $?
VARIANTS="base rilv" ROUNDS=2 C3=1 WEAK=1 tools/r05_abrun.sh $OUT/op
