#!/bin/bash
# the long full-size GPU tests (1000-iteration horizons, 2^32-element instances)
set -o pipefail
OUT=gpurun_out/r04_gpu
mkdir -p $OUT
timeout -k 10 1100 python -u -m pytest -v -s --timeout 600 --timeout-method thread -m gpu tests/test_longrun.py \
    tests/test_fullsize.py > $OUT/pytest_b.txt 2>&1
