#!/bin/bash
# Round 5: the whole -m gpu suite (short + long), smoke(), the driver-shape bench (every N = 1 leg).
# usage: tools/r05_check.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/r05_check}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests \
    --ignore=tests/test_longrun.py --ignore=tests/test_fullsize.py > $OUT/pytest_a.txt 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 900 python -u -m pytest -v -s --timeout 600 --timeout-method thread -m gpu tests/test_longrun.py \
    tests/test_fullsize.py > $OUT/pytest_b.txt 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || exit $?
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_n1.json 2> $OUT/bench_n1.err || exit $?
