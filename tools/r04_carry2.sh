#!/bin/bash
# Round 4: carry_g as the one-block default -- the whole panel test file, the panel long horizon
# (exact and carried forms), the full-size panel checks, then configs[4] benches
set -o pipefail
OUT=gpurun_out/${OUT_DIR:-r04_carry2}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_panel.py \
    > $OUT/pytest_panel.txt 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 900 python -u -m pytest -v -s --timeout 600 --timeout-method thread tests/test_longrun.py -k panel \
    > $OUT/pytest_longrun.txt 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 240 python bench.py --config 4 > $OUT/bench_default.json 2> $OUT/bench_default.err || exit $?
timeout -k 10 240 python bench.py --config 4 --carry-g 0 > $OUT/bench_cg0.json 2> $OUT/bench_cg0.err || exit $?
timeout -k 10 240 python bench.py --config 4 --interleave 3 > $OUT/bench_il3.json 2> $OUT/bench_il3.err || exit $?
timeout -k 10 240 python bench.py --config 4 --defer-x 1 > $OUT/bench_dx1.json 2> $OUT/bench_dx1.err || exit $?
