#!/bin/bash
# Round 4 closing: the whole -m gpu suite (short + long), smoke(), the default bench and configs[4]
set -o pipefail
OUT=gpurun_out/r04_final
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests \
    --ignore=tests/test_longrun.py --ignore=tests/test_fullsize.py > $OUT/pytest_a.txt 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 1100 python -u -m pytest -v -s --timeout 600 --timeout-method thread -m gpu tests/test_longrun.py \
    tests/test_fullsize.py > $OUT/pytest_b.txt 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || exit $?
timeout -k 10 300 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || exit $?
timeout -k 10 240 python bench.py --config 4 > $OUT/bench_config4.json 2> $OUT/bench_config4.err || exit $?
