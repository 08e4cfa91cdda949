#!/bin/bash
# Round 4: deferred x update (defer_x) with the prefetching pass-1 epilogue -- panel tests, then
# configs[4] with defer_x 0 / 1, twice each (alternating)
set -o pipefail
OUT=gpurun_out/${OUT_DIR:-r04_dx}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_panel.py \
    > $OUT/pytest_panel.txt 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for R in 1 2; do
  for D in 0 1; do
    timeout -k 10 240 python bench.py --config 4 --defer-x $D > $OUT/bench_dx${D}_$R.json 2> $OUT/bench_dx${D}_$R.err || exit $?
  done
done
