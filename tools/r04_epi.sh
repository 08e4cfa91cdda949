#!/bin/bash
# Round 4: the pass-1 epilogue with its loads issued ahead of the stores -- panel tests, then
# configs[4] benches (default, exact gradient, d_split 2)
set -o pipefail
OUT=gpurun_out/${OUT_DIR:-r04_epi}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_panel.py \
    > $OUT/pytest_panel.txt 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for V in "-1 -1" "0 -1" "-1 2"; do
  set -- $V
  timeout -k 10 240 python bench.py --config 4 --carry-g $1 --d-split $2 \
      > $OUT/bench_cg$1_ds$2.json 2> $OUT/bench_cg$1_ds$2.err || exit $?
done
