#!/bin/bash
# Round 4: the panel path with the d_split = 1 default -- full panel tests, the 1000-iteration
# long horizon (both direction forms), and configs[4] benches (default, d_split 2, lo8 variants)
set -o pipefail
OUT=gpurun_out/r04_panel
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_panel.py tests/test_rowshard.py -k "gemms or in_kernel_fold or graph_equals" \
    > $OUT/pytest_panel.txt 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for V in "-1 -1" "2 -1"; do
  set -- $V
  timeout -k 10 240 python bench.py --config 4 --d-split $1 --lo8 $2 \
      > $OUT/bench_ds$1_lo8$2.json 2> $OUT/bench_ds$1_lo8$2.err || exit $?
done
