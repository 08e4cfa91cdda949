#!/bin/bash
set -o pipefail
OUT=gpurun_out/r04_tail
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_panel.py -k fused > $OUT/pytest.txt 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for F in 0 1 0 1; do
  timeout -k 10 240 python bench.py --config 4 --fuse-tail $F > $OUT/bench_ft$F.json 2> $OUT/bench_ft$F.err || exit $?
  python -c "import json; d=json.load(open('$OUT/bench_ft$F.json')); print($F, d['value'], d['config']['kernel_avg_ms'])" >> $OUT/summary.txt
done
