#!/bin/bash
# Round 4: the e4m3 lo products of the panel path (configs[4]) -- parity tests, bench per lo8
# setting, and the long-horizon accuracy against the oracle fixture.
set -o pipefail
OUT=gpurun_out/r04_lo8
mkdir -p $OUT
timeout -k 10 60 tools/_mfma_f8_probe > $OUT/mfma_f8_probe.txt 2>&1 &&
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_panel.py -k lo8 \
    > $OUT/pytest_lo8.txt 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi   # test failures (1) still run the benches
for V in "0 -1 -1" "0 1 -1" "1 -1 -1" "1 1 -1" "2 -1 -1" "2 -1 2" "3 -1 -1"; do
  set -- $V
  timeout -k 10 240 python bench.py --config 4 --lo8 $1 --interleave1 $2 --interleave2 $3 \
      > $OUT/bench_lo8_$1_il$2_$3.json 2> $OUT/bench_lo8_$1_il$2_$3.err || exit $?
done &&
timeout -k 10 300 python tools/panel_lo8_accuracy.py 1000 0:0 1:0 2:0 2:128 3:128 3:64 > $OUT/accuracy.jsonl 2> $OUT/accuracy.err
