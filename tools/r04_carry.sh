#!/bin/bash
# Round 4: the carried-gradient panel form (carry_g) -- parity tests, configs[4] benches against the
# default, and the 1000-iteration accuracy at configs[4] for g_refresh 32 / 64 / 128
set -o pipefail
OUT=gpurun_out/r04_carry
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_panel.py -k "carried" \
    > $OUT/pytest_carry.txt 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for V in "0 64" "1 64" "1 32" "1 128"; do
  set -- $V
  timeout -k 10 240 python bench.py --config 4 --carry-g $1 --g-refresh $2 \
      > $OUT/bench_cg$1_$2.json 2> $OUT/bench_cg$1_$2.err || exit $?
done
timeout -k 10 400 python -u tools/panel_lo8_accuracy.py 1000 0:0:1 0:0:1:1:32 0:0:1:1:64 0:0:1:1:128 \
    > $OUT/accuracy.jsonl 2> $OUT/accuracy.err
