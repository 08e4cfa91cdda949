#!/bin/bash
# Round 4: configs[4] accuracy over 1000 iterations for the direction / residual precision forms
set -o pipefail
OUT=gpurun_out/r04_acc
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_panel.py -k lo8 \
    > $OUT/pytest_lo8.txt 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python tools/panel_lo8_accuracy.py 1000 0:0:2 0:0:1 2:128:2 2:0:2 1:0:2 0:0:1 > $OUT/accuracy.jsonl 2> $OUT/accuracy.err &&
timeout -k 10 200 python tools/panel_lo8_accuracy.py 2000 0:0:2 0:0:1 2:128:2 > $OUT/accuracy_2000.jsonl 2> $OUT/accuracy_2000.err
