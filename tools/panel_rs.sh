#!/bin/bash
# configs[4] panel: register-staged LDS images (interleave 4) against the LDS-DMA forms
set -o pipefail
OUT=gpurun_out/panel_rs
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_panel.py -x -q --timeout 200 --timeout-method thread \
    -k "interleave" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
run() { local n=$1; shift; timeout -k 10 200 python3 bench.py --steps 64 --warmup 100 --windows 3 --no-cpu "$@" > $OUT/$n.json 2> $OUT/$n.err || exit 1; }
run base --rhs 128
run rs44 --rhs 128 --interleave 4
run rs4_p1 --rhs 128 --interleave1 4
run rs4_p2 --rhs 128 --interleave2 4
run rs44_k64 --rhs 64 --interleave 4
run rs44_ds1 --rhs 128 --interleave 4 --d-split 1
run base_again --rhs 128
python3 tools/summarize_bench.py $OUT/*.json
