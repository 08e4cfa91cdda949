#!/bin/bash
# configs[4] panel: pass 1 wide split-K form (interleave1 = 4) against the 256-column form
set -o pipefail
OUT=gpurun_out/panel_wide
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_panel.py -x -q --timeout 200 --timeout-method thread \
    -k "wide or interleave or full_configs4" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
run() { local n=$1; shift; timeout -k 10 200 python3 bench.py --steps 64 --warmup 100 --windows 3 --no-cpu "$@" > $OUT/$n.json 2> $OUT/$n.err || exit 1; }
run base --rhs 128
run w4 --rhs 128 --interleave1 4
run w4_k64 --rhs 64 --interleave1 4
run base_k64 --rhs 64
run w4_again --rhs 128 --interleave1 4
run base_again --rhs 128
python3 tools/summarize_bench.py $OUT/*.json
