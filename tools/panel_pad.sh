#!/bin/bash
# configs[4] panel: row pitch of the operand images (op_pad) and of A (lda_pad) -> gpurun_out/panel_pad/
set -o pipefail
OUT=gpurun_out/panel_pad
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_panel.py -x -q --timeout 200 --timeout-method thread \
    -k "padded or interleave or full_configs4" > $OUT/pytest.log 2>&1 || { tail -20 $OUT/pytest.log; exit 1; }
run() { local n=$1; shift; timeout -k 10 200 python3 bench.py --config 4 --steps 64 --warmup 100 --windows 3 --no-cpu "$@" > $OUT/$n.json 2> $OUT/$n.err || exit 1; }
run base
run op64 --op-pad 64
run lda64 --lda-pad 64
run both64 --op-pad 64 --lda-pad 64
run op256 --op-pad 256
run lda256 --lda-pad 256
run base_again
python3 tools/summarize_bench.py $OUT/*.json
