#!/bin/bash
# configs[4]: the panel passes across a 1516-iteration solve, per dispatch, to compare early and late
# iterations: clock (GRBM_GUI_ACTIVE), then HBM writes and fetches -- one counter pass each, no traces.
set -o pipefail
R=$(pwd)
OUT=$R/${1:-gpurun_out/r05_c4clock}
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
B="python3 $R/bench.py --rhs 128 --steps 8 --warmup 1500 --ramp 8 --windows 1 --no-cpu"
if [ -z "$SKIP_CLOCK" ]; then
timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --output-format csv \
    -d $OUT/pmc --kernel-include-regex "k_panel_pass" -- $B > $OUT/b.json 2> $OUT/b.err || exit $?
fi
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv \
    -d $OUT/write --kernel-include-regex "k_panel" -- $B > $OUT/bw.json 2> $OUT/bw.err || exit $?
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv \
    -d $OUT/fetch --kernel-include-regex "k_panel" -- $B > $OUT/bf.json 2> $OUT/bf.err || exit $?
