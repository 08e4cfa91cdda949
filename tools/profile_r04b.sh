#!/bin/bash
# Round-4 profiles of configs[4] with the carried gradient (the one-block default): rocprofv3 kernel
# trace + stats of the bench, FETCH_SIZE / WRITE_SIZE passes over the panel passes (pmc_traffic.json)
# and the MFMA counters at k = 128 and 64 (mfma_util.json).  The PMC runs take 64 timed + 64 eager
# iterations so the exact-gradient pass 1 (every 64th) enters the averages near its steady-state share.
set -o pipefail
R=$(pwd)
OUT=$R/gpurun_out/prof_r04b
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -- \
    python3 $R/bench.py --config 4 --steps 256 --warmup 200 --no-cpu > $OUT/bench_trace_c4.json 2> $OUT/trace_c4.err || exit $?
B="python3 $R/bench.py --rhs 128 --steps 64 --warmup 8 --ramp 64 --windows 1 --no-cpu"
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch_c4 --kernel-include-regex "k_panel_pass" -- \
    $B > $OUT/b_fetch.json 2> $OUT/fetch.err || exit $?
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write_c4 --kernel-include-regex "k_panel_pass" -- \
    $B > $OUT/b_write.json 2> $OUT/write.err || exit $?
for K in 128 64; do
  timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_BF16 SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES \
      SQ_INSTS_MFMA SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/k$K --kernel-include-regex "k_panel_pass" -- \
      python3 $R/bench.py --rhs $K --steps 64 --warmup 8 --ramp 64 --windows 1 --no-cpu > $OUT/b_k$K.json 2> $OUT/k$K.err || exit $?
done
