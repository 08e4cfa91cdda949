#!/bin/bash
# Round-4 profiles (GPU box, repo root): rocprofv3 kernel trace + stats of the default bench
# (configs[1]) and of configs[4] (panel, d_split 1 default); FETCH_SIZE / WRITE_SIZE passes over the
# panel passes (pmc_traffic.json panel entry) and the MFMA counters at k = 128 and 64
# (mfma_util.json).  Every pass is a separate rocprofv3 run (counter limits; no --pmc with traces).
set -o pipefail
R=$(pwd)
OUT=$R/gpurun_out/prof_r04
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_c1 -- \
    python3 $R/bench.py --steps 256 --warmup 100 --no-cpu > $OUT/bench_trace_c1.json 2> $OUT/trace_c1.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_c4 -- \
    python3 $R/bench.py --config 4 --steps 100 --warmup 100 --no-cpu > $OUT/bench_trace_c4.json 2> $OUT/trace_c4.err || exit $?
B="python3 $R/bench.py --rhs 128 --steps 6 --warmup 2 --ramp 6 --windows 1 --no-cpu"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch_c4 --kernel-include-regex "k_panel_pass" -- \
    $B > $OUT/b_fetch.json 2> $OUT/fetch.err || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write_c4 --kernel-include-regex "k_panel_pass" -- \
    $B > $OUT/b_write.json 2> $OUT/write.err || exit $?
for K in 128 64; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_BF16 SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES \
      SQ_INSTS_MFMA SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/mfma_k$K --kernel-include-regex "k_panel_pass" -- \
      python3 $R/bench.py --rhs $K --steps 4 --warmup 2 --ramp 4 --windows 1 --no-cpu > $OUT/b_k$K.json 2> $OUT/k$K.err || exit $?
done
