#!/bin/bash
# MFMA utilisation of the panel passes from counters.  Round 2 read
# SQ_VALU_MFMA_BUSY_CYCLES = 2^28 on both k = 128 passes and took it for a saturated counter; a pass
# at k = 128 issues exactly 2^24 v_mfma_f32_16x16x32_bf16 (2 m w k x 2 hi+lo pieces / 16384 flops),
# 16 busy cycles each = 2^28.  This pass collects the instruction count, the math-op count and the
# busy cycles together with GRBM_GUI_ACTIVE (kernel cycles x 8 XCDs), at k = 128 and k = 64 (2^23
# MFMAs: the counter must halve if it is not saturated).  One pass per k, 5 SQ + 1 GRBM counters.
# Usage (repo root, GPU box): tools/panel_mfma_pmc.sh
set -o pipefail
R=$(pwd)
OUT=$R/gpurun_out/panel_mfma
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
for K in 128 64; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_BF16 SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES \
      SQ_INSTS_MFMA SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/k$K --kernel-include-regex "k_panel_pass" -- \
      python3 $R/bench.py --rhs $K --steps 4 --warmup 2 --ramp 4 --windows 1 --no-cpu > $OUT/b_k$K.json 2> $OUT/k$K.err || exit 1
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -- \
    python3 $R/bench.py --config 4 --steps 100 --warmup 100 --no-cpu > $OUT/bench_trace.json 2> $OUT/trace.err || exit 1
cd $R
python3 tools/pmc_summary.py $OUT/k128 > $OUT/summary_k128.txt
python3 tools/pmc_summary.py $OUT/k64 > $OUT/summary_k64.txt
