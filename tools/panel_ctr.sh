#!/bin/bash
# Load-path counters of the panel passes at k = 64 and k = 128: TA / TD /
# TCP busy and stall cycles beside GRBM_GUI_ACTIVE, each group in its own --pmc pass (slot limits:
# 2 TA, 2 TD, 4 TCP, 2 GRBM).  Usage (repo root, GPU box): tools/panel_ctr.sh -> gpurun_out/panel_ctr/
set -e
R=$(pwd)
OUT=$R/gpurun_out/panel_ctr
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
for K in 64 128; do
  B="python3 $R/bench.py --rhs $K --steps 6 --warmup 2 --windows 1 --ramp 8 --no-cpu"
  p=0
  for C in "TA_TA_BUSY TA_DATA_STALLED_BY_TC_CYCLES GRBM_GUI_ACTIVE" \
           "TA_ADDR_STALLED_BY_TC_CYCLES TA_BUFFER_READ_LDS_WAVEFRONTS GRBM_GUI_ACTIVE" \
           "TD_TD_BUSY TD_TC_STALL GRBM_GUI_ACTIVE" \
           "TCP_PENDING_STALL_CYCLES TCP_TCR_TCP_STALL_CYCLES TCP_TCP_TA_DATA_STALL_CYCLES TCP_READ_TAGCONFLICT_STALL_CYCLES"; do
    p=$((p+1))
    timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $OUT/k${K}_p$p --kernel-include-regex "k_panel_pass" -- \
        $B > $OUT/b_k${K}_p$p.json 2> $OUT/k${K}_p$p.err
  done
done
cd $R
for K in 64 128; do echo "== k=$K"; python3 tools/pmc_summary.py $OUT/k${K}_p1 $OUT/k${K}_p2 $OUT/k${K}_p3 $OUT/k${K}_p4; done > $OUT/summary.txt
cat $OUT/summary.txt
