#!/bin/bash
# Running clock of the panel passes with and without the lo MFMAs (diagnostic build
# build_diag/libbpgl_d16.so from `DIAGS=16 tools/panel_diag.sh`): kernel cycles from GRBM_GUI_ACTIVE / 8
# (one counter pass) over the kernel-trace duration (a separate run), per library.
# Usage (repo root, GPU box): [LIBS="name:path ..."] tools/panel_clock.sh -> gpurun_out/panel_clock/
set -o pipefail
R=$(pwd)
OUT=$R/gpurun_out/panel_clock
mkdir -p $OUT
export TMPDIR=/tmp PANEL_DIAG_WARMUP=300
cd /tmp
for L in ${LIBS:-shipped:$R/convex_optimization_amd/_lib/libbpgl.so nolo:$R/build_diag/libbpgl_d16.so}; do
  n=${L%%:*}; lib=${L#*:}
  timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES --output-format csv \
      -d $OUT/pmc_$n --kernel-include-regex "k_panel_pass" -- python3 $R/tools/panel_diag.py $lib 128 -1 \
      > $OUT/pmc_$n.json 2> $OUT/pmc_$n.err || exit 1
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_$n -- \
      python3 $R/tools/panel_diag.py $lib 128 -1 > $OUT/trace_$n.json 2> $OUT/trace_$n.err || exit 1
done
