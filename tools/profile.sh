#!/bin/bash
# Round profiles (GPU box, repo root; usage: tools/profile.sh [OUTDIR]): rocprofv3 kernel traces + stats
# of the driver's bench command
# (with and without the side legs: configs[3]'s k_onepass shares configs[1]'s instantiation, so only the
# leg-free trace gives configs[1]'s own average), of configs[4] and configs[3]; FETCH_SIZE / WRITE_SIZE
# passes over k_onepass (configs[1]) and the panel passes (configs[4]); the panel MFMA counters at
# k = 128 and 64.  Every counter pass is a run of its own (gfx950 counter limits; no --pmc with traces).
set -o pipefail
R=$(pwd)
OUT=$R/${1:-gpurun_out/prof}
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
B="python3 $R/bench.py"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_driver -- \
    $B --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/trace_driver.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_c1 -- \
    $B --gpus 1 --steps 20 --warmup 5 --no-cpu --no-side-legs > $OUT/bench_c1.json 2> $OUT/trace_c1.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/mfma/trace -- \
    $B --config 4 --steps 256 --warmup 200 --no-cpu > $OUT/bench_c4.json 2> $OUT/trace_c4.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_c3 -- \
    $B --config 3 --no-cpu > $OUT/bench_c3.json 2> $OUT/trace_c3.err || exit $?
C1="$B --steps 16 --warmup 4 --ramp 16 --windows 1 --no-cpu --no-side-legs"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch_c1 --kernel-include-regex "k_onepass" -- \
    $C1 > $OUT/b_fetch_c1.json 2> $OUT/fetch_c1.err || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write_c1 --kernel-include-regex "k_onepass" -- \
    $C1 > $OUT/b_write_c1.json 2> $OUT/write_c1.err || exit $?
C4="$B --rhs 128 --steps 8 --warmup 2 --ramp 8 --windows 1 --no-cpu"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch_c4 --kernel-include-regex "k_panel_pass" -- \
    $C4 > $OUT/b_fetch_c4.json 2> $OUT/fetch_c4.err || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write_c4 --kernel-include-regex "k_panel_pass" -- \
    $C4 > $OUT/b_write_c4.json 2> $OUT/write_c4.err || exit $?
for K in 128 64; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_BF16 SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES \
      SQ_INSTS_MFMA SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/mfma/k$K --kernel-include-regex "k_panel_pass" -- \
      $B --rhs $K --steps 8 --warmup 2 --ramp 8 --windows 1 --no-cpu > $OUT/b_k$K.json 2> $OUT/k$K.err || exit $?
done
