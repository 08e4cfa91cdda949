#!/bin/bash
# PMC passes for the panel (configs[4]) MFMA kernels on the GPU box.
# Usage (repo root, GPU box): tools/profile_panel.sh TAG [K]
set -e
R=$(pwd)
TAG=${1:-panel}
K=${2:-128}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
B="python3 $R/bench.py --rhs $K --steps 6 --warmup 2 --no-cpu"
RX="k_panel_pass"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -- \
    python3 $R/bench.py --rhs $K --steps 100 --warmup 100 --no-cpu > $OUT/bench_trace.json 2> $OUT/trace.err
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $OUT/sq \
    --kernel-include-regex "$RX" -- $B > $OUT/b_sq.json 2> $OUT/sq.err
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_UNALIGNED_STALL GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum \
    --output-format csv -d $OUT/mix --kernel-include-regex "$RX" -- $B > $OUT/b_mix.json 2> $OUT/mix.err
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch --kernel-include-regex "$RX" -- \
    $B > $OUT/b_fetch.json 2> $OUT/fetch.err
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write --kernel-include-regex "$RX" -- \
    $B > $OUT/b_write.json 2> $OUT/write.err
cd $R
python3 tools/pmc_summary.py $OUT > $OUT/summary.txt
python3 tools/pmc_traffic.py $OUT/fetch $OUT/write panel_m8192_n65536_k$K $((2*8192*65536 + 8*$K*(8192+65536)))
cat $OUT/summary.txt
