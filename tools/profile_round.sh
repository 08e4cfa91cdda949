#!/bin/bash
# Profile the bench workloads on the GPU box: kernel trace + stats of configs[1] (default bench) and
# of configs[3], then two separate PMC passes (FETCH_SIZE, WRITE_SIZE) over configs[1], then the
# per-launch traffic summary.  Usage (from the repo root, on the GPU box): tools/profile_round.sh TAG
# Outputs under gpurun_out/prof_TAG/ (pmc_traffic.json there = profiles/pmc_traffic.json updated).
set -e
R=$(pwd)
TAG=${1:-r01}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -- \
    python3 $R/bench.py --steps 256 --warmup 100 --no-cpu > $OUT/bench_trace.json 2> $OUT/trace.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_c3 -- \
    python3 $R/bench.py --config 3 --steps 30 --warmup 40 --no-cpu > $OUT/bench_trace_c3.json 2> $OUT/trace_c3.err
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch \
    --kernel-include-regex "k_iter_a|k_iter_b|k_colpass|k_rowpass|k_onepass" -- \
    python3 $R/bench.py --steps 6 --warmup 2 --no-cpu > $OUT/bench_fetch.json 2> $OUT/fetch.err
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write \
    --kernel-include-regex "k_iter_a|k_iter_b|k_colpass|k_rowpass|k_onepass" -- \
    python3 $R/bench.py --steps 6 --warmup 2 --no-cpu > $OUT/bench_write.json 2> $OUT/write.err
cd $R
cp profiles/pmc_traffic.json $OUT/pmc_traffic.json
PMC_OUT=$OUT/pmc_traffic.json python3 tools/pmc_traffic.py $OUT/fetch $OUT/write m8192_n65536_b1_float_g1 \
    $((8192*65536*4 + 8*8192 + 16*65536)) > $OUT/pmc_summary.json
