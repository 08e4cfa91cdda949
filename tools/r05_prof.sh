#!/bin/bash
# Round 5 baselines (GPU box, repo root): rocprofv3 kernel traces of configs[4] (panel), the N = 8
# strong shard 1024 x 65536 and the configs[2] weak shard 1024 x 524288 (both through the one-rank
# RCCL row leg), and the bench lines beside them.  usage: tools/r05_prof.sh OUTDIR
set -o pipefail
R=$(pwd)
OUT=$R/${1:-gpurun_out/r05_prof}
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
B="python3 $R/bench.py --no-cpu --no-side-legs"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_c4 -- \
    $B --config 4 --steps 100 --warmup 100 > $OUT/bench_c4.json 2> $OUT/c4.err || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_m1024 -- \
    $B --comm --shard rows --m 1024 --n-per-gpu 65536 --steps 256 --warmup 100 --windows 3 > $OUT/bench_m1024.json 2> $OUT/m1024.err || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_m1024w -- \
    $B --comm --shard rows --m 1024 --n-per-gpu 524288 --steps 64 --warmup 32 --windows 3 > $OUT/bench_m1024w.json 2> $OUT/m1024w.err || exit $?
