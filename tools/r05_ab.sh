#!/bin/bash
# Round 5 A/B helper (GPU box): stamps at 8192 x 65536 and the N = 8 strong row shard, then the
# bench lines of configs[1], the strong shard (one-rank RCCL row leg), the configs[2] weak shard
# and configs[4].  usage: tools/r05_ab.sh OUTDIR [skip_stamps]
set -o pipefail
OUT=${1:-gpurun_out/r05_ab}
mkdir -p $OUT
L=build_diag/libbpgl_stamp.so
if [ -z "$2" ]; then
timeout -k 10 120 python3 tools/onepass_stamps.py $L 8192 65536 > $OUT/st_m8192.jsonl 2> $OUT/st_m8192.err || exit $?
timeout -k 10 120 python3 tools/onepass_stamps.py $L 1024 65536 --rows > $OUT/st_m1024_rows.jsonl 2> $OUT/st_m1024_rows.err || exit $?
fi
B="python3 bench.py --no-cpu --no-side-legs"
timeout -k 10 200 $B --steps 256 --warmup 200 --windows 5 > $OUT/c1.json 2> $OUT/c1.err || exit $?
timeout -k 10 200 $B --comm --shard rows --m 1024 --n-per-gpu 65536 --steps 256 --warmup 100 --windows 5 > $OUT/m1024.json 2> $OUT/m1024.err || exit $?
timeout -k 10 200 $B --comm --shard rows --m 1024 --n-per-gpu 524288 --steps 256 --warmup 100 --windows 3 > $OUT/m1024w.json 2> $OUT/m1024w.err || exit $?
timeout -k 10 200 $B --config 4 --steps 256 --warmup 200 --windows 5 > $OUT/c4.json 2> $OUT/c4.err || exit $?
