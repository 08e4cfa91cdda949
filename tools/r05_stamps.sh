#!/bin/bash
# Round 5: k_onepass per-block timelines (diagnostic stamp build, tools/stamp_diag.sh) at the shapes
# the multi-GPU legs give one GPU: configs[1] (8192 x 65536), the N = 8 strong shard (1024 x 65536)
# and the configs[2] weak shard (1024 x 524288), the latter two as row shards.
set -o pipefail
OUT=${1:-gpurun_out/r05_stamps}
mkdir -p $OUT
L=build_diag/libbpgl_stamp.so
timeout -k 10 120 python3 tools/onepass_stamps.py $L 8192 65536 > $OUT/m8192.jsonl 2> $OUT/m8192.err || exit $?
timeout -k 10 120 python3 tools/onepass_stamps.py $L 1024 65536 --rows > $OUT/m1024_rows.jsonl 2> $OUT/m1024_rows.err || exit $?
timeout -k 10 120 python3 tools/onepass_stamps.py $L 1024 65536 > $OUT/m1024_one.jsonl 2> $OUT/m1024_one.err || exit $?
timeout -k 10 180 python3 tools/onepass_stamps.py $L 1024 524288 --rows > $OUT/m1024w_rows.jsonl 2> $OUT/m1024w_rows.err || exit $?
