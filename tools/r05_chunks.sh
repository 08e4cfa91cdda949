#!/bin/bash
# Chunked row interleave ("onepass_rows" C): GPU tests of the changed paths, then C swept per shape on one box.
set -o pipefail
OUT=${1:-gpurun_out/r05_chunks}
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_onepass.py \
    tests/test_rowshard.py > $OUT/pytest.txt 2>&1 || exit $?
B="python3 bench.py --no-cpu --no-side-legs"
for v in 0 1 4 16 64; do
  timeout -k 10 200 $B --config 3 --steps 64 --warmup 20 --windows 3 --onepass-rows $v > $OUT/c3_r${v}.json 2> $OUT/c3_r${v}.err || exit $?
done
for v in 1 4 16; do
  timeout -k 10 200 $B --steps 256 --warmup 100 --windows 5 --onepass-rows $v > $OUT/c1_r${v}.json 2> $OUT/c1_r${v}.err || exit $?
  timeout -k 10 200 $B --comm --shard rows --m 4096 --n-per-gpu 65536 --steps 256 --warmup 100 --windows 5 \
      --onepass-rows $v > $OUT/m4096_r${v}.json 2> $OUT/m4096_r${v}.err || exit $?
done
for v in 0 1 4 16; do
  timeout -k 10 200 $B --comm --shard rows --m 1024 --n-per-gpu 65536 --steps 256 --warmup 100 --windows 5 \
      --onepass-rows $v > $OUT/m1024_r${v}.json 2> $OUT/m1024_r${v}.err || exit $?
done
for v in 0 4 16 64; do
  timeout -k 10 200 $B --comm --shard rows --m 1024 --n-per-gpu 524288 --steps 256 --warmup 50 --windows 3 \
      --onepass-rows $v > $OUT/m1024w_r${v}.json 2> $OUT/m1024w_r${v}.err || exit $?
done
