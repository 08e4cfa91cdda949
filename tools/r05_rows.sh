#!/bin/bash
# Interleaved one-pass row groups ("onepass_rows") across the one-pass shapes, same box, same library:
# configs[1], the N = 2 / 4 / 8 strong row shards (4096 / 2048 / 1024 rows), the weak shard, configs[3];
# then configs[4] with the stage-major pass-2 tiles.  GPU tests of the changed paths first.
set -o pipefail
OUT=${1:-gpurun_out/r05_rows}
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_onepass.py \
    tests/test_rowshard.py tests/test_panel.py > $OUT/pytest.txt 2>&1 || exit $?
B="python3 bench.py --no-cpu --no-side-legs"
for r in 1 2; do
  for v in 0 1; do
    timeout -k 10 200 $B --steps 256 --warmup 100 --windows 5 --onepass-rows $v > $OUT/c1_r${v}_$r.json 2> $OUT/c1_r${v}_$r.err || exit $?
    for m in 4096 2048 1024; do
      timeout -k 10 200 $B --comm --shard rows --m $m --n-per-gpu 65536 --steps 256 --warmup 100 --windows 5 \
          --onepass-rows $v > $OUT/m${m}_r${v}_$r.json 2> $OUT/m${m}_r${v}_$r.err || exit $?
    done
  done
done
timeout -k 10 200 python3 bench.py --config 4 --no-cpu --steps 256 --warmup 200 > $OUT/c4.json 2> $OUT/c4.err || exit $?
