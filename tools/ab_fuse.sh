#!/bin/bash
# A/B of the fused one-pass tail ("tail_fuse" 0 vs 1) on one library build, alternating, two
# repetitions, at configs[1] (256/200 and the driver's 20/5), configs[3] and the N = 8 / N = 4 strong
# row shards on one GPU (m = 1024 / 2048) -> gpurun_out/ab/fuse.txt
set -o pipefail
mkdir -p gpurun_out/ab
OUT=gpurun_out/ab/fuse.txt
: > $OUT
run() {
  timeout -k 10 200 python bench.py --no-cpu "$@" > gpurun_out/ab/_f.json 2> gpurun_out/ab/_f.err || { tail -5 gpurun_out/ab/_f.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/ab/_f.json')); k=d['config']['kernel_avg_ms']
print('$*', round(d['value'],1), 'it/s', round(d['ms_per_step']*1e3,1), 'us', {a: round(b*1e3,1) for a,b in k.items() if b})" >> $OUT
}
for rep in 1 2; do
  for f in 0 1; do
    run --tail-fuse $f --steps 256 --warmup 200
    run --tail-fuse $f --steps 20 --warmup 5
    run --tail-fuse $f --config 3 --steps 64 --warmup 20 --ramp 64
    run --tail-fuse $f --m 1024 --steps 256 --warmup 200
    run --tail-fuse $f --m 2048 --steps 256 --warmup 200
  done
done
cat $OUT
