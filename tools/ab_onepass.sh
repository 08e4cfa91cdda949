#!/bin/bash
# A/B of two in-tree builds of libbpgl.so on the one-pass shapes: build_diag/libbpgl_before.so
# against the current _lib/libbpgl.so, alternating, two repetitions -> gpurun_out/ab/<name>.txt
# (usage: bash tools/ab_onepass.sh <name>)
set -o pipefail
N=${1:-ab}
mkdir -p gpurun_out/ab
OUT=gpurun_out/ab/$N.txt
: > $OUT
run() {   # label lib args...
  local label=$1 lib=$2; shift 2
  BPGL_LIB=$lib timeout -k 10 200 python bench.py --no-cpu "$@" > gpurun_out/ab/_b.json 2> gpurun_out/ab/_b.err || { tail -5 gpurun_out/ab/_b.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/ab/_b.json')); k=d['config']['kernel_avg_ms']
print('$label', '$*', round(d['value'],1), 'it/s', {a: round(b*1e3,1) for a,b in k.items() if b})" >> $OUT
}
for rep in 1 2; do
  for lib in build_diag/libbpgl_before.so convex_optimization_amd/_lib/libbpgl.so; do
    L=$(basename $lib .so)
    run $L $lib --steps 256 --warmup 200
    run $L $lib --config 3 --steps 64 --warmup 20 --ramp 64
    run $L $lib --m 1024 --steps 256 --warmup 200
    run $L $lib --m 2048 --steps 256 --warmup 200
    run $L $lib --m 1024 --comm --shard rows --steps 256 --warmup 200
  done
done
cat $OUT
