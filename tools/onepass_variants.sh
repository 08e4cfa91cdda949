#!/bin/bash
# One-pass ring-depth / prefetch variants (tuning key onepass_variant) per storage type at
# configs[1] (and configs[3] for fp32) -> gpurun_out/opvar.jsonl; run on the GPU box.
OUT=gpurun_out/opvar.jsonl
: > $OUT
for t in float double bf16; do
  for v in 0 1 2 3; do
    timeout -k 10 200 python bench.py --type $t --onepass-variant $v --no-cpu --steps 100 > gpurun_out/_v.json 2>/dev/null || exit 1
    python3 -c "
import json; d=json.load(open('gpurun_out/_v.json')); r=d['roofline']
print(json.dumps({'type': '$t', 'config': 1, 'variant': $v, 'it_s': d['value'], 'onepass_ms': r['avg_launch_ms'], 'frac': r['frac']}))" >> $OUT
  done
done
for v in 0 1 2 3; do
  timeout -k 10 200 python bench.py --config 3 --onepass-variant $v --no-cpu > gpurun_out/_v.json 2>/dev/null || exit 1
  python3 -c "
import json; d=json.load(open('gpurun_out/_v.json')); r=d['roofline']
print(json.dumps({'type': 'float', 'config': 3, 'variant': $v, 'it_s': d['value'], 'onepass_ms': r['avg_launch_ms'], 'frac': r['frac']}))" >> $OUT
done
cat $OUT
