#!/bin/bash
# bf16 one-pass ring variants at configs[1] shape -> gpurun_out/bf16var.jsonl (run on the GPU box)
OUT=gpurun_out/bf16var.jsonl
: > $OUT
for v in 0 1 2 3; do
  timeout -k 10 200 python bench.py --type bf16 --onepass-variant $v --no-cpu --steps 100 > gpurun_out/_b.json 2>/dev/null || exit 1
  python3 -c "
import json; d=json.load(open('gpurun_out/_b.json')); r=d['roofline']
print(json.dumps({'type': 'bf16', 'variant': $v, 'it_s': d['value'], 'onepass_ms': r['avg_launch_ms'], 'frac': r['frac']}))" >> $OUT
done
cat $OUT
