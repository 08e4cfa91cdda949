#!/bin/bash
# One-pass cache-allocating share sweep (tuning key onepass_cache_permille) at configs[1] and
# configs[3] -> gpurun_out/opcache.jsonl; run on the GPU box.
OUT=gpurun_out/opcache.jsonl
: > $OUT
for cfg in 1 3; do
  for c in 0 50 100 150 200 300; do
    timeout -k 10 200 python bench.py --config $cfg --onepass-cache $c --no-cpu --steps 100 > gpurun_out/_c.json 2>/dev/null || exit 1
    python3 -c "
import json; d=json.load(open('gpurun_out/_c.json')); r=d['roofline']
print(json.dumps({'config': $cfg, 'cache_permille': $c, 'it_s': d['value'], 'onepass_ms': r['avg_launch_ms'], 'frac': r['frac']}))" >> $OUT
  done
done
cat $OUT
