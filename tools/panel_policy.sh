#!/bin/bash
# Cache-policy variants of the panel path's LDS-DMA streams (configs[4]): the default library
# (A nt = aux 2, k-wide operand default) against diagnostic builds in build_diag/ with other
# aux bits (BPGL_PANEL_A_AUX / BPGL_PANEL_O_AUX) -> gpurun_out/panel_policy.jsonl
OUT=gpurun_out/panel_policy.jsonl
: > $OUT
for rep in 1 2; do
  for v in default a1 a3 o2; do
    if [ $v = default ]; then L=""; else L=build_diag/libbpgl_panel_$v.so; fi
    BPGL_LIB=$L timeout -k 10 200 python bench.py --config 4 --no-cpu --steps 100 > gpurun_out/_p.json 2>/dev/null || exit 1
    python3 -c "
import json; d=json.load(open('gpurun_out/_p.json')); k=d['config']['kernel_avg_ms']
print(json.dumps({'variant': '$v', 'rep': $rep, 'it_s': d['value'], 'pass1_us': k['pass1_mfma']*1e3, 'pass2_us': k['pass2_mfma']*1e3, 'update_us': k['update']*1e3}))" >> $OUT
  done
done
cat $OUT
