#!/bin/bash
# Pass times of the panel mainloop variants with the LDS-DMA streams removed (diagnostic builds,
# tools/panel_diag.sh: d1 no A stream, d2 no k-wide stream, d3 neither; results are wrong, only
# the timing matters) -> gpurun_out/panel_diag_stag/*.json
set -o pipefail
OUT=gpurun_out/panel_diag_stag
mkdir -p $OUT
for d in 3 1 2; do
  for v in 12 33; do
    a=${v:0:1}; b=${v:1:1}
    BPGL_LIB=build_diag/libbpgl_d$d.so timeout -k 10 200 python3 bench.py --config 4 --steps 64 --warmup 100 --windows 1 \
        --interleave1 $a --interleave2 $b > $OUT/d${d}_i$v.json 2> $OUT/d${d}_i$v.err || exit 1
  done
done
