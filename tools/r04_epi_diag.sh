#!/bin/bash
# timing of the pass-1 epilogue parts (tools/panel_epi_diag.sh builds; results wrong by design)
set -o pipefail
OUT=gpurun_out/r04_epi_diag
mkdir -p $OUT
run() {  # name, lib
  BPGL_LIB=$2 timeout -k 10 240 python bench.py --config 4 --steps 64 --windows 2 > $OUT/bench_$1.json 2> $OUT/bench_$1.err
  rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
run base convex_optimization_amd/_lib/libbpgl.so
for D in 1 2 3 8; do run epi$D build_diag/epi$D/libbpgl.so; done
run base2 convex_optimization_amd/_lib/libbpgl.so
