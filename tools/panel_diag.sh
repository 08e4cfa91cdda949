#!/bin/bash
# Build diagnostic variants of libbpgl.so (BPGL_PANEL_DIAG = 1: no A-side DMA after the
# prologue, 2: no RHS-side DMA, 3: neither, 4: half the lo operand pieces, 8: no lo pieces;
# DIAGS="4 8" picks the set) into build_diag/, for tools/panel_diag.py.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p $R/build_diag
for d in ${DIAGS:-1 2 3}; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -DBPGL_PANEL_DIAG=$d \
    -I$R/include $R/convex_optimization_amd/csrc/bpgl.hip $R/convex_optimization_amd/csrc/bpgl_panel_abi.hip -o $R/build_diag/libbpgl_d$d.so -lrccl &
done
wait
