#!/bin/bash
# Timing-only builds of the panel library (results wrong) that drop parts of the pass-1 epilogue:
# BPGL_PANEL_DIAG bit 0 no carried-G store, bit 1 no D' store, bit 3 no epilogue loop.  Built here
# (CPU) into build_diag/epiN/libbpgl.so; run on the GPU box with BPGL_LIB=build_diag/epiN/libbpgl.so.
set -e
cd "$(dirname "$0")/../convex_optimization_amd/csrc"
for D in ${@:-1 2 3 8}; do
  O=../../build_diag/epi$D
  mkdir -p $O
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -DBPGL_PANEL_DIAG=$D -c -o $O/bpgl_panel_abi.o bpgl_panel_abi.hip
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $O/libbpgl.so ../_lib/bpgl.o $O/bpgl_panel_abi.o -lrccl
done
