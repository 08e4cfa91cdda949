#!/bin/bash
# Diagnostic build with per-block start/end stamps in k_colpass / k_rowpass
# (-DBPGL_STAMP=1) -> build_diag/libbpgl_stamp.so, read by tools/stamp_diag.py.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p $R/build_diag
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -DBPGL_STAMP=1 -I$R/include \
    $R/convex_optimization_amd/csrc/bpgl.hip $R/convex_optimization_amd/csrc/bpgl_panel_abi.hip -o $R/build_diag/libbpgl_stamp.so -lrccl
