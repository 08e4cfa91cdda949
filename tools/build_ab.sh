#!/bin/bash
# Build libbpgl.so from the sources at a git ref (or the working tree: "WT") into build_ab/NAME.so,
# for same-box A/B runs (BPGL_LIB=build_ab/NAME.so selects it; convex_optimization_amd/_native.py).
# usage: tools/build_ab.sh REF NAME [extra hipcc flags...]   (build container only)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
REF=$1; NAME=$2; shift 2
SRC=$(mktemp -d /tmp/ab_src.XXXXXX)
if [ "$REF" = "WT" ]; then
  mkdir -p $SRC/convex_optimization_amd && cp -r $R/convex_optimization_amd/csrc $SRC/convex_optimization_amd/ && cp -r $R/include $SRC/
else
  git -C $R archive $REF convex_optimization_amd/csrc include | tar -x -C $SRC
fi
mkdir -p $R/build_ab
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared "$@" -I$SRC/include \
    $SRC/convex_optimization_amd/csrc/bpgl.hip $SRC/convex_optimization_amd/csrc/bpgl_panel_abi.hip \
    -o $R/build_ab/$NAME.so -lrccl
rm -rf $SRC
echo "built build_ab/$NAME.so from $REF"
