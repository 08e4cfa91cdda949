#!/usr/bin/env python3
"""Per-block start/end of k_onepass (diagnostic build, tools/stamp_diag.sh -> build_diag/libbpgl_stamp.so).

Usage: python tools/onepass_stamps.py [LIB] [M N]
Prints the launch span, start/end spreads, the mean end per XCD (blockIdx % 8) and per row group.
The stamp sits after the row loop, before the epilogue (line-search partials, U stores).
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "build_diag", "libbpgl_stamp.so")
    m = int(sys.argv[2]) if len(sys.argv) > 2 else 8192
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 65536
    import numpy as np
    import torch
    from convex_optimization_amd import _native
    _native.LIB_PATH = os.path.abspath(lib)
    from convex_optimization_amd.parameters import device_instance
    torch.cuda.set_device(0)
    gc, b, mu, _ = device_instance(m, n, 0.4, 1, TYPE="float", seed=1, device=0)
    L = _native.lib()
    L.bpgl_diag_stamps.argtypes = [ctypes.c_void_p]
    gc.solver_reset(b, mu, use_graph=False)
    out = {"m": m, "n": n, "launches": []}
    for it in range(6):
        gc.solver_step(1)
        gc.stream.synchronize()
        st = np.zeros((3, 2, 16384), dtype=np.uint64)
        assert L.bpgl_diag_stamps(st.ctypes.data_as(ctypes.c_void_p)) == 0
        nz = int(np.count_nonzero(st[2, 0]))
        s = st[2, 0, :nz].astype(np.float64) / 100.0
        e = st[2, 1, :nz].astype(np.float64) / 100.0
        t0 = s.min()
        s, e = s - t0, e - t0
        xcd = np.arange(nz) % 8
        rec = {"iter": it, "blocks": nz, "span_us": float(e.max()), "start_spread_us": float(s.max()),
               "end_min_us": float(e.min()), "end_median_us": float(np.median(e)),
               "end_by_xcd_us": [round(float(e[xcd == q].mean()), 1) for q in range(8)],
               "end_max_by_xcd_us": [round(float(e[xcd == q].max()), 1) for q in range(8)]}
        out["launches"].append(rec)
        print(json.dumps(rec))
    return out


if __name__ == "__main__":
    main()
