#!/usr/bin/env python3
"""Ramp/tail of k_colpass and k_rowpass from per-block stamps (diagnostic build).

Build: hipcc ... -DBPGL_STAMP=1 -> build_diag/libbpgl_stamp.so (tools/panel_diag.sh style)
Usage: python tools/stamp_diag.py [LIB] [M N]
Prints, per kernel, the launch span, start and end spreads and block durations (us).
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
    geo = gc.geometry()
    nb = geo["nseg"] * geo["nchunk"]
    gc.solver_reset(b, mu, use_graph=False)
    gc.solver_step(5)
    gc.stream.synchronize()
    st = np.zeros((3, 2, 16384), dtype=np.uint64)
    L = _native.lib()
    L.bpgl_diag_stamps.argtypes = [ctypes.c_void_p]
    assert L.bpgl_diag_stamps(st.ctypes.data_as(ctypes.c_void_p)) == 0
    out = {"m": m, "n": n, "blocks": nb, "geometry": geo}
    for k, name in enumerate(("colpass", "rowpass")):
        s = st[k, 0, :nb].astype(np.float64) / 100.0      # 100 MHz ticks -> us
        e = st[k, 1, :nb].astype(np.float64) / 100.0
        t0 = s.min()
        d = e - s
        out[name] = {
            "span_us": e.max() - t0,
            "start_spread_us": s.max() - t0,
            "end_first_us": e.min() - t0, "end_p50_us": float(np.median(e - t0)), "end_last_us": e.max() - t0,
            "block_us_p10_p50_p90": [float(np.percentile(d, q)) for q in (10, 50, 90)],
            "mean_block_over_span": float(d.mean() / (e.max() - t0)),
        }
        ids = np.arange(nb)
        xcd = ids % 8
        seg, chunk = ids % geo["nseg"], ids // geo["nseg"]
        out[name]["end_by_xcd_us"] = [float((e[xcd == x] - t0).mean()) for x in range(8)]
        out[name]["end_by_chunk_us"] = [float((e[chunk == c] - t0).mean()) for c in range(geo["nchunk"])][:32]
        out[name]["end_by_seg_mod16_us"] = [float((e[seg % 16 == q] - t0).mean()) for q in range(16)]
        out[name]["raw_end_us"] = [round(float(v - t0), 1) for v in e]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
