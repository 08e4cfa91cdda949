#!/usr/bin/env python3
"""Per-block timeline of k_onepass (diagnostic build, tools/stamp_diag.sh -> build_diag/libbpgl_stamp.so).

Usage: python tools/onepass_stamps.py [LIB] [M N [--rows]]
Stamps (s_memrealtime, 100 MHz) per block: 0 start (after the LDS init), 2 first row's phase 1 done
(wave 0), 3 last row's phase 1 done (wave 0), 1 row loop done (all waves), 4 kernel end (stores
drained).  Prints, per launch, the medians over blocks of: first row (2 - 0), steady row step
((3 - 2) / (rows - 1)), drain (1 - 3), epilogue (4 - 1), and the launch span, the start spread and
the end spread.  --rows: the row-shard form through a one-rank RCCL communicator.
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    lib = args[0] if args else os.path.join(ROOT, "build_diag", "libbpgl_stamp.so")
    m = int(args[1]) if len(args) > 1 else 8192
    n = int(args[2]) if len(args) > 2 else 65536
    rows = "--rows" in sys.argv
    import numpy as np
    import torch
    from convex_optimization_amd import _native
    _native.LIB_PATH = os.path.abspath(lib)
    from convex_optimization_amd.parameters import device_instance
    torch.cuda.set_device(0)
    comm = None
    if rows:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29611")
        dist.init_process_group("gloo", rank=0, world_size=1)
        from convex_optimization_amd.distributed import RankComm
        comm = RankComm(0, 1)
    gc, b, mu, _ = device_instance(m, n, 0.4, 1, TYPE="float", seed=1, device=0, comm=comm,
                                   row_range=(0, m) if rows else None)
    L = _native.lib()
    L.bpgl_diag_stamps.argtypes = [ctypes.c_void_p]
    gc.solver_reset(b, mu, use_graph=False)
    gc.solver_step(20)
    gc.stream.synchronize()
    R = gc.solver_stat("onepass_grid")
    out = {"m": m, "n": n, "rows_mode": rows, "grid": R, "launches": []}
    for it in range(8):
        gc.solver_step(1)
        gc.stream.synchronize()
        st = np.zeros((3, 5, 16384), dtype=np.uint64)
        assert L.bpgl_diag_stamps(st.ctypes.data_as(ctypes.c_void_p)) == 0
        nz = int(np.count_nonzero(st[2, 0]))
        t = st[2, :, :nz].astype(np.float64) / 100.0   # us
        t0 = t[0].min()
        t = t - t0
        med = lambda v: round(float(np.median(v)), 2)
        rec = {"iter": it, "blocks": nz, "span_us": round(float(t[4].max()), 2),
               "start_spread_us": round(float(t[0].max()), 2),
               "first_row_us": med(t[2] - t[0]), "rows_phase1_us": med(t[3] - t[2]),
               "drain_us": med(t[1] - t[3]), "epilogue_us": med(t[4] - t[1]),
               "end_spread_us": round(float(t[4].max() - t[4].min()), 2),
               "loop_end_by_xcd_us": [round(float(t[1][np.arange(nz) % 8 == q].mean()), 1) for q in range(8)]}
        out["launches"].append(rec)
        print(json.dumps(rec), flush=True)
    return out


if __name__ == "__main__":
    main()
