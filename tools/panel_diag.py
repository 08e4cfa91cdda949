#!/usr/bin/env python3
"""Time the panel passes with a given libbpgl.so (normal or a diagnostic build).

Usage: python tools/panel_diag.py LIB K [interleave]   -> one JSON line of per-kernel ms
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    lib, k = sys.argv[1], int(sys.argv[2])
    ilv = int(sys.argv[3]) if len(sys.argv) > 3 else 1   # -1: the library's per-pass defaults
    import torch
    from convex_optimization_amd import _native
    _native.LIB_PATH = os.path.abspath(lib)
    from convex_optimization_amd.panel import PanelLasso
    m, n = 8192, 65536
    g = torch.Generator(device="cuda").manual_seed(1)
    A = torch.randn(m, n, device="cuda", generator=g)
    pl = PanelLasso(A, 1, nrhs=k, device=0)
    del A
    if ilv >= 0:
        pl.set_tuning("interleave", ilv)
    B = torch.randn(m, k, device="cuda", generator=g, dtype=torch.float64)
    pl.solver_reset(B, 0.1, use_graph=False)
    warm = int(os.environ.get("PANEL_DIAG_WARMUP", "0"))   # untimed iterations first (clock ramp)
    if warm:
        pl.solver_step(warm)
        pl.stream.synchronize()
    pl.set_kernel_timing(True)
    pl.solver_step(30)
    pl.stream.synchronize()
    kms, ns = pl.kernel_times()
    print(json.dumps({"lib": os.path.basename(lib), "k": k, "interleave": ilv,
                      "us": {a: round(b * 1e3, 1) for a, b in kms.items()}}))


if __name__ == "__main__":
    main()
