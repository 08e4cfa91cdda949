#!/usr/bin/env python3
"""Panel path (configs[4]: 8192 x 65536 bf16 A, k = 128 RHS) against the fp64 oracle on the same
bf16-rounded A over a longer horizon: ITERS iterations (default 400), 8 RHS spread over the
panel.  Prints one JSON line (heartbeat on stderr while the oracle runs).

Usage (GPU box, repo root): python3 tools/panel_longrun.py [ITERS] > gpurun_out/panel_longrun.json
"""
import json
import os
import sys
import threading

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    it = int(sys.argv[1]) if len(sys.argv) > 1 else 400
    import numpy as np
    import torch
    from convex_optimization_amd.panel import PanelLasso
    from oracle import oracle
    oracle.build()
    m, n, k = 8192, 65536, 128
    g = torch.Generator(device="cuda").manual_seed(7)
    A = torch.randn(m, n, device="cuda", generator=g)
    A /= A.norm(dim=1, keepdim=True)
    pl = PanelLasso(A, 1, nrhs=k, device=0)
    del A
    A64 = pl.A_bf16.double()
    Xt = torch.randn(n, k, device="cuda", generator=g, dtype=torch.float64) * \
        (torch.rand(n, k, device="cuda", generator=g) < 0.4)
    B = A64 @ Xt + 0.01 * torch.randn(m, k, device="cuda", generator=g, dtype=torch.float64)
    mu = (0.1 * (A64.t() @ B).abs().amax(dim=0)).cpu().numpy()
    X = pl.run(B, mu, it)["x"]
    Ah, Bh = A64.cpu().numpy(), B.cpu().numpy()
    del A64
    stop = threading.Event()

    def beat():
        while not stop.wait(30):
            print("# oracle running", file=sys.stderr, flush=True)
    threading.Thread(target=beat, daemon=True).start()

    def obj(j, x):
        r = Ah @ x - Bh[:, j]
        return 0.5 * float(r @ r) + float(mu[j]) * float(np.abs(x).sum())
    rows = []
    for j in (0, 17, 38, 55, 64, 91, 110, 127):
        ref = oracle.run(Ah, Bh[:, j], float(mu[j]), 1, it, nthreads=min(16, os.cpu_count() or 1))["x"]
        f_dev, f_ref = obj(j, X[:, j]), obj(j, ref)
        rows.append({"rhs": j, "x_rel_l2": float(np.linalg.norm(X[:, j] - ref) / np.linalg.norm(ref)),
                     "objective_rel": abs(f_dev - f_ref) / f_ref, "objective_dev_minus_ref_rel": (f_dev - f_ref) / f_ref})
    stop.set()
    print(json.dumps({"workload": "configs[4] 8192x65536 bf16 A, k=128, seed 7 (default d_split 2)", "iters": it,
                      "rhs": rows, "worst_x_rel_l2": max(r["x_rel_l2"] for r in rows),
                      "worst_objective_rel": max(r["objective_rel"] for r in rows),
                      "stated_tolerance": "x 1e-2 relative l2, objective 1e-5 relative"}), flush=True)


if __name__ == "__main__":
    main()
