#!/usr/bin/env python3
"""lo8 accuracy at the full configs[4] shape (8192 x 65536 bf16 A, k = 128), GPU only.

Runs ITERS (default 1000) iterations of the panel solver on the long-run hash instance of
tests/golden/longrun_configs4.npz (the fixture holds the C oracle's x and objective for RHS 0 and
127 after 1000 iterations) for each setting "lo8:r_refresh" given on the command line (default:
the bf16 form and the e4m3 forms), and reports per setting: x and objective error of RHS 0 / 127
against the oracle fixture, and over all 128 RHS the x / objective difference against the bf16
hi + lo run (lo8 = 0), plus the drift |R - (A X - B)| of the incrementally updated residual at the
end of the run.  One JSON line per setting.

Usage (GPU box, repo root): python3 tools/panel_lo8_accuracy.py [ITERS] [lo8:r_refresh[:d_split[:carry_g[:g_refresh]]] ...]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    args = sys.argv[1:]
    it = int(args.pop(0)) if args and ":" not in args[0] else 1000
    settings = [tuple(int(v) for v in a.split(":")) for a in args] or [(0, 0), (1, 0), (2, 128), (3, 128)]
    # lo8:r_refresh[:d_split[:carry_g[:g_refresh]]]
    settings = [tuple(t) + (2, 0, 64)[len(t) - 2:] if len(t) < 5 else t for t in settings]
    import numpy as np
    import torch
    import hash_instance as H
    from convex_optimization_amd.panel import PanelLasso
    fx = dict(np.load(os.path.join(ROOT, "tests", "golden", "longrun_configs4.npz")))
    m, n, k = int(fx["m"]), int(fx["n"]), int(fx["k"])
    A = H.torch_A_bf16(m, n, "cuda:0")
    B = H.torch_B(A, k)
    A64 = A.double()
    mu = (0.1 * (A64.t() @ B).abs().amax(dim=0)).cpu().numpy()
    for r in fx["rhs"]:
        mu[int(r)] = float(fx[f"mu_{r}"])
    pl = PanelLasso(A, 1, nrhs=k, device=0)
    muv = torch.from_numpy(mu).cuda()

    def objectives(X):
        Xd = torch.from_numpy(X).cuda()
        R = A64 @ Xd - B
        return (0.5 * (R * R).sum(dim=0) + muv * Xd.abs().sum(dim=0)).cpu().numpy(), R
    base = None
    for lo8, rr, ds, cg, gp in settings:
        pl.set_tuning("lo8", lo8)
        pl.set_tuning("r_refresh", rr)
        pl.set_tuning("d_split", ds)
        pl.set_tuning("carry_g", cg)
        pl.set_tuning("g_refresh", gp)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        res = pl.run(B, mu, it)
        el = time.perf_counter() - t0
        X = res["x"]
        f, Rex = objectives(X)
        torch.cuda.synchronize()
        Rdev = pl.residual_device().t()
        drift = float((Rdev - Rex).abs().max() / Rex.abs().max())
        row = {"lo8": lo8, "r_refresh": rr, "d_split": ds, "carry_g": cg, "g_refresh": gp, "iters": it, "seconds_incl_setup": el,
               "refreshes": pl.stat("refreshes"), "residual_drift_rel_max": drift}
        for r in fx["rhs"]:
            r = int(r)
            row[f"x_rel_vs_oracle_{r}"] = float(np.linalg.norm(X[:, r] - fx[f"x_{r}"]) / np.linalg.norm(fx[f"x_{r}"]))
            row[f"objective_rel_vs_oracle_{r}"] = float(abs(f[r] - fx[f"objective_{r}"]) / fx[f"objective_{r}"])
        if base is None and lo8 == 0 and cg == 0:
            base = (X, f)
        elif base is not None:
            dx = np.linalg.norm(X - base[0], axis=0) / np.maximum(np.linalg.norm(base[0], axis=0), 1e-300)
            df = np.abs(f - base[1]) / base[1]
            row.update({"x_rel_vs_bf16_worst": float(dx.max()), "x_rel_vs_bf16_median": float(np.median(dx)),
                        "objective_rel_vs_bf16_worst": float(df.max()),
                        "objective_dev_minus_bf16_worst": float(((f - base[1]) / base[1]).max())})
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
