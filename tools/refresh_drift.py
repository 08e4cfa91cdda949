#!/usr/bin/env python3
"""Drift of the one-pass gradient recurrence g += gamma A^T (A D) between exact refreshes.

At configs[1] (8192 x 65536 fp32), runs ITERS iterations with onepass_refresh in {0, 64, 256,
1024} and the two-pass iteration (exact g every iteration), and reports the relative l2
difference of x from the two-pass run and the objective.  Usage: python tools/refresh_drift.py [ITERS]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    from convex_optimization_amd.parameters import device_instance
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    torch.cuda.set_device(0)
    gc, b, mu, _ = device_instance(8192, 65536, 0.4, 1, TYPE="float", seed=5, device=0)
    A = gc._A_dev

    def objective(x):
        xt = torch.from_numpy(x).to(A.device)
        r = (A.double() @ xt) - b
        return 0.5 * float(r @ r) + mu * float(xt.abs().sum())

    gc.set_tuning("onepass", 0)
    ref = gc.run(b, mu, iters)
    f_ref = objective(ref["x"])
    print(json.dumps({"mode": "two-pass", "iters": iters, "objective": f_ref}))
    gc.set_tuning("onepass", 1)
    for period in (0, 1024, 256, 64):
        gc.set_tuning("onepass_refresh", period)
        out = gc.run(b, mu, iters)
        rel = float(np.linalg.norm(out["x"] - ref["x"]) / np.linalg.norm(ref["x"]))
        print(json.dumps({"mode": "one-pass", "refresh": period, "iters": iters, "x_rel_l2_vs_two_pass": rel,
                          "objective_rel_diff": (objective(out["x"]) - f_ref) / abs(f_ref)}))


if __name__ == "__main__":
    main()
