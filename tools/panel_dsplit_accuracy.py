"""Accuracy of the panel solver's two direction encodings at the full configs[4] shape.

Runs PanelLasso (m=8192, n=65536, k=128, bf16 A) for ITERS iterations with d_split = 2 (hi + lo
direction) and d_split = 1 (bf16 direction), evaluates every RHS's objective in fp64 on the GPU,
and runs the fp64 C oracle (oracle/, test infrastructure) on a few RHS of the same bf16 A.
Usage (GPU box): python tools/panel_dsplit_accuracy.py [ITERS] > gpurun_out/panel_dsplit.json
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from convex_optimization_amd.panel import PanelLasso  # noqa: E402
from oracle import oracle  # noqa: E402


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    m, n, k = 8192, 65536, 128
    torch.cuda.set_device(0)
    g = torch.Generator(device="cuda").manual_seed(20190325)
    A = torch.randn(m, n, device="cuda", generator=g)
    A /= A.norm(dim=1, keepdim=True)
    Xt = torch.randn(n, k, device="cuda", generator=g) * (torch.rand(n, k, device="cuda", generator=g) < 0.4)
    pl = PanelLasso(A, 1, nrhs=k, device=0)
    del A
    A64 = pl.A_bf16.double()
    B = (A64 @ Xt.double() + 0.01 * torch.randn(m, k, device="cuda", generator=g, dtype=torch.float64))
    mu = (0.1 * (A64.t() @ B).abs().amax(dim=0)).cpu().numpy()

    def objective(X):   # X (n, k) fp64 on the GPU
        R = A64 @ X - B
        return (0.5 * (R * R).sum(dim=0) + torch.from_numpy(mu).cuda() * X.abs().sum(dim=0)).cpu().numpy()

    out = {"m": m, "n": n, "k": k, "iters": iters}
    xs, fs = {}, {}
    for ds in (2, 1):
        pl.set_tuning("d_split", ds)
        t0 = time.perf_counter()
        res = pl.run(B, mu, iters)
        out[f"run_s_d{ds}"] = time.perf_counter() - t0
        xs[ds] = torch.from_numpy(res["x"]).cuda()
        fs[ds] = objective(xs[ds])
    f0 = objective(torch.zeros(n, k, dtype=torch.float64, device="cuda"))
    out["objective_rel_diff_d1_vs_d2_max"] = float(np.max(np.abs(fs[1] - fs[2]) / fs[2]))
    out["objective_decrease_d2_median"] = float(np.median((f0 - fs[2]) / f0))
    out["x_rel_l2_d1_vs_d2_max"] = float(
        ((xs[1] - xs[2]).norm(dim=0) / xs[2].norm(dim=0)).max().item())
    # the fp64 oracle on a few RHS of the same bf16 A
    Ah = A64.cpu().numpy()
    Bh = B.cpu().numpy()
    rows = []
    for j in (0, 64, 127):
        t0 = time.perf_counter()
        xo = oracle.run(Ah, Bh[:, j], float(mu[j]), 1, iters, nthreads=16)["x"]
        fo = float(objective(torch.from_numpy(np.ascontiguousarray(
            np.repeat(xo[:, None], k, axis=1))).cuda())[j])
        row = {"rhs": j, "oracle_s": time.perf_counter() - t0, "f_oracle": fo}
        for ds in (2, 1):
            xd = xs[ds][:, j].cpu().numpy()
            row[f"x_rel_l2_d{ds}"] = float(np.linalg.norm(xd - xo) / np.linalg.norm(xo))
            row[f"f_rel_d{ds}"] = float(abs(fs[ds][j] - fo) / fo)
        rows.append(row)
    out["vs_oracle"] = rows
    print(json.dumps(out))


if __name__ == "__main__":
    main()
