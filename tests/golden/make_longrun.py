"""Offline generator of the long-horizon parity fixtures tests/golden/longrun_*.npz
(TEST INFRASTRUCTURE; run in the build container, not on the GPU box).

For each BASELINE shape the hash instance of tests/hash_instance.py (bit-identical under numpy
and torch) is built here, mu = 0.1 ||A^T b||_inf is taken with the C oracle's A^T r, and the C
oracle (oracle/bpgl_oracle.c, the restatement of lasso.py:102-157 pinned to the reference's own
ClassLassoCPU fixtures) runs ITER_MAX = 1000 iterations -- the reference's timing protocol,
cpu_vs_gpu.py:66 -- from x = 0.  The fixture keeps x (fp32: 6e-8 relative, far inside the 1e-5
bound), err_iter, mu, a SHA-256 of b and A at 4096 sample points, so the GPU test
(tests/test_longrun.py) can check it rebuilt the same instance before comparing.

usage: python tests/golden/make_longrun.py [configs1 configs3 configs2 configs4] [--iters 1000] [--threads 8]
"""
import argparse
import hashlib
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import hash_instance as H  # noqa: E402
from oracle import oracle  # noqa: E402

SHAPES = {"configs1": (8192, 65536), "configs3": (1048576, 4096), "configs2": (8192, 524288),
          "configs4": (8192, 65536)}
PANEL_K, PANEL_RHS = 128, (0, 42, 85, 127)   # configs[4]: k right-hand sides; the ones the oracle follows


def panel_case(a):
    """configs[4]: bf16 A (exact hash values), k = 128 right-hand sides; the oracle runs the
    single-RHS iteration on RHS 0, 42, 85 and 127 (the panel path solves each RHS with it,
    lasso.py:102-157).  RHS already in an existing fixture with the same iteration count are kept
    (round 3 computed 0 and 127; round 4 added 42 and 85)."""
    m, n = SHAPES["configs4"]
    t0 = time.time()
    A = H.np_A_bf16(m, n)
    path = os.path.join(HERE, "longrun_configs4.npz")
    old = dict(np.load(path)) if os.path.exists(path) else {}
    if old and int(old["iters"]) != a.iters:
        old = {}
    out = dict(m=m, n=n, k=PANEL_K, iters=a.iters, rhs=np.array(PANEL_RHS), threads=a.threads)
    rows, cols = H.sample_points(m, n)
    out.update(A_rows=rows, A_cols=cols, A_samples=A[rows, cols])
    for r in PANEL_RHS:
        if f"x_{r}" in old:
            for key in ("mu", "x", "x_norm", "objective", "err_iter", "b_sha256"):
                out[f"{key}_{r}"] = old[f"{key}_{r}"]
            print(f"configs4 RHS {r}: kept from the existing fixture", flush=True)
            continue
        b = H.np_b_rhs(A, r)
        mu = 0.1 * float(np.abs(oracle.mtv(A, 0, n, b, nthreads=a.threads)).max())
        t1 = time.time()
        ref = oracle.run(A, b, mu, 1, a.iters, nthreads=a.threads)
        res = A.astype(np.float64) @ ref["x"] - b
        out[f"mu_{r}"] = mu
        out[f"x_{r}"] = ref["x"].astype(np.float32)
        out[f"x_norm_{r}"] = np.linalg.norm(ref["x"])
        out[f"objective_{r}"] = 0.5 * res @ res + mu * np.abs(ref["x"]).sum()
        out[f"err_iter_{r}"] = ref["err_iter"]
        out[f"b_sha256_{r}"] = hashlib.sha256(b.tobytes()).hexdigest()
        print(f"configs4 RHS {r}: mu {mu:.17g}, {a.iters} oracle iterations in {time.time() - t1:.1f} s", flush=True)
    np.savez_compressed(path, **out)
    print(f"configs4: {time.time() - t0:.1f} s -> {path}, {os.path.getsize(path)} B", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("which", nargs="*", default=list(SHAPES))   # configs4: the bf16 k-RHS panel case
    ap.add_argument("--iters", type=int, default=1000)
    ap.add_argument("--threads", type=int, default=os.cpu_count())
    a = ap.parse_args()
    for name in a.which:
        if name == "configs4":
            panel_case(a)
            continue
        m, n = SHAPES[name]
        t0 = time.time()
        A = H.np_A(m, n)
        b = H.np_b(A)
        g = oracle.mtv(A, 0, n, b, nthreads=a.threads)
        mu = 0.1 * float(np.abs(g).max())
        t1 = time.time()
        print(f"{name}: instance {m}x{n} built in {t1 - t0:.1f} s, mu {mu:.17g}", flush=True)
        ref = oracle.run(A, b, mu, 1, a.iters, nthreads=a.threads)
        t2 = time.time()
        rows, cols = H.sample_points(m, n)
        out = dict(m=m, n=n, iters=a.iters, mu=mu, x=ref["x"].astype(np.float32), x_norm=np.linalg.norm(ref["x"]),
                   err_iter=ref["err_iter"], t_last=ref["t_last"], b_sha256=hashlib.sha256(b.tobytes()).hexdigest(),
                   A_rows=rows, A_cols=cols, A_samples=A[rows, cols], oracle_s=t2 - t1, threads=a.threads)
        path = os.path.join(HERE, f"longrun_{name}.npz")
        np.savez_compressed(path, **out)
        print(f"{name}: {a.iters} oracle iterations in {t2 - t1:.1f} s ({a.threads} threads) -> {path}, "
              f"{os.path.getsize(path)} B, err_iter[-1] {ref['err_iter'][-1]:.3e}", flush=True)
        del A, b


if __name__ == "__main__":
    main()
