"""Offline generator of the full-size Gaussian-recipe parity fixtures tests/golden/gauss_configs3.npz
and gauss_configs2.npz (TEST INFRASTRUCTURE; run in the build container, not on the GPU box).

configs[3] (1048576 x 4096 fp32, 2^32 elements; seed 41) or configs[2] (8192 x 524288 fp32, 2^32
elements; seed 43) on the reference's instance recipe
(parameters.py:17-33: A ~ N(0, 1) with unit-norm rows, x_true density 0.4, e ~ N(0, 1e-4)) as
oracle/gauss_instance.c generates it -- bit-identical here and on the GPU box, which rebuilds it
with the same library (the N(0, 1) draws are the Irwin-Hall approximant; see that file).  The C
oracle (oracle/bpgl_oracle.c, the restatement of lasso.py:102-157 pinned to the reference's own
ClassLassoCPU fixtures) runs ITERS iterations from x = 0 -- 300 by default, past the product
path's exact-gradient refresh at 256.  The fixture keeps x, err_iter, mu, the objective, a
SHA-256 of b and A at 4096 sample points, so the GPU test (tests/test_fullsize.py) can prove it
rebuilt the same instance before comparing.

usage: python tests/golden/make_gauss.py [--config 3|2] [--iters 300] [--threads 8] [--seed S]
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

SHAPES = {3: (1048576, 4096, 41), 2: (8192, 524288, 43)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=3, choices=sorted(SHAPES))
    ap.add_argument("--iters", type=int, default=300)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--seed", type=int, default=None)
    a = ap.parse_args()
    M, N, seed = SHAPES[a.config]
    a.seed = seed if a.seed is None else a.seed
    oracle.build()
    t0 = time.time()
    A, b, mu, xt = oracle.gauss_instance(a.seed, M, N, 0.4, nthreads=a.threads)
    print(f"instance {M}x{N} seed {a.seed}: {time.time() - t0:.1f} s, mu {mu:.6g}", flush=True)
    t1 = time.time()
    ref = oracle.run(A, b, mu, 1, a.iters, nthreads=a.threads)
    print(f"oracle {a.iters} iterations: {time.time() - t1:.1f} s", flush=True)
    x = ref["x"]
    r = oracle.mv(A, 0, N, x, nthreads=a.threads) - b
    objective = 0.5 * float(r @ r) + mu * float(np.abs(x).sum())
    rows, cols = H.sample_points(M, N)
    out = dict(m=M, n=N, seed=a.seed, den=0.4, iters=a.iters, threads=a.threads, mu=mu, x=x,
               err_iter=ref["err_iter"], objective=objective,
               b_sha256=np.frombuffer(hashlib.sha256(b.tobytes()).digest(), dtype=np.uint8),
               A_rows=rows, A_cols=cols, A_samples=A[rows, cols])
    path = os.path.join(HERE, f"gauss_configs{a.config}.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {path}: |x|_0 {int((x != 0).sum())}, objective {objective:.12g}, "
          f"err_iter[-1] {ref['err_iter'][-1]:.3e}", flush=True)


if __name__ == "__main__":
    main()
