"""ORACLE-SIDE CPU BASELINE -- TEST / BENCH INFRASTRUCTURE ONLY.

The reference's own CPU path, restated: ``ClassLassoCPU.run`` (lasso.py:70-169) with its
``multiprocessing.Pool`` of P worker processes, each iteration mapping ``fun_s12`` over the
P column shards of the active block (lasso.py:107-111), the host shrink (:114-119), mapping
``fun_s22`` over the shards and summing (:121-126), the line search (:129-136) and the
update (:153-155).  The per-shard functions are the drop-in ``cpu_calculation`` module of
this repository (convex_optimization_amd/cpu_calculation.py), i.e. the CPU half of the call
surface the reference drivers import.

Used only by bench.py's ``cpu_baseline`` leg, at BASELINE configs[0] (m=512, n=2048, fp64,
200 iterations): SURVEY.md section 8d asks for the Pool variant at that size only, because
at configs[1] each iteration pickles the 2 GiB block to the workers (~29 s per iteration).

The pool is created with the ``fork`` start method and must be used before the calling
process initialises the GPU (bench.py runs it first).
"""
import multiprocessing as mp
import time
from itertools import product

import numpy as np

from convex_optimization_amd.cpu_calculation import (A_bp_get, element_proj, fun_dd_p, fun_diag_ATA, fun_s12,
                                                     fun_s22, soft_thresholding)


def instance(m, n, seed=20190325, den=0.4):
    """parameters.py:17-33's recipe with a fixed seed (row-normalised N(0,1) A, sparse x_true,
    b = A x_true + N(0, 1e-4), mu = 0.1 ||A^T b||_inf)."""
    rs = np.random.RandomState(seed)
    A = rs.randn(m, n)
    A /= np.linalg.norm(A, axis=1, keepdims=True)
    x_true = np.where(rs.rand(n) < den, rs.randn(n), 0.0)
    b = (A @ x_true + rs.normal(0.0, 1e-2, m)).reshape(m, 1)
    mu = 0.1 * float(np.max(np.abs(A.T @ b)))
    return A, b, mu


def largest_divisor_at_most(n, p):
    p = max(1, min(int(p), int(n)))
    while n % p:
        p -= 1
    return p


def run_pool(A, b, mu, BLOCK, P, iters):
    """lasso.py:70-157 with a Pool of P processes (no ERR_BOUND, no records); returns
    (x, seconds for the `iters` iterations, pool start-up seconds)."""
    m, n = A.shape
    A_bp = A_bp_get(A, BLOCK, P)                       # lasso.py (cpu_vs_gpu.py builds it the same way)
    d_ATA = fun_diag_ATA(A_bp)
    d_rec = [1.0 / d_ATA[i] for i in range(BLOCK)]
    x_block = np.zeros((BLOCK, n // BLOCK, 1))
    Ax = np.zeros((BLOCK, m, 1))
    t0 = time.perf_counter()
    pool = mp.get_context("fork").Pool(processes=P)
    try:
        pool.starmap(fun_s12, product(A_bp[0], (np.zeros((m, 1)),)))   # workers up before the clock
        t1 = time.perf_counter()
        for t in range(iters):
            k = t % BLOCK
            s11 = np.sum(Ax, axis=0) - b                                  # lasso.py:105
            s13 = np.vstack(pool.starmap(fun_s12, product(A_bp[k], (s11,))))   # :107-111
            rx = d_ATA[k] * x_block[k] - s13                              # :114
            Bx = d_rec[k] * soft_thresholding(rx, mu)                     # :115-117
            D = Bx - x_block[k]                                           # :119
            s23 = np.sum(pool.starmap(fun_s22, zip(A_bp[k], fun_dd_p(P, D))), axis=0)   # :121-126
            r1 = (s11.T @ s23).item() + mu * (np.abs(Bx).sum() - np.abs(x_block[k]).sum())   # :129-131
            r2 = (s23.T @ s23).item()                                     # :132
            gamma = 0.0 if r2 == 0.0 else float(element_proj(-r1 / r2, 0, 1))   # :133-136
            x_block[k] += gamma * D                                       # :153
            Ax[k] += gamma * s23                                          # :155
        el = time.perf_counter() - t1
    finally:
        # close + join, not terminate: the workers exit on their own once the task queue drains,
        # so no SIGTERM stack traces land in the logs of a profiled bench run
        pool.close()
        pool.join()
    return x_block.reshape(-1), el, t1 - t0


def pool_baseline(cores, m=512, n=2048, iters=200, BLOCK=1):
    """configs[0] timed with the reference's Pool structure, P = the largest divisor of n/BLOCK
    not above `cores`."""
    A, b, mu = instance(m, n)
    P = largest_divisor_at_most(n // BLOCK, cores)
    x, el, start = run_pool(A, b, mu, BLOCK, P, iters)
    return {"value": iters / el, "unit": "iters/s", "processes": P, "iters": iters,
            "pool_start_s": start,
            "sample": f"configs[0]: m={m} n={n} fp64, BLOCK={BLOCK}, {iters} iterations of the reference's "
                      f"ClassLassoCPU loop (lasso.py:101-157) restated with a multiprocessing Pool of {P} "
                      f"processes over this repository's drop-in cpu_calculation (oracle/pool_baseline.py)"}
