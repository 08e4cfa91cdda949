"""Solver drivers over the MI355X ``GPU_Calculation`` (the callers of the path).

Reference drivers (lasso.py:25-613) and what stands in for each here:

  ClassLasso      (lasso.py:173-292)  host elementwise + device GEMVs through
                  ``mat_tMulVec_DiffSize`` / ``matMulVec_DiffSize``: same loop,
                  our kernels underneath.
  ClassLassoR     (lasso.py:296-306)  ClassLasso with a fresh stdlib
                  ``random.shuffle`` of the block order every sweep.
  ClassLassoCB_v1 (lasso.py:310-353)  cuBLAS Dgemv variant -> ClassLasso (the
                  GEMVs are already ours); the leading cuBLAS handle ``h`` is
                  accepted and ignored.
  ClassLassoCB_v2 (lasso.py:357-613)  "pure GPU" loop -> ClassLassoDevice: every
                  step on the device, one hipGraph replay per iteration, no
                  host round trip until the end.
  ClassLassoCPU   (lasso.py:25-169)   not provided: the reference's Pool-based
                  CPU path stays the reference's (tests/ and bench.py time its
                  restatement in oracle/ as the CPU baseline).

Run-contract kept from the reference (lasso.py:70-169): ``run(ERR_BOUND=None,
err_iter=None, time_iter=None, SILENCE=False, DEBUG=False) -> t_elapsed``;
``ERR_BOUND`` active only when it is a float; ``err_iter`` / ``time_iter``
filled only when they are numpy arrays.  Differences, all deliberate:
  * the solution is returned: after ``run`` the driver's ``x`` is the (K, 1)
    iterate (the reference rebuilt a local and dropped it, lasso.py:167, :609);
  * when r2 == 0 the step is 0 instead of a stale one (lasso.py:133-136);
  * DEBUG prints the true objective (the reference's ``debug`` evaluates an x
    that is never updated, lasso.py:46, :89-90).
"""
import random
import time

import numpy as np

from .cpu_calculation import element_proj, error_crit, soft_thresholding


def cyclic_order(nblock, n_iter):
    """Block index per iteration for ascending order (lasso.py:40-41)."""
    return np.arange(n_iter, dtype=np.int64) % nblock


def shuffled_order(nblock, n_iter, rng=None):
    """Block order of ClassLassoR.index_get (lasso.py:303-306).

    One permutation array is shuffled in place at the start of every sweep, so
    with a seeded ``random.Random`` (or the seeded stdlib module) the sequence
    is the reference's.
    """
    rng = random if rng is None else rng
    perm = np.arange(nblock)
    out = np.empty(n_iter, dtype=np.int64)
    for t in range(n_iter):
        if t % nblock == 0:
            rng.shuffle(perm)
        out[t] = perm[t % nblock]
    return out


class _Driver:
    descript = "driver"

    def __init__(self, gpu_cal, d_ATA, A, b, mu, BLOCK, ITER_MAX):
        self.gpu_cal = gpu_cal
        self.d_ATA = np.asarray(d_ATA, dtype=np.float64)
        self.d_ATA_rec = [1.0 / self.d_ATA[k] for k in range(BLOCK)]
        self.A = A
        self.A_SHAPE = tuple(A.shape)
        self.b = np.asarray(b, dtype=np.float64).reshape(-1, 1)
        self.mu = float(mu)
        self.BLOCK = int(BLOCK)
        self.ITER_MAX = int(ITER_MAX)
        self.x = None

    def index_get(self, t):
        return t % self.BLOCK

    def rlt_display(self, SILENCE, t_elapsed, t):
        if not SILENCE:
            print(f"{self.descript:>20}, time used: {t_elapsed:.8f} s, "
                  f"with {t + 1:4d} loops, and block number: {self.BLOCK:2d}.")


class ClassLasso(_Driver):
    """Host loop of lasso.py:190-292 with the two GEMVs on the MI355X."""
    descript = "GPU ascend index"

    def _mtv(self, s13, m, s11):
        self.gpu_cal.mat_tMulVec_DiffSize(s13, m, s11)

    def _mv(self, s23, m, descent_D):
        self.gpu_cal.matMulVec_DiffSize(s23, m, descent_D)

    def run(self, ERR_BOUND=None, err_iter=None, time_iter=None, SILENCE=False, DEBUG=False):
        bounded = isinstance(ERR_BOUND, float)
        rec_err = isinstance(err_iter, np.ndarray)
        rec_time = isinstance(time_iter, np.ndarray)
        H, K = self.A_SHAPE
        W = K // self.BLOCK
        xb = np.zeros((self.BLOCK, W, 1))
        Ax = np.zeros((self.BLOCK, H, 1))
        g = np.zeros((W, 1))
        s23 = np.zeros((H, 1))
        below = 0
        t = 0
        start = time.time()
        if rec_time:
            time_iter[0] = 0
        for t in range(self.ITER_MAX):
            m = self.index_get(t)
            s11 = Ax.sum(axis=0) - self.b
            self._mtv(g, m, s11)
            Bx = self.d_ATA_rec[m] * soft_thresholding(self.d_ATA[m] * xb[m] - g, self.mu)
            D = Bx - xb[m]
            self._mv(s23, m, D)
            r1 = (s11.T @ s23).item() + self.mu * (np.abs(Bx).sum() - np.abs(xb[m]).sum())
            r2 = (s23.T @ s23).item()
            gamma = 0.0 if r2 == 0.0 else float(element_proj(-r1 / r2, 0.0, 1.0))
            err = error_crit(g, xb[m], self.mu) if (DEBUG or rec_err or bounded) else None
            if DEBUG:
                x_full = xb.reshape(-1, 1)
                obj = 0.5 * float(np.square(s11).sum()) + self.mu * float(np.abs(x_full).sum())
                print(f"Loop {t:4d} block {m:2d} updated, with Error {err:.8f}, "
                      f"optimum value {obj:4.6f}, Stepsize {gamma:.6f}")
            if rec_err:
                err_iter[t] = err
            if bounded:
                below += err < ERR_BOUND
                if m == self.BLOCK - 1:
                    if below == self.BLOCK:
                        break
                    below = 0
            xb[m] += gamma * D
            Ax[m] += gamma * s23
            if rec_time:
                time_iter[t + 1] = time.time() - start
        t_elapsed = time_iter[t] if rec_time else time.time() - start
        self.rlt_display(SILENCE, t_elapsed, t)
        self.x = xb.reshape(-1, 1).copy()
        self.iters = t + 1
        return t_elapsed


class ClassLassoR(ClassLasso):
    """ClassLasso with a per-sweep shuffled block order (lasso.py:296-306)."""
    descript = "GPU random index"

    def __init__(self, gpu_cal, d_ATA, A, b, mu, BLOCK, ITER_MAX):
        ClassLasso.__init__(self, gpu_cal, d_ATA, A, b, mu, BLOCK, ITER_MAX)
        self.idx_shuffle = np.arange(self.BLOCK)

    def index_get(self, t):
        if t % self.BLOCK == 0:
            random.shuffle(self.idx_shuffle)
        return self.idx_shuffle[t % self.BLOCK]


class ClassLassoDevice(_Driver):
    """Every step of every iteration on the device (stands in for lasso.py:357-613).

    The block order is drawn on the host up front with ``index_get`` (so a
    subclass overriding it, e.g. a shuffled order, is honoured) and uploaded
    once; the device reads its entry per iteration.
    """
    descript = "MI355X device loop"

    def __init__(self, gpu_cal, d_ATA, A, b, mu, BLOCK, ITER_MAX, use_graph=True):
        _Driver.__init__(self, gpu_cal, d_ATA, A, b, mu, BLOCK, ITER_MAX)
        self.use_graph = use_graph

    def _order(self):
        if type(self).index_get is _Driver.index_get:
            return None
        return np.array([self.index_get(t) for t in range(self.ITER_MAX)], dtype=np.int32)

    def run(self, ERR_BOUND=None, err_iter=None, time_iter=None, SILENCE=False, DEBUG=False):
        bounded = isinstance(ERR_BOUND, float)
        rec_err = isinstance(err_iter, np.ndarray)
        rec_time = isinstance(time_iter, np.ndarray)
        gc = self.gpu_cal
        record = rec_err or rec_time or DEBUG
        start = time.time()
        gc.solver_reset(self.b, self.mu, order=self._order(), err_bound=ERR_BOUND if bounded else None,
                        record_len=self.ITER_MAX if record else 0, use_graph=self.use_graph and not DEBUG)
        if DEBUG:
            import torch
            res = gc._ctx_residual()
            for t in range(self.ITER_MAX):
                gc.solver_step(1)
                st = gc.solver_status()
                xs = gc.solver_x_device()
                obj = 0.5 * float(torch.square(res).sum()) + self.mu * float(xs.abs().sum())
                print(f"Loop {t:4d} updated, with Error {st['err']:.8f}, "
                      f"optimum value {obj:4.6f}, Stepsize {st['gamma']:.6f}")
                if st["stopped"]:
                    break
        else:
            gc.solver_step(self.ITER_MAX)
        # solver_status is collective for RCCL row shards (a pending one-pass recovery enqueues
        # all-reduces): every rank runs this driver; the reads after it need no communication
        st = gc.solver_status()
        wall = time.time() - start
        t = st["t_last"]
        if record:
            e, ti = gc.solver_records(complete=False)
            if rec_err:
                err_iter[:] = e[:len(err_iter)]
            if rec_time:
                time_iter[:] = ti[:len(time_iter)]
        t_elapsed = time_iter[t] if rec_time else wall
        self.rlt_display(SILENCE, t_elapsed, t)
        self.x = gc.solver_x(complete=False).reshape(-1, 1)
        self.iters = st["iters"]
        self.stopped = st["stopped"]
        return t_elapsed


class ClassLassoCB_v1(ClassLasso):
    """Name-compatible stand-in for lasso.py:310-353 (cuBLAS handle ignored)."""
    descript = "Cublas CPU combined"

    def __init__(self, h, gpu_cal, d_ATA, A, b, mu, BLOCK, ITER_MAX):
        ClassLasso.__init__(self, gpu_cal, d_ATA, A, b, mu, BLOCK, ITER_MAX)
        self.h = h


class ClassLassoCB_v2(ClassLassoDevice):
    """Name-compatible stand-in for lasso.py:357-613 (cuBLAS handle ignored)."""
    descript = "Pure Cublas"

    def __init__(self, h, gpu_cal, d_ATA, A, b, mu, BLOCK, ITER_MAX):
        ClassLassoDevice.__init__(self, gpu_cal, d_ATA, A, b, mu, BLOCK, ITER_MAX)
        self.h = h
