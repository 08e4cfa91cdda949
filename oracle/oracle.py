"""ORACLE -- TEST INFRASTRUCTURE ONLY.

ctypes front end of ``oracle/liboracle.so`` (the C restatement in
``oracle/bpgl_oracle.c``) plus a small numpy restatement used to cross-check
it.  Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg import this module; the product package
``convex_optimization_amd`` never does.

Parity pinning: both restatements are checked against golden vectors that the
reference's own ``ClassLassoCPU`` (lasso.py:25-169) produced in the build
container (``tests/golden/make_golden.py``, fixtures ``tests/golden/*.npz``).
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None

_p = ctypes.c_void_p
_i64 = ctypes.c_int64
_i32 = ctypes.c_int32
_f64 = ctypes.c_double


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.oracle_diag_ata.argtypes = [ctypes.c_int, _p, _i64, _i64, _i64, _i32, _p, ctypes.c_int]
        L.oracle_mtv.argtypes = [ctypes.c_int, _p, _i64, _i64, _i64, _i64, _p, _p, ctypes.c_int]
        L.oracle_mv.argtypes = [ctypes.c_int, _p, _i64, _i64, _i64, _i64, _i32, _p, _p, ctypes.c_int]
        L.oracle_run.argtypes = [ctypes.c_int, _p, _i64, _i64, _i64, _i32, _i32, _p, _f64, _i64,
                                 _p, _f64, _p, _p, _p, _p, ctypes.c_int]
        L.oracle_gauss_instance.argtypes = [ctypes.c_uint64, _i64, _i64, _f64, _p, _p, _p, ctypes.c_int]
        L.oracle_gauss_rows.argtypes = [ctypes.c_uint64, _i64, _i64, _i64, _p]
        for f in (L.oracle_diag_ata, L.oracle_mtv, L.oracle_mv, L.oracle_run, L.oracle_gauss_instance,
                  L.oracle_gauss_rows):
            f.restype = ctypes.c_int
        _lib = L
    return _lib


def _a(A):
    if A.dtype not in (np.float32, np.float64):
        raise TypeError("A must be float32 or float64")
    if not A.flags.c_contiguous:
        A = np.ascontiguousarray(A)
    return A, int(A.dtype == np.float64)


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def diag_ata(A, nblock, nthreads=0):
    """(nblock, w, 1) fp64, as cpu_calculation.fun_diag_ATA (cpu_calculation.py:35-42)."""
    A, f64 = _a(A)
    m, n = A.shape
    out = np.zeros(n)
    rc = lib().oracle_diag_ata(f64, _ptr(A), n, m, n, nblock, _ptr(out), nthreads)
    assert rc == 0, rc
    return out.reshape(nblock, n // nblock, 1)


def mtv(A, col0, w, r, nthreads=0):
    """A[:, col0:col0+w]^T r in fp64 (cpu_calculation.py:30-31)."""
    A, f64 = _a(A)
    r = np.ascontiguousarray(r, dtype=np.float64).reshape(-1)
    g = np.zeros(w)
    rc = lib().oracle_mtv(f64, _ptr(A), A.shape[1], A.shape[0], col0, w, _ptr(r), _ptr(g), nthreads)
    assert rc == 0, rc
    return g


def mv(A, col0, w, d, P=1, nthreads=0):
    """A[:, col0:col0+w] d, summed over P column shards (lasso.py:121-126)."""
    A, f64 = _a(A)
    d = np.ascontiguousarray(d, dtype=np.float64).reshape(-1)
    s = np.zeros(A.shape[0])
    rc = lib().oracle_mv(f64, _ptr(A), A.shape[1], A.shape[0], col0, w, P, _ptr(d), _ptr(s), nthreads)
    assert rc == 0, rc
    return s


def run(A, b, mu, nblock, iter_max, P=1, order=None, err_bound=None, x0=None,
        nthreads=0, want_gamma=False):
    """ClassLassoCPU.run restated (lasso.py:70-169). Returns dict(x, err_iter, t_last[, gamma])."""
    A, f64 = _a(A)
    m, n = A.shape
    b = np.ascontiguousarray(b, dtype=np.float64).reshape(-1)
    x = np.zeros(n) if x0 is None else np.array(x0, dtype=np.float64).reshape(-1).copy()
    err_iter = np.zeros(iter_max)
    gam = np.zeros(iter_max)
    t_last = np.zeros(1, dtype=np.int64)
    ordp = None
    if order is not None:
        order = np.ascontiguousarray(order, dtype=np.int32)
        assert order.shape[0] >= iter_max
        ordp = _ptr(order)
    rc = lib().oracle_run(f64, _ptr(A), n, m, n, nblock, P, _ptr(b), float(mu), iter_max,
                          ordp, -1.0 if err_bound is None else float(err_bound),
                          _ptr(x), _ptr(err_iter), _ptr(t_last), _ptr(gam), nthreads)
    assert rc == 0, rc
    out = dict(x=x, err_iter=err_iter, t_last=int(t_last[0]))
    if want_gamma:
        out["gamma"] = gam
    return out


def gauss_instance(seed, m, n, den=0.4, nthreads=0, A_out=None):
    """The Gaussian-recipe instance of oracle/gauss_instance.c (parameters.py:17-33 with the
    Irwin-Hall N(0, 1) approximant; bit-identical on every x86 host): (A fp32 [m][n], b, mu, x_true).
    b = A x_true + e and mu = 0.1 ||A^T b||_inf with the oracle's thread-count-invariant products.
    A_out: a C-contiguous float32 (m, n) array to fill (e.g. one view of pinned memory)."""
    A = np.empty((m, n), dtype=np.float32) if A_out is None else A_out
    assert A.dtype == np.float32 and A.shape == (m, n) and A.flags.c_contiguous
    xt, e = np.zeros(n), np.zeros(m)
    rc = lib().oracle_gauss_instance(int(seed), m, n, float(den), _ptr(A), _ptr(xt), _ptr(e), nthreads)
    assert rc == 0, rc
    b = mv(A, 0, n, xt, nthreads=nthreads) + e
    mu = 0.1 * float(np.abs(mtv(A, 0, n, b, nthreads=nthreads)).max())
    return A, b, mu, xt


def gauss_rows(seed, row0, nrows, n):
    """rows row0 .. row0 + nrows - 1 of gauss_instance's A, without building the rest"""
    out = np.empty((nrows, n), dtype=np.float32)
    assert lib().oracle_gauss_rows(int(seed), int(row0), int(nrows), int(n), _ptr(out)) == 0
    return out


# ---------------------------------------------------------------------------
# numpy restatement (small cases only), used to cross-check the C restatement
# ---------------------------------------------------------------------------
def run_numpy(A, b, mu, nblock, iter_max, order=None, err_bound=None, gemv_f32=False, dg=None):
    """gemv_f32: A kept in fp32 and the two GEMVs done in fp32 (OpenBLAS sgemv: the reference's
    TYPE='float' CPU path), everything else in fp64 -- the CPU-baseline variant of SURVEY 8d.
    dg: diag(A^T A) computed by the caller (so a timed call holds the iterations only)."""
    A = np.asarray(A, dtype=np.float32 if gemv_f32 else np.float64)
    gd = A.dtype
    m, n = A.shape
    w = n // nblock
    b = np.asarray(b, dtype=np.float64).reshape(-1)
    if dg is None:
        dg = np.square(A.astype(np.float64) if gemv_f32 else A).sum(axis=0)
    dg = np.asarray(dg, dtype=np.float64).reshape(nblock, w)
    x = np.zeros((nblock, w))
    Ax = np.zeros((nblock, m))
    err_iter = np.zeros(iter_max)
    cnt = 0
    t = 0
    for t in range(iter_max):
        mb = int(order[t]) if order is not None else t % nblock
        Am = A[:, mb * w:(mb + 1) * w]
        r = Ax.sum(axis=0) - b
        g = (Am.T @ r.astype(gd)).astype(np.float64)
        rx = dg[mb] * x[mb] - g
        st = np.sign(rx) * np.maximum(np.abs(rx) - mu, 0)
        Bx = (1.0 / dg[mb]) * st
        D = Bx - x[mb]
        s23 = (Am @ D.astype(gd)).astype(np.float64)
        r1 = r @ s23 + mu * (np.abs(Bx).sum() - np.abs(x[mb]).sum())
        r2 = s23 @ s23
        gamma = 0.0 if r2 == 0 else float(np.clip(-r1 / r2, 0, 1))
        err = np.max(np.abs(g - np.clip(g - x[mb], -mu, mu)))
        err_iter[t] = err
        if err_bound is not None:
            if err < err_bound:
                cnt += 1
            if nblock - 1 == mb:
                if cnt == nblock:
                    break
                cnt = 0
        x[mb] += gamma * D
        Ax[mb] += gamma * s23
    return dict(x=x.reshape(-1), err_iter=err_iter, t_last=t)


def regen_A(seed, N, K):
    """A of parameters.py:17-20 for a fixed seed (row-normalised N(0,1))."""
    A = np.random.RandomState(int(seed)).randn(int(N), int(K))
    return A / (np.linalg.norm(A, ord=2, axis=1, keepdims=True))


def fixture_A(fx):
    """Regenerate the fixture's A (fp32-rounded when the fixture says so) and check it."""
    A = regen_A(fx["seed"], fx["N"], fx["K"])
    if bool(fx["f32_inputs"]):
        A = A.astype(np.float32).astype(np.float64)
    ck = np.array([A.sum(), np.square(A).sum(), A[0, 0], A[-1, -1],
                   A[A.shape[0] // 2, A.shape[1] // 3]])
    if not np.array_equal(ck, fx["A_checksum"]):
        raise AssertionError("regenerated A does not match the fixture checksum")
    return A
