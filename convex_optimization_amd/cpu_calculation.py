"""Host-side helpers of the reference's ``cpu_calculation`` call surface.

The reference drivers import these eight functions (lasso.py:17-18,
cpu_vs_gpu.py:11) for the host part of each iteration.  They are kept here with
the same names, signatures, shapes and values so those drivers can import this
module in place of the reference's.  They act on host numpy arrays; the device
path (``gpu_calculation``) never calls them.

  soft_thresholding   cpu_calculation.py:5-6    S_tau(t) = sign(t) max(|t| - tau, 0)
  element_proj        cpu_calculation.py:10-11  clip(v, lo, hi)
  error_crit          cpu_calculation.py:15-20  || g - P_[-mu,mu](g - x) ||_inf
  A_bp_get            cpu_calculation.py:23-27  (N, K) -> (BLOCK, P, N, K/(BLOCK P)) view
  fun_s12             cpu_calculation.py:30-31  A_p^T s11
  fun_diag_ATA        cpu_calculation.py:35-42  per-block column sums of squares
  fun_s22             cpu_calculation.py:45-46  A_p s21
  fun_dd_p            cpu_calculation.py:49-50  (w, 1) -> (P, w/P, 1)
"""
import numpy as np


def soft_thresholding(tensor, threshold):
    shrunk = np.abs(tensor) - threshold
    np.maximum(shrunk, 0, out=shrunk)
    return np.sign(tensor) * shrunk


def element_proj(vec, lower_bound, upper_bound):
    return np.clip(vec, lower_bound, upper_bound) if np.ndim(vec) else \
        max(min(vec, upper_bound), lower_bound)


def error_crit(grad_fx, x, mu):
    resid = grad_fx - element_proj(grad_fx - x, -mu, mu)
    return np.max(np.abs(resid))


def A_bp_get(A, BLOCK, P):
    rows, cols = A.shape
    width = cols // (BLOCK * P)
    if width * BLOCK * P != cols:
        raise ValueError(f"K={cols} is not divisible by BLOCK*P={BLOCK * P}")
    # column c = (b P + p) width + j  ->  [b, p, :, j]
    return A.reshape(rows, BLOCK, P, width).transpose(1, 2, 0, 3)


def fun_s12(A_bp, s11):
    return A_bp.T @ s11


def fun_diag_ATA(A_bp):
    nblock, nshard, rows, width = A_bp.shape
    sq = np.einsum("bpij,bpij->bpj", A_bp, A_bp)
    return sq.reshape(nblock, nshard * width)[:, :, None]


def fun_s22(A_bp, s21):
    return A_bp @ s21


def fun_dd_p(P, descent_d):
    return np.reshape(descent_d, (P, -1, 1))
