"""TEST INFRASTRUCTURE -- a lasso instance that numpy (here, in the build container) and torch (on
the GPU box) generate bit for bit identically, so long-horizon oracle runs too slow for a gated
test can be computed once offline (tests/golden/make_longrun.py) and committed as small fixtures.

  A[i, j] = (u24(h(i n + j, sA)) - 2^23) 2^-24 s     s = 2^-round(log2 sqrt(n / 12)) (rows ~unit norm)
  x_true[j] = c_j in {-3..3} \\ {0} with probability ~0.4 (the density of cpu_vs_gpu.py:58), else 0
  b = A x_true + e,   e_i = (u24(h(i, sE)) - 2^23) 2^-34

h is a 32-bit integer mix with multipliers below 2^31, so every product fits in int64 on both
sides; u24 = h >> 8.  Every A entry is exact in fp32, and b is exact in fp64 whatever the
summation order: the terms are multiples of 2^-34 (A's grid times small integers, e's grid), and
every partial sum stays below 2^12 in magnitude at the BASELINE shapes -- so b needs < 47 significant bits.  mu is not
exact (A^T b products); the fixture stores the mu its oracle run used.
"""
import math

import numpy as np

M32 = 0xFFFFFFFF
GOLD = 0x61C88647
MUL1 = 0x7FEB352D
MUL2 = 0x68E31DA5
SEED_A, SEED_X, SEED_E = 0x1234567, 0x2345678, 0x3456789


def a_scale(n):
    return 2.0 ** -round(math.log2(math.sqrt(n / 12.0)))


def _mix(h):
    h = h ^ (h >> 16)
    h = (h * MUL1) & M32
    h = h ^ (h >> 15)
    h = (h * MUL2) & M32
    return h ^ (h >> 16)


def _hash(idx, seed):
    return _mix(((idx & M32) * GOLD + seed) & M32)


# ---------------------------------------------------------------- numpy (offline generator)
def np_rows(i0, i1, n):
    """rows [i0, i1) of A as float32"""
    idx = np.arange(i0 * n, i1 * n, dtype=np.int64)
    u = (_hash(idx, SEED_A) >> 8) - (1 << 23)
    return (u.astype(np.float32) * np.float32(2.0 ** -24 * a_scale(n))).reshape(i1 - i0, n)


def np_entries(rows, cols, n):
    """A[rows, cols] without building A"""
    idx = np.asarray(rows, dtype=np.int64) * n + np.asarray(cols, dtype=np.int64)
    u = (_hash(idx, SEED_A) >> 8) - (1 << 23)
    return u.astype(np.float32) * np.float32(2.0 ** -24 * a_scale(n))


def np_A(m, n, chunk_rows=None):
    chunk_rows = chunk_rows or max(1, (1 << 26) // n)
    A = np.empty((m, n), dtype=np.float32)
    for i0 in range(0, m, chunk_rows):
        i1 = min(m, i0 + chunk_rows)
        A[i0:i1] = np_rows(i0, i1, n)
    return A


def np_x_true(n):
    h = _hash(np.arange(n, dtype=np.int64), SEED_X)
    keep = (h & 0xFFFF) < int(0.4 * 65536)
    c = ((h >> 16) % 6).astype(np.int64)
    c = np.where(c < 3, c - 3, c - 2)          # -3, -2, -1, 1, 2, 3
    return np.where(keep, c, 0).astype(np.float64)


def np_e(m):
    u = (_hash(np.arange(m, dtype=np.int64), SEED_E) >> 8) - (1 << 23)
    return u.astype(np.float64) * 2.0 ** -34


def np_b(A, chunk_rows=None):
    m, n = A.shape
    x = np_x_true(n)
    chunk_rows = chunk_rows or max(1, (1 << 25) // n)
    b = np.empty(m)
    for i0 in range(0, m, chunk_rows):
        i1 = min(m, i0 + chunk_rows)
        b[i0:i1] = A[i0:i1].astype(np.float64) @ x
    return b + np_e(m)


# ---------------------------------------------------------------- torch (on the GPU box)
def torch_A(m, n, device, chunk_rows=None, row0=0):
    """rows [row0, row0 + m) of the instance's A (row0 > 0: one rank's row shard)"""
    import torch
    chunk_rows = chunk_rows or max(1, (1 << 26) // n)
    A = torch.empty((m, n), dtype=torch.float32, device=device)
    sc = 2.0 ** -24 * a_scale(n)
    for i0 in range(0, m, chunk_rows):
        i1 = min(m, i0 + chunk_rows)
        idx = torch.arange((row0 + i0) * n, (row0 + i1) * n, dtype=torch.int64, device=device)
        u = (_hash(idx, SEED_A) >> 8) - (1 << 23)
        A[i0:i1] = (u.to(torch.float32) * sc).reshape(i1 - i0, n)
    return A


def torch_b(A, chunk_rows=None, row0=0, m_total=None):
    """b of A's rows; for a row shard (A = rows [row0, row0 + m) of an m_total-row instance) the
    shard's entries of the whole instance's b"""
    import torch
    m, n = A.shape
    dev = A.device
    x = torch.from_numpy(np_x_true(n)).to(dev)
    chunk_rows = chunk_rows or max(1, (1 << 25) // n)
    b = torch.empty(m, dtype=torch.float64, device=dev)
    for i0 in range(0, m, chunk_rows):
        i1 = min(m, i0 + chunk_rows)
        b[i0:i1] = A[i0:i1].double() @ x
    e = np_e(m_total or m)[row0:row0 + m]
    return b + torch.from_numpy(e).to(dev)


def sample_points(m, n, k=4096, seed=7):
    """(rows, cols) of the A entries a fixture stores to prove both sides generated the same A"""
    rs = np.random.RandomState(seed)
    rows = np.concatenate([[0, m - 1], rs.randint(0, m, k - 2)])
    cols = np.concatenate([[0, n - 1], rs.randint(0, n, k - 2)])
    return rows.astype(np.int64), cols.astype(np.int64)


# ---------------------------------------------------------------- configs[4]: bf16 A, k right-hand sides
# A[i, j] = (h(i n + j, sA) >> 24 - 128) 2^-s, s = round(log2 sqrt(n * 5461)) (rows ~unit norm): an
# integer of at most 8 significant bits times a power of two, exact in bf16.  X_true[:, r] and e[:, r] as
# above with the seeds offset per right-hand side r; B = A X_true + E exact in fp64 in any summation
# order (terms on the 2^-34 grid, partial sums below 2^12 at m = 8192, n = 65536).
SEED_XK, SEED_EK = 0x4567891, 0x5678912


def bf16_scale(n):
    return 2.0 ** -round(math.log2(math.sqrt(n * 5461.0)))


def np_A_bf16(m, n, chunk_rows=None):
    """as float32 (every value exact in bf16)"""
    chunk_rows = chunk_rows or max(1, (1 << 26) // n)
    A = np.empty((m, n), dtype=np.float32)
    sc = np.float32(bf16_scale(n))
    for i0 in range(0, m, chunk_rows):
        i1 = min(m, i0 + chunk_rows)
        idx = np.arange(i0 * n, i1 * n, dtype=np.int64)
        A[i0:i1] = (((_hash(idx, SEED_A) >> 24) - 128).astype(np.float32) * sc).reshape(i1 - i0, n)
    return A


def np_entries_bf16(rows, cols, n):
    """A[rows, cols] of np_A_bf16 without building A"""
    idx = np.asarray(rows, dtype=np.int64) * n + np.asarray(cols, dtype=np.int64)
    return ((_hash(idx, SEED_A) >> 24) - 128).astype(np.float32) * np.float32(bf16_scale(n))


def torch_A_bf16(m, n, device, chunk_rows=None):
    import torch
    chunk_rows = chunk_rows or max(1, (1 << 26) // n)
    A = torch.empty((m, n), dtype=torch.float32, device=device)
    sc = bf16_scale(n)
    for i0 in range(0, m, chunk_rows):
        i1 = min(m, i0 + chunk_rows)
        idx = torch.arange(i0 * n, i1 * n, dtype=torch.int64, device=device)
        A[i0:i1] = (((_hash(idx, SEED_A) >> 24) - 128).to(torch.float32) * sc).reshape(i1 - i0, n)
    return A


def np_x_true_rhs(n, r):
    h = _hash(np.arange(n, dtype=np.int64) + np.int64(r) * n, SEED_XK)
    keep = (h & 0xFFFF) < int(0.4 * 65536)
    c = ((h >> 16) % 6).astype(np.int64)
    c = np.where(c < 3, c - 3, c - 2)
    return np.where(keep, c, 0).astype(np.float64)


def np_e_rhs(m, r):
    u = (_hash(np.arange(m, dtype=np.int64) + np.int64(r) * m, SEED_EK) >> 8) - (1 << 23)
    return u.astype(np.float64) * 2.0 ** -34


def np_b_rhs(A, r, chunk_rows=None):
    """column r of B (A as produced by np_A_bf16)"""
    m, n = A.shape
    x = np_x_true_rhs(n, r)
    chunk_rows = chunk_rows or max(1, (1 << 25) // n)
    b = np.empty(m)
    for i0 in range(0, m, chunk_rows):
        i1 = min(m, i0 + chunk_rows)
        b[i0:i1] = A[i0:i1].astype(np.float64) @ x
    return b + np_e_rhs(m, r)


def torch_B(A, k):
    """(m, k) fp64 right-hand sides for the torch A of torch_A_bf16"""
    import torch
    m, n = A.shape
    dev = A.device
    X = torch.from_numpy(np.stack([np_x_true_rhs(n, r) for r in range(k)], axis=1)).to(dev)
    E = torch.from_numpy(np.stack([np_e_rhs(m, r) for r in range(k)], axis=1)).to(dev)
    B = torch.empty((m, k), dtype=torch.float64, device=dev)
    for i0 in range(0, m, 1024):
        i1 = min(m, i0 + 1024)
        B[i0:i1] = A[i0:i1].double() @ X
    return B + E
