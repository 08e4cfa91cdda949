"""Problem instances for the lasso path (the step before it, reference parameters.py:13-69).

``parameters`` keeps the reference's signature and recipe: A ~ N(0, 1) with
rows scaled to unit l2 norm, x_true sparse with density ``den`` and N(0, 1)
values, b = A x_true + N(0, 1e-4), mu = 0.1 ||A^T b||_inf.  The reference seeds
numpy with ``int(time())`` (parameters.py:17); here ``seed`` pins that value,
and the same global-RNG draw order makes a seeded instance identical to the
reference's for that seed.  ``SAVE_FLAG`` / ``READ_FLAG`` read and write the
reference's text files (A_matrix.txt comma-delimited, x_true.txt,
b_vector.txt, parameters.txt = [N, K, den, mu]) in ``directory``.

``device_instance`` builds the large benchmark instances directly in HBM
(torch RNG, not the reference's stream) and derives b and mu with this
package's own kernels.
"""
import os
import time

import numpy as np


def parameters(N, K, den, SAVE_FLAG=False, READ_FLAG=False, SILENCE=False, seed=None,
               directory=None):
    directory = directory or os.path.join(os.path.expanduser("~"), "Documents", "python")
    if not READ_FLAG:
        np.random.seed(int(time.time()) if seed is None else int(seed))
        A = np.random.randn(N, K)
        A = A / np.linalg.norm(A, ord=2, axis=1, keepdims=True)
        from scipy import sparse
        x_true = sparse.random(K, 1, density=den, format="csc", data_rvs=np.random.randn)
        e = np.random.normal(0.0, np.sqrt(1e-4), (N, 1))
        b = A @ x_true + e
        mu = 0.1 * np.max(np.abs(A.T @ b))
        if not SILENCE:
            print(f"Parameters @@created with N: {N} , K: {K} , DENSITY: {den:f} , mu: {mu:f}.")
    else:
        A = np.loadtxt(os.path.join(directory, "A_matrix.txt"), delimiter=",", ndmin=2)
        x_true = np.loadtxt(os.path.join(directory, "x_true.txt"), ndmin=1)[:, None]
        b = np.loadtxt(os.path.join(directory, "b_vector.txt"), ndmin=1)[:, None]
        N, K, den, mu = np.loadtxt(os.path.join(directory, "parameters.txt"))
        if not SILENCE:
            print(f"Parameters @@loaded with N: {int(N)} , K: {int(K)} , DENSITY: {den:f} , mu: {mu:f} .")
    if SAVE_FLAG:
        os.makedirs(directory, exist_ok=True)
        np.savetxt(os.path.join(directory, "A_matrix.txt"), A, delimiter=",")
        xt = x_true.todense() if hasattr(x_true, "todense") else x_true
        np.savetxt(os.path.join(directory, "x_true.txt"), xt)
        np.savetxt(os.path.join(directory, "b_vector.txt"), b)
        np.savetxt(os.path.join(directory, "parameters.txt"), [N, K, den, mu])
        if not SILENCE:
            print("Paramenters @@saved!")
    return A, x_true, b, mu


def device_instance(N, K, den, Block, TYPE="float", seed=0, device=None, gpu_cal_cls=None, comm=None,
                    col_range=None, row_range=None, cu_mask=None):
    """Build (gpu_cal, b, mu, x_true) with A generated in HBM.

    A is drawn with torch's CUDA generator in fp32, its rows scaled to unit
    norm, and stored as ``TYPE``.  b = A x_true + 0.01 e is formed with the
    package's own A.d kernel (fp64), mu = 0.1 ||A^T b||_inf with its A^T r
    kernel.  ``row_range=(start, stop)``: this rank's rows only (row shards, one
    block; b is local, A^T b summed over ranks).  ``col_range``/``comm``: build only this rank's column shard (the
    full row normalisation is computed from row sums all ranks agree on).
    ``cu_mask``: passed to GPU_Calculation (the solver stream's CUs, several ranks on one GPU).
    """
    import torch
    from .gpu_calculation import GPU_Calculation
    cls = gpu_cal_cls or GPU_Calculation
    dev = torch.device("cuda", torch.cuda.current_device() if device is None else device)
    g = torch.Generator(device=dev)
    g.manual_seed(int(seed))
    A = torch.randn((N, K), generator=g, device=dev, dtype=torch.float32)
    A.div_(torch.linalg.vector_norm(A, dim=1, keepdim=True))
    xg = torch.Generator(device=dev)
    xg.manual_seed(int(seed) + 1)
    mask = torch.rand(K, generator=xg, device=dev) < den
    x_true = torch.where(mask, torch.randn(K, generator=xg, device=dev, dtype=torch.float64),
                         torch.zeros((), dtype=torch.float64, device=dev))
    e = 0.01 * torch.randn(N, generator=xg, device=dev, dtype=torch.float64)
    if row_range is not None:
        if col_range is not None or Block != 1:
            raise ValueError("row shards take one feature block and no column range")
        r0, r1 = int(row_range[0]), int(row_range[1])
        A = A[r0:r1].clone()
        e = e[r0:r1]
    if col_range is not None:
        A = A[:, col_range].contiguous()
        x_loc = x_true[col_range]
    else:
        x_loc = x_true
    tdt = {"float": torch.float32, "double": torch.float64, "bf16": torch.bfloat16}[TYPE]
    if tdt != torch.float32:
        A = A.to(tdt)
    old = cls.TYPE
    cls.TYPE = TYPE
    try:
        gc = cls(A, Block, device=dev, comm=comm, shard="rows" if row_range is not None else "columns",
                 cu_mask=cu_mask)
    finally:
        cls.TYPE = old
    del A
    H, W = gc.MAT_HEIGHT, gc.MAT_WIDTH
    b = torch.zeros(H, dtype=torch.float64, device=dev)
    tmp = torch.empty(H, dtype=torch.float64, device=dev)
    for k in range(Block):
        gc.matMulVec_DiffSize(tmp, k, x_loc[k * W:(k + 1) * W])
        b += tmp
    if comm is not None and comm.world > 1 and row_range is None:
        import torch.distributed as dist
        bc = b.cpu()
        dist.all_reduce(bc, group=comm.group)
        b = bc.to(dev)
    b += e
    gmax = torch.zeros((), dtype=torch.float64, device=dev)
    gt = torch.empty(W, dtype=torch.float64, device=dev)
    for k in range(Block):
        gc.mat_tMulVec_DiffSize(gt, k, b)
        if row_range is not None and comm is not None and comm.world > 1:
            import torch.distributed as dist
            gp = gt.cpu()                      # this rank's rows' share of A^T b
            dist.all_reduce(gp, group=comm.group)
            gt = gp.to(dev)
        gmax = torch.maximum(gmax, gt.abs().max())
    if comm is not None and comm.world > 1:
        import torch.distributed as dist
        gm = gmax.cpu().reshape(1)
        dist.all_reduce(gm, op=dist.ReduceOp.MAX, group=comm.group)
        gmax = gm[0]
    mu = 0.1 * float(gmax)
    return gc, b, mu, x_true
