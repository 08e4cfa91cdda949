"""Vendor-library yardstick: the same iteration on rocBLAS GEMVs.

The reference's ``ClassLassoCB_v1`` / ``ClassLassoCB_v2`` (lasso.py:310-613) run the
iteration on cuBLAS ``Dgemv`` plus level-1 BLAS.  ``VendorLasso`` is that design on
MI355X: every step on the device through PyTorch, whose GEMVs dispatch to
rocBLAS / hipBLASLt; the block loop (lasso.py:102-157) is the reference's.

It is a comparison point for the bench, not the product path (that is
``GPU_Calculation.run`` on libbpgl.so): with ``dtype=torch.float64`` it is
numerically the reference (fp64 GEMV, vendor summation order); with
``torch.float32`` the GEMVs accumulate in fp32 (faster, not parity-equivalent).
"""
import torch


class VendorLasso:
    def __init__(self, A, Block, dtype=torch.float64, device=None):
        dev = torch.device("cuda", torch.cuda.current_device() if device is None else device)
        At = A if isinstance(A, torch.Tensor) else torch.from_numpy(A)
        H, K = At.shape
        if K % Block:
            raise ValueError("array split does not result in an equal division")
        self.Block, self.H, self.W = int(Block), int(H), int(K) // int(Block)
        self.dtype = dtype
        A_dev = At.to(device=dev, dtype=dtype)
        # (Block, H, W) contiguous blocks, as gpu_calculation.py:172-173 lays them out
        self.A_b = torch.stack([A_dev[:, k * self.W:(k + 1) * self.W].contiguous() for k in range(self.Block)])
        del A_dev
        self.device = dev
        # column norms per block (cpu_calculation.py:35-42), fp64
        self.diag = (self.A_b.to(torch.float64) ** 2).sum(dim=1)           # (Block, W)
        self.rec = 1.0 / self.diag

    def _gemv_t(self, m, r):
        return torch.mv(self.A_b[m].t(), r.to(self.dtype)).to(torch.float64)

    def _gemv(self, m, d):
        return torch.mv(self.A_b[m], d.to(self.dtype)).to(torch.float64)

    def reset(self, b, mu):
        self.b = torch.as_tensor(b, dtype=torch.float64, device=self.device).reshape(-1)
        self.mu = float(mu)
        self.x = torch.zeros(self.Block, self.W, dtype=torch.float64, device=self.device)
        self.Ax = torch.zeros(self.Block, self.H, dtype=torch.float64, device=self.device)
        self.t = 0

    def step(self, n_iter):
        """n_iter iterations of lasso.py:102-157 (cyclic blocks), all on the device."""
        mu = self.mu
        for _ in range(int(n_iter)):
            m = self.t % self.Block
            s11 = self.Ax.sum(dim=0) - self.b                                   # lasso.py:105
            g = self._gemv_t(m, s11)                                            # lasso.py:107-111
            xm = self.x[m]
            t_ = self.diag[m] * xm - g
            Bx = self.rec[m] * torch.sign(t_) * torch.clamp(t_.abs() - mu, min=0.0)   # lasso.py:114-117
            D = Bx - xm                                                         # lasso.py:119
            s23 = self._gemv(m, D)                                              # lasso.py:121-126
            r1 = torch.dot(s11, s23) + mu * (Bx.abs().sum() - xm.abs().sum())  # lasso.py:129-131
            r2 = torch.dot(s23, s23)                                            # lasso.py:132
            gamma = torch.where(r2 == 0, torch.zeros_like(r2), torch.clamp(-r1 / r2, 0.0, 1.0))
            self.x[m] += gamma * D                                              # lasso.py:153
            self.Ax[m] += gamma * s23                                           # lasso.py:155
            self.t += 1

    def solution(self):
        return self.x.reshape(-1).cpu().numpy()
