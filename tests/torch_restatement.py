"""TEST INFRASTRUCTURE -- the reference iteration (lasso.py:102-157, one feature block) restated in
torch fp64 on the GPU: the checker for full-size long horizons where the C oracle
(oracle/bpgl_oracle.c) would need many minutes (16 GiB of A, two passes per iteration).  It is the
same arithmetic as oracle.run_numpy (oracle/oracle.py) -- fp64 GEMVs on the stored A, the
reference's shrink (cpu_calculation.py:5-6), exact line search, err (cpu_calculation.py:15-20) --
with torch's summation order; tests/test_fullsize.py pins it to the C oracle on a small instance
before trusting it.  Never imported by the package."""
import torch


def run_torch(A, b, mu, iters, A64=None):
    """A (m, n) fp32/fp64 CUDA tensor, b (m,) -> dict(x, err_iter) (fp64 CUDA tensors).  A64: an
    fp64 copy of A the caller already holds (the GEMVs run on it)."""
    A64 = A.double() if A64 is None else A64
    b = b.double()
    m, n = A64.shape
    dg = (A64 * A64).sum(dim=0)
    x = torch.zeros(n, dtype=torch.float64, device=A.device)
    Ax = torch.zeros(m, dtype=torch.float64, device=A.device)
    err = torch.zeros(iters, dtype=torch.float64, device=A.device)
    for t in range(iters):
        r = Ax - b
        g = A64.t() @ r
        rx = dg * x - g
        Bx = torch.sign(rx) * torch.clamp(rx.abs() - mu, min=0.0) / dg
        D = Bx - x
        s23 = A64 @ D
        r1 = torch.dot(r, s23) + mu * (Bx.abs().sum() - x.abs().sum())
        r2 = torch.dot(s23, s23)
        gamma = torch.where(r2 == 0, torch.zeros_like(r2), torch.clamp(-r1 / r2, 0.0, 1.0))
        err[t] = (g - torch.clamp(g - x, -mu, mu)).abs().max()
        x = x + gamma * D
        Ax = Ax + gamma * s23
    return dict(x=x, err_iter=err)
