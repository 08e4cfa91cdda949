"""k right-hand sides at once with bf16 A on CDNA4 MFMA (BASELINE configs[4]).

The reference solves one lasso problem per run (lasso.py:102-157).  The panel
path runs k in {16, 32, 64, 128} of them together on one matrix: each block
update computes G = A_m^T R and S = A_m D as MFMA panel products instead of
GEMVs, then applies the reference's shrink, exact line search and update to
every right-hand side (cyclic block order, fixed iteration count).

Numerics (stated tolerance): A is stored as bf16 (the problem is defined by the
bf16-rounded A); fp32 accumulation per block tile, fp64 after that.  The default
path (one feature block) is:

* the direction enters the A D pass as its bf16 rounding (d_split = 1; 2 = a
  hi + lo bf16 pair), and the line search is exact along the direction the MFMA
  saw, so every step is an exact line search (monotone objective);
* the gradient is carried (carry_g = 1): G_t = G_{t-1} + gamma A^T bf16(V) in
  fp32, with V = gamma S + the previous rounding (error feedback), and computed
  exactly from the residual's hi + lo bf16 pair every g_refresh = 64 iterations;
* x += gamma D' is applied by the next pass-1 epilogue (defer_x = 1; bitwise the
  same x).

Against the fp64 oracle on the same bf16 A: after the reference's 1000
iterations at the full configs[4] shape, x within 1e-4 relative l2 (measured
3.6-4.1e-6 for the default, 1.7-2.2e-5 for the exact-gradient forms) and the
objective within 1e-5 (measured ~1e-12) (tests/test_longrun.py).  Over short
runs the forms follow different trajectories to the same fixed point: x within
1e-2 and the objective within 1e-4 on the default path (tests/test_panel.py;
1e-5 for the exact-gradient hi + lo form).

All compute goes through libbpgl.so (bpgl_panel_* in include/bpgl.h).
"""
import contextlib
import ctypes

import numpy as np
import torch

from . import _native as N

_p = ctypes.c_void_p
_i64 = ctypes.c_int64
_i32 = ctypes.c_int32
_PANEL_SIGS = {
    "bpgl_panel_create": (ctypes.c_int, [ctypes.POINTER(_p), ctypes.c_int, _i64, _i64, _i32, _i32, _i32, _p]),
    "bpgl_panel_destroy": (None, [_p]),
    "bpgl_panel_scratch_bytes": (_i64, [_p]),
    "bpgl_panel_bind": (ctypes.c_int, [_p, _p, _i64, _p, _i64]),
    "bpgl_panel_diag": (ctypes.c_int, [_p, _p]),
    "bpgl_panel_mtm": (ctypes.c_int, [_p, _i32, _p, _p]),
    "bpgl_panel_mm": (ctypes.c_int, [_p, _i32, _p, _p]),
    "bpgl_panel_reset": (ctypes.c_int, [_p, _p, _p, _p, _i64, ctypes.c_int]),
    "bpgl_panel_step": (ctypes.c_int, [_p, _i64]),
    "bpgl_panel_status": (ctypes.c_int, [_p, ctypes.POINTER(_i64), ctypes.POINTER(ctypes.c_double)]),
    "bpgl_panel_x": (_p, [_p]),
    "bpgl_panel_set_kernel_timing": (ctypes.c_int, [_p, ctypes.c_int]),
    "bpgl_panel_kernel_times": (ctypes.c_int, [_p, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_i64)]),
    "bpgl_panel_geometry": (ctypes.c_int, [_p, ctypes.POINTER(_i32)]),
    "bpgl_panel_set_tuning": (ctypes.c_int, [_p, ctypes.c_char_p, _i64]),
    "bpgl_panel_get_tuning": (ctypes.c_int, [_p, ctypes.c_char_p, ctypes.POINTER(_i64)]),
    "bpgl_panel_stat": (ctypes.c_int, [_p, ctypes.c_char_p, ctypes.POINTER(_i64)]),
    "bpgl_panel_residual": (_p, [_p]),
}
N._SIGS.update(_PANEL_SIGS)


def _lib():
    L = N.lib()
    for name, (res, args) in _PANEL_SIGS.items():
        f = getattr(L, name)
        f.restype, f.argtypes = res, args
    return L


class PanelLasso:
    """k lasso problems sharing A (m x n, bf16), one block update per iteration for all of them."""

    KERNEL_KINDS = ("pass1_mfma", "pass2_mfma", "reduce", "step", "update")

    def __init__(self, A, Block=1, nrhs=128, device=None, kchunks=0, cu_mask=None, lda=None):
        """cu_mask: CU mask words (bit i = CU i) -> the solver runs on a CU-masked stream of its own
        (bpgl_stream_create; the fused reduce + update is admitted only if it fits those CUs).
        lda: row stride of the stored bf16 A (>= n, a multiple of 8; default n), the padding zeroed."""
        L = _lib()
        self.Block = int(Block)
        self.nrhs = int(nrhs)
        H, K = int(A.shape[0]), int(A.shape[1])
        if K % self.Block:
            raise ValueError("array split does not result in an equal division")
        self.MAT_HEIGHT, self.MAT_WIDTH, self.MAT_WIDTH_ALL = H, K // self.Block, K
        if device is None:
            device = A.device if isinstance(A, torch.Tensor) and A.is_cuda else torch.cuda.current_device()
        self.device = torch.device("cuda", torch.device(device).index if not isinstance(device, int) else device)
        torch.cuda.set_device(self.device)
        if cu_mask is not None:
            from .gpu_calculation import _masked_stream
            self.stream = _masked_stream(self.device, list(cu_mask))
        else:
            self.stream = torch.cuda.Stream(device=self.device)
        ctx = ctypes.c_void_p()
        N.check(L.bpgl_panel_create(ctypes.byref(ctx), self.device.index, H, K, self.Block, self.nrhs,
                                    int(kchunks), ctypes.c_void_p(self.stream.cuda_stream)), "bpgl_panel_create")
        self._ctx = ctx
        lda = K if lda is None else int(lda)
        self.lda = lda
        self.stream.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(self.stream):
            A_src = A if isinstance(A, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(A))
            A_src = A_src.to(device=self.device, dtype=torch.bfloat16)
            if lda == K:
                self._A = A_src.contiguous()                                                # [m][n]
            else:                                                                           # [m][lda]
                self._A_store = torch.zeros(H, lda, dtype=torch.bfloat16, device=self.device)
                self._A_store[:, :K] = A_src
                self._A = self._A_store[:, :K]
            nbytes = int(L.bpgl_panel_scratch_bytes(ctx))
            self._scratch = torch.empty(nbytes // 8 + 64, dtype=torch.float64, device=self.device)
            base = (self._scratch.data_ptr() + 255) // 256 * 256
            N.check(L.bpgl_panel_bind(ctx, ctypes.c_void_p(self._A.data_ptr()), lda, ctypes.c_void_p(base), nbytes),
                    "bpgl_panel_bind")
            self._diag = torch.empty(K, dtype=torch.float64, device=self.device)
            N.check(L.bpgl_panel_diag(ctx, N.ptr(self._diag)), "bpgl_panel_diag")
        self.stream.synchronize()
        kc = ctypes.c_int32()
        N.check(L.bpgl_panel_geometry(ctx, ctypes.byref(kc)), "bpgl_panel_geometry")
        self.kchunks = kc.value

    def __del__(self):
        try:
            if self._ctx is not None and N._lib is not None:
                self.stream.synchronize()
                N.lib().bpgl_panel_destroy(self._ctx)
                self._ctx = None
        except Exception:
            pass

    @contextlib.contextmanager
    def _on_stream(self):
        cur = torch.cuda.current_stream(self.device)
        self.stream.wait_stream(cur)
        with torch.cuda.stream(self.stream):
            yield
        cur.wait_stream(self.stream)

    @property
    def A_bf16(self):
        """A copy of the stored A (m x n, bf16) -- the matrix the problems are defined by.  A copy:
        bind took the passes' tiled images of A (include/bpgl.h), so writing into the stored A
        would change bpgl_panel_diag's input but not the solver's."""
        return self._A.clone()

    @property
    def diag_ATA(self):
        self.stream.synchronize()
        return self._diag.cpu().numpy().reshape(self.Block, self.MAT_WIDTH, 1)

    def _dev(self, v, shape):
        t = v if isinstance(v, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(v, dtype=np.float64))
        return t.to(device=self.device, dtype=torch.float64).reshape(shape)

    def mat_tMulMat(self, R, block=0):
        """G = A_block^T R for R (m, k) -> (w, k) fp64 (split-bf16 MFMA)."""
        with self._on_stream():
            Rt = self._dev(R, (self.MAT_HEIGHT, self.nrhs)).t().contiguous()
            G = torch.empty((self.nrhs, self.MAT_WIDTH), dtype=torch.float64, device=self.device)
            N.check(_lib().bpgl_panel_mtm(self._ctx, int(block), N.ptr(Rt), N.ptr(G)), "bpgl_panel_mtm")
            out = G.t().contiguous()
        return out

    def matMulMat(self, D, block=0):
        """S = A_block D for D (w, k) -> (m, k) fp64."""
        with self._on_stream():
            Dt = self._dev(D, (self.MAT_WIDTH, self.nrhs)).t().contiguous()
            S = torch.empty((self.nrhs, self.MAT_HEIGHT), dtype=torch.float64, device=self.device)
            N.check(_lib().bpgl_panel_mm(self._ctx, int(block), N.ptr(Dt), N.ptr(S)), "bpgl_panel_mm")
            out = S.t().contiguous()
        return out

    def solver_reset(self, B, mu, record_len=0, use_graph=True):
        """B (m, k) right-hand sides, mu scalar or (k,)."""
        with self._on_stream():
            self._Bt = self._dev(B, (self.MAT_HEIGHT, self.nrhs)).t().contiguous()
            mu_v = np.broadcast_to(np.asarray(mu, dtype=np.float64), (self.nrhs,)).copy()
            self._mu = torch.from_numpy(mu_v).to(self.device)
            self._err_iter = torch.zeros(max(1, record_len), dtype=torch.float64, device=self.device) \
                if record_len else None
            N.check(_lib().bpgl_panel_reset(self._ctx, N.ptr(self._Bt), N.ptr(self._mu), N.ptr(self._err_iter),
                                            int(record_len), int(bool(use_graph))), "bpgl_panel_reset")

    def solver_step(self, n_iter):
        with self._on_stream():
            N.check(_lib().bpgl_panel_step(self._ctx, int(n_iter)), "bpgl_panel_step")

    def solver_status(self):
        it, err = ctypes.c_int64(), ctypes.c_double()
        N.check(_lib().bpgl_panel_status(self._ctx, ctypes.byref(it), ctypes.byref(err)), "bpgl_panel_status")
        return dict(iters=it.value, err=err.value)

    def solver_x_device(self):
        """(k, n) fp32 view of the iterates (row j = right-hand side j)."""
        addr = _lib().bpgl_panel_x(self._ctx)
        off = (addr - self._scratch.data_ptr())
        assert off % 4 == 0
        flat = self._scratch.view(torch.float32)[off // 4: off // 4 + self.Block * self.nrhs * self.MAT_WIDTH]
        return flat.view(self.Block, self.nrhs, self.MAT_WIDTH).permute(1, 0, 2).reshape(self.nrhs, -1)

    def solver_x(self):
        self.stream.synchronize()
        return self.solver_x_device().to(torch.float64).cpu().numpy().T.copy()   # (n, k)

    def set_tuning(self, key, value):
        """Speed-only knobs (bitwise-identical results): 'interleave1' / 'interleave2' / 'interleave'
        0-2 (the mainloop form; default: the measured best per pass); 'defer_x' 0 / 1 (default 1, one
        block: where x += gamma D' is applied; a reset must follow).

        Knobs that change the arithmetic (each an exact line search along the direction taken; the
        accuracy of each against the oracle is in the module docstring): 'd_split' 1 (default) / 2 --
        the direction as its bf16 rounding or a hi + lo pair; 'carry_g' 1 (default, one block) / 0 --
        the carried fp32 gradient or the exact A^T R product every iteration; 'g_refresh' (default 64,
        a multiple of 8) -- the carried gradient's exact recompute period (include/bpgl.h)."""
        N.check(_lib().bpgl_panel_set_tuning(self._ctx, key.encode(), int(value)), "bpgl_panel_set_tuning")

    def get_tuning(self, key):
        v = ctypes.c_int64()
        N.check(_lib().bpgl_panel_get_tuning(self._ctx, key.encode(), ctypes.byref(v)), "bpgl_panel_get_tuning")
        return v.value

    def stat(self, key):
        """Counter since the last reset: "iters_enqueued", "exact_gradients"."""
        v = ctypes.c_int64()
        N.check(_lib().bpgl_panel_stat(self._ctx, key.encode(), ctypes.byref(v)), "bpgl_panel_stat")
        return v.value

    def residual_device(self):
        """(k, m) fp64 device view of the solver's residual R = A X - B (drain the stream first)."""
        addr = _lib().bpgl_panel_residual(self._ctx)
        off = addr - self._scratch.data_ptr()
        assert off % 8 == 0
        return self._scratch[off // 8: off // 8 + self.nrhs * self.MAT_HEIGHT].view(self.nrhs, self.MAT_HEIGHT)

    def set_kernel_timing(self, enable):
        N.check(_lib().bpgl_panel_set_kernel_timing(self._ctx, int(bool(enable))), "bpgl_panel_set_kernel_timing")

    def kernel_times(self):
        arr = (ctypes.c_double * 5)()
        ns = ctypes.c_int64()
        N.check(_lib().bpgl_panel_kernel_times(self._ctx, arr, ctypes.byref(ns)), "bpgl_panel_kernel_times")
        return dict(zip(self.KERNEL_KINDS, list(arr))), ns.value

    def run(self, B, mu, iters, record=False, use_graph=True):
        """Returns dict(x (n, k) fp64 copy of the fp32 iterates, iters, err[, err_iter])."""
        self.solver_reset(B, mu, record_len=int(iters) if record else 0, use_graph=use_graph)
        self.solver_step(int(iters))
        out = self.solver_status()
        out["x"] = self.solver_x()
        if record:
            self.stream.synchronize()
            out["err_iter"] = self._err_iter.cpu().numpy().copy()
        return out
