"""MI355X drop-in for the reference's ``gpu_calculation`` module.

``GPU_Calculation`` keeps the reference's names, attributes and call
semantics (gpu_calculation.py:141-292) so the reference drivers
(``ClassLasso`` / ``ClassLassoR``, lasso.py:173-306) run unchanged on it:

  * class tunables ``T_WIDTH_TRANS / T_WIDTH / T_HEIGHT / TYPE``
    (gpu_calculation.py:143-146).  ``TYPE`` selects how A is stored on the
    device ('double' as in the reference, 'float', or 'bf16'); arithmetic is
    fp64 in every case.  The three tile tunables belonged to the reference's
    CUDA tiling and are accepted but have no effect (the gfx950 geometry is
    derived from the shape, see ``geometry``).
  * attributes ``Block, MAT_HEIGHT, MAT_WIDTH, MAT_WIDTH_ALL`` and the device
    view ``A_b_gpu`` (Block, H, W) (gpu_calculation.py:149-150, 175, 224).
  * ``diag_ATA`` property -> host ndarray (Block, W, 1) fp64 (:246-261).
  * ``mat_tMulVec_DiffSize(s13, index_m, s11)`` and
    ``matMulVec_DiffSize(s23, index_m, descent_d)`` write into caller-owned
    arrays and return None (:264-292).  Host numpy arrays are accepted exactly
    as in the reference; CUDA tensors are accepted too and then nothing
    crosses PCIe.

New: ``run`` -- the whole solver loop resident on the
device, captured once as hipGraphs of 1, 2, 4, ..., 64 iterations, returning x, which
the reference's drivers never did (lasso.py:167-169, :609).  With one feature
block an iteration is ``k_onepass`` (A read once: s23 = A D and U = A^T s23,
the line search by its last row group) + ``k_onepass_tail`` (x, Ax, r,
g += gamma U and the next shrink), with an exact g = A^T r every 256
iterations; with several blocks (or ``onepass`` = 0) it is the two-pass
sequence colpass / shrink / rowpass / rowreduce (+ line search) / update.

Every compute call goes through libbpgl.so (``_native``); there is no
alternative path.  Multi-GPU: pass ``comm=`` (see ``distributed.RankComm``);
A is then this rank's column shard of every feature block (``shard="columns"``,
the reference's P-way split), or, with ``shard="rows"`` and one feature block,
this rank's rows of A (x replicated, one pass over A per iteration; see
``distributed`` and include/bpgl.h ``bpgl_set_shard``).  In row mode the GEMV
entry points return this rank's partial A_q^T r_q and its rows of A d.
"""
import contextlib
import ctypes

import numpy as np
import torch

from . import _native as N


def _resolve_device(A, device):
    if device is None:
        if isinstance(A, torch.Tensor) and A.is_cuda:
            return A.device
        return torch.device("cuda", torch.cuda.current_device())
    if isinstance(device, int):
        return torch.device("cuda", device)
    d = torch.device(device)
    return torch.device("cuda", d.index if d.index is not None else torch.cuda.current_device())


_MASKED_STREAMS = {}


def _masked_stream(device, mask):
    """The CU-masked stream of (device, mask), created once per process by libbpgl
    (bpgl_stream_create) and kept for the life of the process: torch's caching allocator keys the
    blocks of every tensor allocated on a stream by that stream, so the stream must outlive them
    (destroying it with the context crashed the allocator at exit)."""
    key = (device.index, tuple(mask))
    st = _MASKED_STREAMS.get(key)
    if st is None:
        words = (ctypes.c_uint32 * len(mask))(*mask)
        sp = ctypes.c_void_p()
        N.check(N.lib().bpgl_stream_create(device.index, words, len(mask), ctypes.byref(sp)), "bpgl_stream_create")
        st = torch.cuda.ExternalStream(sp.value, device=device)
        _MASKED_STREAMS[key] = st
    return st


class GPU_Calculation:
    T_WIDTH_TRANS = 64
    T_WIDTH = 64
    T_HEIGHT = 512
    TYPE = 'double'

    def __init__(self, A, Block, device=None, comm=None, shard="columns", cu_mask=None):
        """``cu_mask``: optional sequence of uint32 words (bit i = CU i) restricting the solver's
        stream to those CUs (several ranks sharing one GPU; see
        ``distributed.xcd_symmetric_cu_mask``); the persistent one-pass grid is then sized to them."""
        if shard not in ("columns", "rows"):
            raise ValueError("shard must be 'columns' or 'rows'")
        self.shard = shard
        self._cu_mask = None if cu_mask is None else [int(w) & 0xFFFFFFFF for w in cu_mask]
        self.Block = int(Block)
        self.MAT_WIDTH_ALL = int(A.shape[1])
        self.device = _resolve_device(A, device)
        self._dt = N.dtype_code(self.TYPE)
        self._comm = comm
        self._ctx = None
        self.init_cpu_array(A)
        self.init_gpu_array(A)

    # -- gpu_calculation.py:171-220 -------------------------------------------
    def init_cpu_array(self, A):
        H, K = int(A.shape[0]), int(A.shape[1])
        if self.Block <= 0 or K % self.Block:
            # np.hsplit(A, Block) raises the same way (gpu_calculation.py:172)
            raise ValueError("array split does not result in an equal division")
        self.MAT_HEIGHT, self.MAT_WIDTH = H, K // self.Block
        V = N.VEC_ELEMS[self._dt]
        self.MAT_WIDTH_PAD = -(-self.MAT_WIDTH // V) * V

    # -- gpu_calculation.py:222-236 -------------------------------------------
    def init_gpu_array(self, A):
        L = N.lib()
        H, W, Wp, B = self.MAT_HEIGHT, self.MAT_WIDTH, self.MAT_WIDTH_PAD, self.Block
        tdt = N.TORCH_DTYPE[self._dt]
        torch.cuda.set_device(self.device)
        if self._cu_mask is not None:
            self.stream = _masked_stream(self.device, self._cu_mask)
        else:
            self.stream = torch.cuda.Stream(device=self.device)
        ctx = ctypes.c_void_p()
        N.check(L.bpgl_create(ctypes.byref(ctx), self.device.index, self._dt, H, B * W, B,
                              ctypes.c_void_p(self.stream.cuda_stream)), "bpgl_create")
        self._ctx = ctx
        assert L.bpgl_block_width_padded(ctx) == Wp
        if self.shard == "rows":
            N.check(L.bpgl_set_shard(ctx, N.BPGL_SHARD_ROWS), "bpgl_set_shard")
        self.stream.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(self.stream):
            At = A if isinstance(A, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(A))
            if (At.is_cuda and At.dtype == tdt and At.is_contiguous() and Wp == W
                    and At.device == self.device and At.data_ptr() % 16 == 0):
                # bind the caller's (H, K) matrix in place: block b = columns [b W, (b+1) W)
                self._A_dev = At
                lda, bstride = B * W, W
            else:
                src = At.to(device=self.device, dtype=tdt, non_blocking=False)
                # reference layout np.hsplit -> (Block, H, W) (gpu_calculation.py:172-173), padded to Wp
                dev = torch.zeros((B, H, Wp), dtype=tdt, device=self.device)
                dev[:, :, :W].copy_(src.reshape(H, B, W).permute(1, 0, 2))
                del src
                self._A_dev = dev
                lda, bstride = Wp, H * Wp
            nbytes = int(L.bpgl_scratch_bytes(ctx))
            self._scratch = torch.empty(nbytes // 8 + 64, dtype=torch.float64, device=self.device)
            base = self._scratch.data_ptr()
            aligned = (base + 255) // 256 * 256
            self._lda, self._bstride = lda, bstride
            N.check(L.bpgl_bind(ctx, ctypes.c_void_p(self._A_dev.data_ptr()), lda, bstride,
                                ctypes.c_void_p(aligned), nbytes), "bpgl_bind")
            if self._comm is not None:
                self._comm.attach(self)
            self._diag = torch.empty((B, Wp), dtype=torch.float64, device=self.device)
            N.check(L.bpgl_diag_ata(ctx, N.ptr(self._diag)), "bpgl_diag_ata")
            self._vin_h = torch.empty(H, dtype=torch.float64, device=self.device)
            self._vin_w = torch.zeros(Wp, dtype=torch.float64, device=self.device)
            self._vout_h = torch.empty(H, dtype=torch.float64, device=self.device)
            self._vout_w = torch.empty(Wp, dtype=torch.float64, device=self.device)
        self.stream.synchronize()

    def __del__(self):
        try:
            if self._ctx is not None and N._lib is not None:
                self.stream.synchronize()
                N.lib().bpgl_destroy(self._ctx)
                self._ctx = None
        except Exception:
            pass

    # -- views / properties ---------------------------------------------------
    @property
    def A_b_gpu(self):
        """Device view (Block, H, W) of A (the reference's gpuarray, gpu_calculation.py:224)."""
        H, W, B = self.MAT_HEIGHT, self.MAT_WIDTH, self.Block
        if self._A_dev.dim() == 3:
            return self._A_dev[:, :, :W]
        return self._A_dev.view(H, B, W).permute(1, 0, 2)

    @property
    def diag_ATA(self):
        """Host (Block, W, 1) fp64 column sums of squares per block (gpu_calculation.py:246-261)."""
        self.stream.synchronize()
        return self._diag[:, :self.MAT_WIDTH].cpu().numpy().reshape(self.Block, self.MAT_WIDTH, 1)

    def geometry(self):
        v = [ctypes.c_int32() for _ in range(4)]
        N.check(N.lib().bpgl_geometry(self._ctx, *[ctypes.byref(x) for x in v]), "bpgl_geometry")
        return dict(nseg=v[0].value, nchunk=v[1].value, rows_per_chunk=v[2].value, seg_width=v[3].value)

    # -- GEMV entry points ----------------------------------------------------
    def _pinned(self, key, n):
        """Page-locked host staging buffer (fp64, >= n values) for the host-array GEMV calls of the
        reference's hybrid drivers: DMA straight from/to it instead of a pageable bounce."""
        buf = self.__dict__.setdefault("_pin", {}).get(key)
        if buf is None or buf.numel() < n:
            buf = torch.empty(n, dtype=torch.float64).pin_memory()
            self._pin[key] = buf
        return buf[:n]

    def _stage_in(self, v, dst, n):
        if isinstance(v, torch.Tensor):
            dst[:n].copy_(v.reshape(-1)[:n].to(dtype=torch.float64), non_blocking=True)
        else:
            a = np.asarray(v, dtype=np.float64).reshape(-1)[:n]
            pin = self._pinned("in%d" % dst.numel(), n)
            # the previous copy out of this buffer must have finished before it is overwritten
            if getattr(self, "_pin_in_event", None) is not None:
                self._pin_in_event.synchronize()
            pin.numpy()[...] = a
            dst[:n].copy_(pin, non_blocking=True)
            self._pin_in_event = torch.cuda.Event()
            self._pin_in_event.record(torch.cuda.current_stream(self.device))

    def _stage_out(self, src, out):
        if isinstance(out, torch.Tensor):
            out.view(-1).copy_(src.to(dtype=out.dtype))
        else:
            pin = self._pinned("out%d" % src.numel(), src.numel())
            pin.copy_(src, non_blocking=True)
            torch.cuda.current_stream(self.device).synchronize()
            out[...] = pin.numpy().reshape(out.shape)

    def mat_tMulVec_DiffSize(self, s13, index_m, s11):
        """s13 <- A_m^T s11 (gpu_calculation.py:264-277)."""
        m = self._block_index(index_m)
        with self._on_stream():
            self._stage_in(s11, self._vin_h, self.MAT_HEIGHT)
            N.check(N.lib().bpgl_mtv(self._ctx, m, N.ptr(self._vin_h), N.ptr(self._vout_w)), "bpgl_mtv")
            self._stage_out(self._vout_w[:self.MAT_WIDTH], s13)

    def matMulVec_DiffSize(self, s23, index_m, descent_d):
        """s23 <- A_m descent_d (gpu_calculation.py:280-292)."""
        m = self._block_index(index_m)
        with self._on_stream():
            self._stage_in(descent_d, self._vin_w, self.MAT_WIDTH)
            N.check(N.lib().bpgl_mv(self._ctx, m, N.ptr(self._vin_w), N.ptr(self._vout_h)), "bpgl_mv")
            self._stage_out(self._vout_h, s23)

    @contextlib.contextmanager
    def _on_stream(self):
        """Run on the library's stream, ordered after the caller's current stream and
        before anything the caller enqueues afterwards (so device tensors produced or
        consumed on torch's current stream are race-free)."""
        cur = torch.cuda.current_stream(self.device)
        self.stream.wait_stream(cur)
        with torch.cuda.stream(self.stream):
            yield
        cur.wait_stream(self.stream)

    def _block_index(self, index_m):
        m = int(index_m)
        if not 0 <= m < self.Block:
            raise IndexError(f"block index {m} out of range [0, {self.Block})")
        return m

    # -- device-resident solver (new) --------------------
    def solver_reset(self, b, mu, x0=None, order=None, err_bound=None, record_len=0, use_graph=True):
        """Prepare a device-resident run.  ``order``: None (cyclic) or a sequence of block indices."""
        L = N.lib()
        H, W, Wp, B = self.MAT_HEIGHT, self.MAT_WIDTH, self.MAT_WIDTH_PAD, self.Block
        with self._on_stream():
            self._b = torch.empty(H, dtype=torch.float64, device=self.device)
            self._stage_in(b, self._b, H)
            self._x = torch.zeros((B, Wp), dtype=torch.float64, device=self.device)
            if x0 is not None:
                x0t = x0 if isinstance(x0, torch.Tensor) else torch.from_numpy(
                    np.ascontiguousarray(np.asarray(x0, dtype=np.float64).reshape(-1)))
                self._x[:, :W].copy_(x0t.reshape(B, W).to(device=self.device, dtype=torch.float64))
            self._order = None
            if order is not None:
                o = np.ascontiguousarray(np.asarray(order, dtype=np.int32).reshape(-1))
                if o.size == 0 or o.min() < 0 or o.max() >= B:
                    raise ValueError("block order entries must lie in [0, Block)")
                self._order = torch.from_numpy(o).to(self.device)
            self._rec_len = int(record_len)
            self._err_iter = torch.zeros(max(1, record_len), dtype=torch.float64, device=self.device) \
                if record_len else None
            self._time_iter = torch.zeros(record_len + 1, dtype=torch.float64, device=self.device) \
                if record_len else None
            N.check(L.bpgl_solver_reset(
                self._ctx, N.ptr(self._b), float(mu), N.ptr(self._x), N.ptr(self._order),
                0 if self._order is None else int(self._order.numel()),
                -1.0 if err_bound is None else float(err_bound),
                N.ptr(self._err_iter), N.ptr(self._time_iter), self._rec_len, int(bool(use_graph))),
                "bpgl_solver_reset")

    def solver_step(self, n_iter):
        with self._on_stream():
            N.check(N.lib().bpgl_solver_step(self._ctx, int(n_iter)), "bpgl_solver_step")

    def solver_status(self):
        it, st, tl = ctypes.c_int64(), ctypes.c_int(), ctypes.c_int64()
        ga, er = ctypes.c_double(), ctypes.c_double()
        N.check(N.lib().bpgl_solver_status(self._ctx, ctypes.byref(it), ctypes.byref(st), ctypes.byref(tl),
                                           ctypes.byref(ga), ctypes.byref(er)), "bpgl_solver_status")
        return dict(iters=it.value, stopped=bool(st.value), t_last=tl.value, gamma=ga.value, err=er.value)

    def solver_stat(self, key):
        """Counter since the last reset (include/bpgl.h bpgl_solver_stat): "onepass", "refreshes",
        "fallbacks", "requested", "enqueued", "refresh_period", "cus", "cu_masked", "onepass_grid",
        "onepass_rows", "onepass_sb1"."""
        v = ctypes.c_int64()
        N.check(N.lib().bpgl_solver_stat(self._ctx, key.encode(), ctypes.byref(v)), "bpgl_solver_stat")
        return v.value

    def solver_x(self, complete=True):
        """Current iterate as a host ndarray (K_local,) in the reference's block order.

        complete=True (default) goes through solver_status first, so iterations a failed one-pass
        launch lost are re-run before x is read.  That call is COLLECTIVE for RCCL row shards (a
        pending recovery enqueues all-reduces): every rank must call it, as solver_status.  A caller
        that reads x on some ranks only (a gather on rank 0, say) passes complete=False on those
        ranks after a collective solver_status() -- x is then read as it stands, with no
        communication."""
        if complete:
            self.solver_status()
        else:
            self.stream.synchronize()
        return self._x[:, :self.MAT_WIDTH].reshape(-1).cpu().numpy().copy()

    def _ctx_residual(self):
        """Device view (H,) of the solver's residual s11 = sum_k Ax_k - b (lives in the scratch)."""
        addr = N.lib().bpgl_solver_residual(self._ctx)
        off = (addr - self._scratch.data_ptr()) // 8
        return self._scratch[off:off + self.MAT_HEIGHT]

    def solver_x_device(self):
        """Device view of x; call solver_status() first (it re-runs lost one-pass iterations)."""
        return self._x[:, :self.MAT_WIDTH]

    def solver_records(self, complete=True):
        """(err_iter, time_iter) host copies, after solver_status (as solver_x; collective for RCCL
        row shards unless complete=False)."""
        if complete:
            self.solver_status()
        else:
            self.stream.synchronize()
        if self._err_iter is None:
            return None, None
        return self._err_iter.cpu().numpy().copy(), self._time_iter.cpu().numpy().copy()

    # -- caller-performed exchange (validation of the sharded kernels on one GPU) --
    def set_ranks(self, rank, nranks):
        N.check(N.lib().bpgl_set_ranks(self._ctx, int(rank), int(nranks)), "bpgl_set_ranks")

    def set_diag(self, diag):
        """Install column norms computed elsewhere (external-exchange row shards: the sum of
        every rank's own ``_diag``); also refreshes 1/diag."""
        with self._on_stream():
            self._diag.copy_(diag.reshape(self._diag.shape).to(self._diag))
            N.check(N.lib().bpgl_set_diag(self._ctx, N.ptr(self._diag)), "bpgl_set_diag")

    def solver_phase(self, phase):
        with self._on_stream():
            N.check(N.lib().bpgl_solver_phase(self._ctx, int(phase)), "bpgl_solver_phase")

    def exchange_buffer(self, fp32=False):
        """Device view of the per-iteration exchange (lives in the scratch): column shards
        [s23 (m) | sum|Bx| | sum|x| | err slot per rank]; row shards [U (w_pad) | r.s23 | s23.s23 |
        failed] (``failed``: the rank's one-pass failure flag, see include/bpgl.h).
        ``fp32``: the row shards' fp32 format of phases 0/1 ("exchange_fp32" = 1), w_pad + 5
        float32 [U | r.s23 hi, lo | s23.s23 hi, lo | failed] at the same address."""
        cnt = ctypes.c_int64()
        addr = N.lib().bpgl_solver_exchange_buffer(self._ctx, ctypes.byref(cnt))
        off = (addr - self._scratch.data_ptr()) // 8
        if fp32:
            return self._scratch.view(torch.float32)[2 * off:2 * off + cnt.value + 2]
        return self._scratch[off:off + cnt.value]

    def set_tuning(self, key, value):
        N.check(N.lib().bpgl_set_tuning(self._ctx, key.encode(), int(value)), "bpgl_set_tuning")

    def set_kernel_timing(self, enable):
        N.check(N.lib().bpgl_set_kernel_timing(self._ctx, int(bool(enable))), "bpgl_set_kernel_timing")

    KERNEL_KINDS = ("colpass", "shrink", "rowpass", "rowreduce", "allreduce", "step", "update", "onepass",
                    "refresh")

    def kernel_times(self):
        arr = (ctypes.c_double * len(self.KERNEL_KINDS))()
        ns = ctypes.c_int64()
        N.check(N.lib().bpgl_kernel_times(self._ctx, arr, ctypes.byref(ns)), "bpgl_kernel_times")
        return dict(zip(self.KERNEL_KINDS, list(arr))), ns.value

    def run(self, b, mu, iters, err_bound=None, order=None, x0=None, record=False, use_graph=True):
        """Device-resident solver loop (lasso.py:102-157 per iteration).

        Returns dict(x, iters, stopped, t_last, gamma, err[, err_iter, time_iter]).
        ``order``: None -> cyclic t % Block (lasso.py:40-41); an int array -> that block sequence.
        """
        iters = int(iters)
        self.solver_reset(b, mu, x0=x0, order=order, err_bound=err_bound,
                          record_len=iters if record else 0, use_graph=use_graph)
        self.solver_step(iters)
        out = self.solver_status()
        out["x"] = self.solver_x()
        if record:
            out["err_iter"], out["time_iter"] = self.solver_records()
        return out
