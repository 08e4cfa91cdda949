"""Column-sharded multi-GPU path: one process per GPU, RCCL over xGMI.

The reference's only parallelism is the P-way column sharding of every
feature block across ``multiprocessing.Pool`` workers (cpu_calculation.py:23-27,
lasso.py:101-126): A_p^T r is concatenated over shards, A_p d_p is summed over
shards.  Here the shards are GPUs: rank g holds columns
[b w + g w/G, b w + (g+1) w/G) of every feature block b, resident in its HBM.
Per iteration each rank computes its slice of D with no communication (the
shrink is per column) and the partial s23 = A_g D_g; one RCCL all-reduce
(SUM) of m + 2 + G fp64 values (s23 | ||Bx||_1 | ||x||_1 | per-rank error
slots) then gives every rank the identical step size.  The all-reduce is
issued by libbpgl on the solver stream (inside the captured graph).

Row shards (``shard="rows"``, one feature block; no reference counterpart):
rank g holds rows ``row_bounds(m, g, G)`` of A, its rows of b and of the
residual, and a replicated x.  Every iteration streams the local A once
(k_onepass: s23_g = A_g D and U_g = A_g^T s23_g together), and ONE all-reduce
(SUM) of w_pad + 3 fp64 [U | r.s23 | s23.s23 | failed] gives every rank the identical
gradient update g += gamma U and step size.  Column shards need A read twice
per iteration (the exchange of s23 sits between the two products); row shards
trade that second pass for a w-sized exchange, which is the better deal on
xGMI whenever w * 8 B / (all-reduce bandwidth) < the pass time (configs[2]:
4 MiB vs ~2 GiB of A per GPU).

torch.distributed is only the side channel that carries the 128-byte RCCL
unique id (gloo, CPU tensors); the data path never touches it.
"""
import ctypes
import os

import numpy as np


def env_rank_world():
    """(rank, world, local_rank) from torchrun-style environment variables."""
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return rank, world, local


def shard_bounds(K, Block, rank, nranks):
    """Global column ranges [(start, stop)] this rank owns, one per feature block."""
    if K % Block:
        raise ValueError("K must be divisible by Block")
    w = K // Block
    if w % nranks:
        raise ValueError(f"block width {w} must be divisible by the number of ranks {nranks}")
    ws = w // nranks
    return [(b * w + rank * ws, b * w + (rank + 1) * ws) for b in range(Block)]


def shard_columns(A, Block, rank, nranks):
    """This rank's (H, K/nranks) slice of A, blocks kept in order (numpy or torch)."""
    parts = [A[:, s:e] for s, e in shard_bounds(A.shape[1], Block, rank, nranks)]
    if isinstance(A, np.ndarray):
        return np.ascontiguousarray(np.concatenate(parts, axis=1))
    import torch
    return torch.cat(parts, dim=1).contiguous()


def row_bounds(m, rank, nranks):
    """Rows [start, stop) of rank `rank` (balanced; the first m % nranks ranks get one more)."""
    if not 0 <= rank < nranks or m < nranks:
        raise ValueError(f"cannot split {m} rows over {nranks} ranks")
    q, r = divmod(m, nranks)
    start = rank * q + min(rank, r)
    return start, start + q + (1 if rank < r else 0)


def shard_rows(A, rank, nranks):
    """This rank's rows of A (numpy or torch; contiguous copy)."""
    s, e = row_bounds(A.shape[0], rank, nranks)
    if isinstance(A, np.ndarray):
        return np.ascontiguousarray(A[s:e])
    return A[s:e].contiguous()


def xcd_symmetric_cu_mask(rank, nranks, cus=256):
    """CU mask words (bit i = CU i) giving rank `rank` of `nranks` (1, 2, 4 or 8) processes that
    share one GPU a disjoint 1/nranks of its CUs, the same number on every XCD.

    The mask is built so that it does not depend on how the driver maps mask bits to XCDs: bits
    interleaved over the 8 XCDs (bit i on XCD i mod 8) or in XCD-sized runs (word j = XCD j's 32
    CUs).  For 1, 2 or 4 ranks every 32-bit word is split into four bytes and a rank takes whole
    bytes (rank k of 2: bytes k and k + 2; of 4: byte k): a byte holds one bit of each residue
    mod 8 and a word is one XCD, so either way every XCD gets 32/nranks of the rank's CUs.  For 8
    ranks (4 CUs per XCD each; needs 8 words) rank k takes, in word j, the four bits of residue
    (k + j) mod 8: 4 bits of every word (runs), and over the 8 words 4 bits of every residue
    (interleaved).  The one-pass grid is persistent: an XCD left without CUs would never run its
    share of blocks."""
    if nranks not in (1, 2, 4, 8):
        raise ValueError("CU partitions are built for 1, 2, 4 or 8 ranks per GPU")
    if not 0 <= rank < nranks:
        raise ValueError(f"rank {rank} out of range for {nranks}")
    if cus % 32:
        raise ValueError("the device's CU count must be a multiple of 32")
    words = cus // 32
    if nranks == 8:
        if words != 8:
            raise ValueError("8 CU partitions need 8 XCD-sized mask words (256 CUs)")
        return [sum(1 << (8 * q + (rank + j) % 8) for q in range(4)) for j in range(words)]
    per = 4 // nranks
    word = 0
    for k in range(per):
        word |= 0xFF << (8 * (rank + k * nranks))
    return [word] * words


def row_exchange_layout(wp):
    """Offsets in the row-shard all-reduce buffer (SUM over ranks); `failed` carries each rank's
    one-pass failure flag (a nonzero sum makes every rank skip the iteration)."""
    return dict(u=(0, wp), rs=wp, ss=wp + 1, failed=wp + 2, count=wp + 3)


def assemble_x(x_shards, Block):
    """Inverse of the sharding: list (rank order) of local x -> global x (K,)."""
    nr = len(x_shards)
    per = [np.asarray(x).reshape(Block, -1) for x in x_shards]
    return np.concatenate([np.concatenate([per[g][b] for g in range(nr)]) for b in range(Block)])


def _rccl_unique_id():
    from . import _native as N
    buf = (ctypes.c_uint8 * 128)()
    N.check(N.lib().bpgl_comm_unique_id(buf), "bpgl_comm_unique_id")
    return bytes(buf)


def exchange_layout(m, nranks):
    """Offsets in the per-iteration all-reduce buffer (SUM over ranks)."""
    return dict(s23=(0, m), l1_bx=m, l1_x=m + 1, err=(m + 2, m + 2 + nranks), count=m + 2 + nranks)


class RankComm:
    """RCCL communicator of one rank, created inside libbpgl for a GPU_Calculation.

    ``group`` is a torch.distributed process group (any backend; gloo is used
    by bench.py and the CPU tests) used once to broadcast the unique id.
    """

    def __init__(self, rank, world, group=None, id_provider=None):
        self.rank, self.world, self.group = int(rank), int(world), group
        self._id_provider = id_provider or _rccl_unique_id

    def unique_id(self):
        """Rank 0 creates the 128-byte RCCL id; every rank returns the same bytes."""
        import torch
        import torch.distributed as dist
        raw = self._id_provider() if self.rank == 0 else bytes(128)
        if len(raw) != 128:
            raise ValueError("an RCCL unique id is 128 bytes")
        t = torch.tensor(list(raw), dtype=torch.uint8)
        if self.world > 1:
            dist.broadcast(t, src=0, group=self.group)
        return bytes(t.tolist())

    def attach(self, gpu_cal):
        from . import _native as N
        uid = self.unique_id()
        raw = (ctypes.c_uint8 * 128).from_buffer_copy(uid)
        N.check(N.lib().bpgl_comm_init(gpu_cal._ctx, raw, self.rank, self.world), "bpgl_comm_init")
