"""Multi-rank host logic on CPU (gloo, world_size 2): column sharding, the RCCL
id broadcast, and the per-iteration exchange protocol of the sharded solver
(one SUM all-reduce of [s23 | sum|Bx| | sum|x| | per-rank err slots]) checked
against the single-rank oracle."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from convex_optimization_amd import distributed as D
from oracle import oracle


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _spawn(fn, world, *args):
    port = _free_port()
    mp.spawn(fn, args=(world, port) + args, nprocs=world, join=True)


def _init(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)


def test_shard_bounds_and_assemble():
    K, B, G = 48, 3, 4
    bounds = [D.shard_bounds(K, B, g, G) for g in range(G)]
    cols = sorted(c for g in range(G) for s, e in bounds[g] for c in range(s, e))
    assert cols == list(range(K))
    A = np.arange(2 * K, dtype=np.float64).reshape(2, K)
    shards = [D.shard_columns(A, B, g, G) for g in range(G)]
    # local layout keeps the feature blocks in order
    assert shards[1].shape == (2, K // G)
    x = np.arange(K, dtype=np.float64)
    xs = [np.concatenate([x[s:e] for s, e in bounds[g]]) for g in range(G)]
    np.testing.assert_array_equal(D.assemble_x(xs, B), x)
    with pytest.raises(ValueError):
        D.shard_bounds(50, 3, 0, 2)


def _uid_worker(rank, world, port, out):
    _init(rank, world, port)
    provider = (lambda: bytes(range(128))) if rank == 0 else (lambda: (_ for _ in ()).throw(AssertionError))
    comm = D.RankComm(rank, world, id_provider=provider)
    uid = comm.unique_id()
    out[rank] = list(uid)
    dist.destroy_process_group()


def test_unique_id_broadcast_gloo():
    mgr = mp.Manager()
    out = mgr.dict()
    _spawn(_uid_worker, 2, out)
    assert out[0] == out[1] == list(range(128))


def _rank_iterations(A_loc, b, mu, B, iters, rank, world):
    """One rank of the column-sharded solver, restating the device kernels'
    per-rank work (k_colpass/k_shrink/k_rowpass/k_rowreduce mode 2, k_step,
    k_update) with the gloo all-reduce standing in for RCCL."""
    m, nloc = A_loc.shape
    w = nloc // B
    dg = np.square(A_loc).sum(axis=0).reshape(B, w)
    x = np.zeros((B, w))
    Ax = np.zeros((B, m))
    lay = D.exchange_layout(m, world)
    for t in range(iters):
        mb = t % B
        Am = A_loc[:, mb * w:(mb + 1) * w]
        r = Ax.sum(axis=0) - b
        g = Am.T @ r
        bx = (1.0 / dg[mb]) * np.sign(dg[mb] * x[mb] - g) * np.maximum(np.abs(dg[mb] * x[mb] - g) - mu, 0)
        Dv = bx - x[mb]
        buf = np.zeros(lay["count"])
        buf[:m] = Am @ Dv
        buf[lay["l1_bx"]] = np.abs(bx).sum()
        buf[lay["l1_x"]] = np.abs(x[mb]).sum()
        buf[lay["err"][0] + rank] = np.max(np.abs(g - np.clip(g - x[mb], -mu, mu)))
        tb = torch.from_numpy(buf)
        dist.all_reduce(tb)
        buf = tb.numpy()
        s23 = buf[:m]
        r1 = r @ s23 + mu * (buf[lay["l1_bx"]] - buf[lay["l1_x"]])
        r2 = s23 @ s23
        gamma = 0.0 if r2 == 0 else min(max(-r1 / r2, 0.0), 1.0)
        x[mb] += gamma * Dv
        Ax[mb] += gamma * s23
    return x.reshape(-1)


def _solver_worker(rank, world, port, out):
    _init(rank, world, port)
    fx = dict(np.load(os.path.join(os.path.dirname(__file__), "golden", "c1_b2_p4_f32in.npz")))
    A = oracle.fixture_A(fx)
    B = int(fx["BLOCK"])
    A_loc = D.shard_columns(A, B, rank, world)
    out[rank] = _rank_iterations(A_loc, fx["b"].reshape(-1), float(fx["mu"]), B, 60, rank, world).tolist()
    dist.destroy_process_group()


def test_sharded_exchange_protocol_matches_single_rank():
    mgr = mp.Manager()
    out = mgr.dict()
    _spawn(_solver_worker, 2, out)
    fx = dict(np.load(os.path.join(os.path.dirname(__file__), "golden", "c1_b2_p4_f32in.npz")))
    A = oracle.fixture_A(fx)
    ref = oracle.run(A, fx["b"], float(fx["mu"]), int(fx["BLOCK"]), 60)["x"]
    x = D.assemble_x([np.array(out[0]), np.array(out[1])], int(fx["BLOCK"]))
    assert np.linalg.norm(x - ref) <= 1e-10 * np.linalg.norm(ref)


def test_row_bounds_cover_and_balance():
    for m, G in [(10, 3), (8192, 8), (7, 7), (1001, 4)]:
        b = [D.row_bounds(m, g, G) for g in range(G)]
        assert b[0][0] == 0 and b[-1][1] == m
        assert all(b[g][1] == b[g + 1][0] for g in range(G - 1))
        sizes = [e - s for s, e in b]
        assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        D.row_bounds(3, 0, 4)
    A = np.arange(20.0).reshape(5, 4)
    np.testing.assert_array_equal(np.concatenate([D.shard_rows(A, g, 2) for g in range(2)]), A)
    assert D.row_exchange_layout(16) == dict(u=(0, 16), rs=16, ss=17, failed=18, count=19)


def _row_rank_iterations(A_loc, b_loc, mu, iters, refresh, fail_at=None):
    """One rank of the row-sharded one-pass solver, restating the device kernels' per-rank
    work (k_onepass, k_onepass_fold, k_onepass_tail with the line search at its head; colpass +
    all-reduce for the exact gradient) with the gloo all-reduce standing in for RCCL.
    ``fail_at``: this rank's launch of that iteration reports a hand-off failure once; the
    summed `failed` slot makes every rank skip the iteration, which is then run again (what
    bpgl_solver_status does for RCCL row shards)."""
    def allreduce(v):
        t = torch.from_numpy(np.ascontiguousarray(v, dtype=np.float64))
        dist.all_reduce(t)
        return t.numpy()

    w = A_loc.shape[1]
    dg = allreduce(np.square(A_loc).sum(axis=0))
    x = np.zeros(w)
    Ax = np.zeros(A_loc.shape[0])
    r = Ax - b_loc
    g = allreduce(A_loc.T @ r)

    def shrink(g, x):
        rx = dg * x - g
        bx = np.sign(rx) * np.maximum(np.abs(rx) - mu, 0) / dg
        return bx, bx - x
    bx, Dv = shrink(g, x)
    lay = D.row_exchange_layout(w)
    t = 0
    while t < iters:
        if refresh and t and t % refresh == 0:
            g = allreduce(A_loc.T @ r)
            bx, Dv = shrink(g, x)
        s23 = A_loc @ Dv
        buf = np.zeros(lay["count"])
        buf[:w] = A_loc.T @ s23
        buf[lay["rs"]] = r @ s23
        buf[lay["ss"]] = s23 @ s23
        buf[lay["failed"]] = 1.0 if t == fail_at else 0.0
        if t == fail_at:
            fail_at = None                      # the failure happens once
        buf = allreduce(buf)
        if buf[lay["failed"]] != 0.0:           # every rank skips, then runs the iteration again
            continue
        t += 1
        r1 = buf[lay["rs"]] + mu * (np.abs(bx).sum() - np.abs(x).sum())
        r2 = buf[lay["ss"]]
        gamma = 0.0 if r2 == 0 else min(max(-r1 / r2, 0.0), 1.0)
        x = x + gamma * Dv
        Ax = Ax + gamma * s23
        r = Ax - b_loc
        g = g + gamma * buf[:w]
        bx, Dv = shrink(g, x)
    return x


def _row_solver_worker(rank, world, port, out):
    _init(rank, world, port)
    fx = dict(np.load(os.path.join(os.path.dirname(__file__), "golden", "c1_b1_p1_f32in.npz")))
    A = oracle.fixture_A(fx)
    s, e = D.row_bounds(A.shape[0], rank, world)
    args = (D.shard_rows(A, rank, world), fx["b"].reshape(-1)[s:e], float(fx["mu"]), 120)
    out[rank] = _row_rank_iterations(*args, refresh=50).tolist()
    # rank 1's launch of iteration 37 fails: both ranks skip it and run it again
    out[("failed", rank)] = _row_rank_iterations(*args, refresh=50, fail_at=37 if rank == 1 else None).tolist()
    dist.destroy_process_group()


def test_row_sharded_exchange_protocol_matches_reference():
    mgr = mp.Manager()
    out = mgr.dict()
    _spawn(_row_solver_worker, 2, out)
    fx = dict(np.load(os.path.join(os.path.dirname(__file__), "golden", "c1_b1_p1_f32in.npz")))
    A = oracle.fixture_A(fx)
    ref = oracle.run(A, fx["b"], float(fx["mu"]), 1, 120)["x"]
    np.testing.assert_array_equal(np.array(out[0]), np.array(out[1]))   # x replicated bit for bit
    assert np.linalg.norm(np.array(out[0]) - ref) <= 1e-9 * np.linalg.norm(ref)
    # a failure on one rank: the same iterates bit for bit, on both ranks
    np.testing.assert_array_equal(np.array(out[("failed", 0)]), np.array(out[0]))
    np.testing.assert_array_equal(np.array(out[("failed", 1)]), np.array(out[0]))


def test_xcd_symmetric_cu_masks():
    """distributed.xcd_symmetric_cu_mask: the ranks' masks are disjoint, cover
    the device, and give every XCD the same number of each rank's CUs whether the driver maps mask bit i
    to XCD i % 8 (interleaved) or to XCD i // 32 (runs) -- an XCD without CUs would never run its share of
    a persistent grid"""
    import pytest
    from convex_optimization_amd.distributed import xcd_symmetric_cu_mask
    cus = 256
    for nranks in (1, 2, 4, 8):
        masks = [xcd_symmetric_cu_mask(r, nranks, cus) for r in range(nranks)]
        bits = [{i for i in range(cus) if (m[i // 32] >> (i % 32)) & 1} for m in masks]
        assert set().union(*bits) == set(range(cus))
        assert sum(len(b) for b in bits) == cus                       # disjoint
        for b in bits:
            assert [sum(1 for i in b if i % 8 == x) for x in range(8)] == [32 // nranks] * 8
            assert [sum(1 for i in b if i // 32 == x) for x in range(8)] == [32 // nranks] * 8
    with pytest.raises(ValueError):
        xcd_symmetric_cu_mask(0, 3)
    with pytest.raises(ValueError):
        xcd_symmetric_cu_mask(0, 8, 128)
    with pytest.raises(ValueError):
        xcd_symmetric_cu_mask(2, 2)
