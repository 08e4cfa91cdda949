"""Worker of tests/test_rccl_ranks.py: one rank of a multi-rank RCCL solve on ONE GPU.

Launched by torch.distributed.run (RANK / WORLD_SIZE / MASTER_* in the environment).  Every
rank uses device 0; each rank announces its own NCCL_HOSTID, so RCCL treats them as separate
hosts and moves the all-reduce over loopback sockets (the same trick as tools/rehearse_n2.sh).
The data path is the product's: libbpgl's communicator, the all-reduce issued on the solver
stream.

usage: rccl_ranks_worker.py CASE SHARD OUTDIR [--cumask] [--fail-rank R --fail-at T] [--iters N]
                           [--exchange-fp32] [--chunk N] [--eager]
  CASE: a reference fixture of tests/golden, or longrun_<config> (a full-size long-horizon fixture,
        row shards only: see longrun())
  SHARD: columns | rows
  --cumask: the rank's solver stream gets a disjoint, XCD-symmetric 1/WORLD_SIZE of the CUs
            (distributed.xcd_symmetric_cu_mask), so each rank's persistent one-pass grid is
            sized to its CUs and stays resident beside the other ranks' kernels
  --fail-rank / --fail-at: in the first (graph) solve, rank R's one-pass launch of iteration T
            reports a hand-off failure (tuning key "onepass_fail_at"), exercising the collective
            recovery; the second (eager) solve runs undisturbed
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("case")
    ap.add_argument("shard")
    ap.add_argument("outdir")
    ap.add_argument("--cumask", action="store_true")
    ap.add_argument("--fail-rank", type=int, default=-1)
    ap.add_argument("--fail-at", type=int, default=-1)
    ap.add_argument("--iters", type=int, default=0, help="longrun: iterations (0: the fixture's own)")
    ap.add_argument("--exchange-fp32", action="store_true", help="longrun: the opt-in fp32 exchange (tuning -1)")
    ap.add_argument("--chunk", type=int, default=0, help="longrun: enqueue this many iterations at a time (0: all)")
    ap.add_argument("--eager", action="store_true", help="longrun: eager launches instead of hipGraph replay")
    a = ap.parse_args()
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    os.environ["NCCL_HOSTID"] = f"bpgl-test-rank{rank}"   # before the communicator is created
    os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    os.environ.setdefault("NCCL_IB_DISABLE", "1")
    import numpy as np
    import torch
    import torch.distributed as dist

    from convex_optimization_amd import distributed as D
    from convex_optimization_amd.gpu_calculation import GPU_Calculation
    from oracle import oracle

    dist.init_process_group("gloo")
    torch.cuda.set_device(0)
    fx = dict(np.load(os.path.join(ROOT, "tests", "golden", a.case + ".npz")))
    if a.case.startswith("longrun_"):
        return longrun(a, fx, rank, world, np, torch, dist, D, GPU_Calculation)
    A = oracle.fixture_A(fx)
    block, iters = int(fx["BLOCK"]), int(fx["ITER_MAX"])
    eb = None if fx["err_bound"] < 0 else float(fx["err_bound"])
    b = np.asarray(fx["b"]).reshape(-1)
    GC = type("GC_float", (GPU_Calculation,), {"TYPE": "float"})
    comm = D.RankComm(rank, world)
    mask = None
    if a.cumask:
        cus = torch.cuda.get_device_properties(0).multi_processor_count
        mask = D.xcd_symmetric_cu_mask(rank, world, cus)
    if a.shard == "rows":
        s, e = D.row_bounds(A.shape[0], rank, world)
        gc = GC(D.shard_rows(A, rank, world), 1, device=0, comm=comm, shard="rows", cu_mask=mask)
        b_local = b[s:e]
    else:
        gc = GC(D.shard_columns(A, block, rank, world), block, device=0, comm=comm, cu_mask=mask)
        b_local = b
    out = {"cus": np.int64(gc.solver_stat("cus")), "cu_masked": np.int64(gc.solver_stat("cu_masked")),
           "onepass_grid": np.int64(gc.solver_stat("onepass_grid"))}
    for graph in (True, False):
        if rank == a.fail_rank and a.fail_at >= 0:
            # the first (graph) solve only; cleared explicitly before the eager solve rather than
            # relying on the library's one-shot hook (round 3: the hook once fired in both solves)
            gc.set_tuning("onepass_fail_at", a.fail_at if graph else -1)
        # every rank's set-up is finished before any rank's solve starts (nothing else on the GPU)
        torch.cuda.synchronize()
        dist.barrier()
        order = fx["order"] if bool(fx["random_order"]) else None   # the reference's shuffled block order
        res = gc.run(b_local, float(fx["mu"]), iters, err_bound=eb, order=order, record=True, use_graph=graph)
        tag = "graph" if graph else "eager"
        out[f"x_{tag}"] = np.asarray(res["x"]).reshape(-1)
        out[f"err_{tag}"] = np.asarray(res["err_iter"])
        out[f"t_last_{tag}"] = np.int64(res["t_last"])
        out[f"stopped_{tag}"] = np.bool_(res["stopped"])
        out[f"fallbacks_{tag}"] = np.int64(gc.solver_stat("fallbacks"))
        out[f"onepass_{tag}"] = np.int64(gc.solver_stat("onepass"))
    out["diag"] = np.asarray(gc.diag_ATA).reshape(-1)
    out["fallbacks"] = out["fallbacks_eager"]
    np.savez(os.path.join(a.outdir, f"rank{rank}.npz"), **out)
    dist.barrier()
    dist.destroy_process_group()


def longrun(a, fx, rank, world, np, torch, dist, D, GPU_Calculation):
    """A full-size long-horizon fixture (tests/golden/longrun_*.npz: the C oracle's x after ITER
    iterations on the hash instance of tests/hash_instance.py) over WORLD_SIZE RCCL row ranks: each
    rank builds its own rows in HBM, proves them (the fixture's A samples in its rows; b's SHA-256
    over the gathered shards) and runs the whole horizon in graph replay."""
    import hashlib

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import hash_instance as H

    m, n, iters, mu = int(fx["m"]), int(fx["n"]), int(fx["iters"]), float(fx["mu"])
    iters = a.iters or iters
    s, e = D.row_bounds(m, rank, world)
    A = H.torch_A(e - s, n, "cuda:0", row0=s)
    rows, cols = fx["A_rows"], fx["A_cols"]
    mine = (rows >= s) & (rows < e)
    got = A[torch.from_numpy(rows[mine] - s).cuda(), torch.from_numpy(cols[mine]).cuda()].cpu().numpy()
    samples_ok = bool(np.array_equal(got, fx["A_samples"][mine]))
    b = H.torch_b(A, row0=s, m_total=m)
    parts = [None] * world
    dist.all_gather_object(parts, b.cpu().numpy())
    b_ok = hashlib.sha256(np.concatenate(parts).tobytes()).hexdigest() == str(fx["b_sha256"])
    GC = type("GC_float", (GPU_Calculation,), {"TYPE": "float"})
    mask = D.xcd_symmetric_cu_mask(rank, world, torch.cuda.get_device_properties(0).multi_processor_count) \
        if a.cumask else None
    gc = GC(A, 1, device=0, comm=D.RankComm(rank, world), shard="rows", cu_mask=mask)
    if a.exchange_fp32:
        gc.set_tuning("exchange_fp32", -1)
    torch.cuda.synchronize()
    dist.barrier()
    if a.chunk:
        # the solve enqueued `chunk` iterations at a time, the stream drained in between (see the world-8
        # case of test_rccl_row_shards_configs1_long_horizon_exchange)
        gc.solver_reset(b, mu, record_len=iters, use_graph=not a.eager)
        for k in range(0, iters, a.chunk):
            gc.solver_step(min(a.chunk, iters - k))
            gc.stream.synchronize()
        res = gc.solver_status()
        res["x"] = gc.solver_x()
        res["err_iter"], _ = gc.solver_records()
    else:
        res = gc.run(b, mu, iters, record=True, use_graph=not a.eager)
    out = {"x": np.asarray(res["x"]).reshape(-1), "err": np.asarray(res["err_iter"]),
           "iters": np.int64(res["iters"]), "samples_ok": np.bool_(samples_ok), "b_ok": np.bool_(b_ok),
           "in_place": np.bool_(gc._A_dev.data_ptr() == A.data_ptr()),
           "onepass": np.int64(gc.solver_stat("onepass")), "fallbacks": np.int64(gc.solver_stat("fallbacks")),
           "refreshes": np.int64(gc.solver_stat("refreshes")), "cus": np.int64(gc.solver_stat("cus"))}
    np.savez(os.path.join(a.outdir, f"rank{rank}.npz"), **out)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
