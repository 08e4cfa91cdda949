"""Worker of tests/test_rccl_ranks.py: one rank of a two-rank RCCL solve on ONE GPU.

Launched by torch.distributed.run (RANK / WORLD_SIZE / MASTER_* in the environment).  Both
ranks use device 0; each rank announces its own NCCL_HOSTID, so RCCL treats them as two hosts
and moves the all-reduce over loopback sockets (the same trick as tools/rehearse_n2.sh).  The
data path is the product's: libbpgl's communicator, the all-reduce issued on the solver stream.

usage: rccl_ranks_worker.py CASE SHARD OUTDIR   (SHARD: columns | rows)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    case, shard, outdir = sys.argv[1], sys.argv[2], sys.argv[3]
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
    fx = dict(np.load(os.path.join(ROOT, "tests", "golden", case + ".npz")))
    A = oracle.fixture_A(fx)
    block, iters = int(fx["BLOCK"]), int(fx["ITER_MAX"])
    eb = None if fx["err_bound"] < 0 else float(fx["err_bound"])
    b = np.asarray(fx["b"]).reshape(-1)
    GC = type("GC_float", (GPU_Calculation,), {"TYPE": "float"})
    comm = D.RankComm(rank, world)
    if shard == "rows":
        s, e = D.row_bounds(A.shape[0], rank, world)
        gc = GC(D.shard_rows(A, rank, world), 1, device=0, comm=comm, shard="rows")
        b_local = b[s:e]
    else:
        gc = GC(D.shard_columns(A, block, rank, world), block, device=0, comm=comm)
        b_local = b
    out = {}
    for graph in (True, False):
        res = gc.run(b_local, float(fx["mu"]), iters, err_bound=eb, record=True, use_graph=graph)
        tag = "graph" if graph else "eager"
        out[f"x_{tag}"] = np.asarray(res["x"]).reshape(-1)
        out[f"err_{tag}"] = np.asarray(res["err_iter"])
        out[f"t_last_{tag}"] = np.int64(res["t_last"])
        out[f"stopped_{tag}"] = np.bool_(res["stopped"])
    out["diag"] = np.asarray(gc.diag_ATA).reshape(-1)
    out["fallbacks"] = np.int64(gc.solver_stat("fallbacks"))
    np.savez(os.path.join(outdir, f"rank{rank}.npz"), **out)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
