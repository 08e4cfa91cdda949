"""One process, a CU-masked solver stream (diagnostic for tests/rccl_ranks_worker.py --cumask).

usage: python -X faulthandler tools/cumask_smoke.py [rows]
Step 1: the one-pass solver on half the CUs, no communicator.  Step 2 (arg "rows"): the same
with a one-rank RCCL communicator and row shards.  Prints the stats and the error against the
reference fixture after each step.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from convex_optimization_amd import distributed as D  # noqa: E402
from convex_optimization_amd.gpu_calculation import GPU_Calculation  # noqa: E402
from oracle import oracle  # noqa: E402


def main():
    torch.cuda.set_device(0)
    fx = dict(np.load(os.path.join(ROOT, "tests", "golden", "c1_b1_p1_f32in.npz")))
    A = oracle.fixture_A(fx)
    GC = type("GC_float", (GPU_Calculation,), {"TYPE": "float"})
    mask = D.xcd_symmetric_cu_mask(0, 2, torch.cuda.get_device_properties(0).multi_processor_count)
    print("mask", [hex(w) for w in mask[:2]], flush=True)
    steps = ["plain"] + (["rows"] if "rows" in sys.argv[1:] else [])
    for step in steps:
        print("step", step, flush=True)
        if step == "plain":
            gc = GC(A, 1, device=0, cu_mask=mask)
        else:
            import torch.distributed as dist
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29533")
            dist.init_process_group("gloo", rank=0, world_size=1)
            gc = GC(A, 1, device=0, comm=D.RankComm(0, 1), shard="rows", cu_mask=mask)
        print("created: cus", gc.solver_stat("cus"), "masked", gc.solver_stat("cu_masked"), "grid",
              gc.solver_stat("onepass_grid"), flush=True)
        res = gc.run(fx["b"], float(fx["mu"]), int(fx["ITER_MAX"]))
        e = np.linalg.norm(res["x"] - fx["x"].reshape(-1)) / np.linalg.norm(fx["x"])
        print(step, "onepass", gc.solver_stat("onepass"), "fallbacks", gc.solver_stat("fallbacks"),
              "rel", e, flush=True)
        del gc


if __name__ == "__main__":
    main()
