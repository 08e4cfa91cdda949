#!/usr/bin/env python3
"""Long-horizon parity at a bench shape (configs[1], 8192 x 65536 fp32; configs[2]'s whole problem on
one GPU, 8192 x 524288 fp32; or configs[3], 1048576 x 4096 fp32 -- both 2^32 elements): the default one-pass solver (carried gradient g += gamma A^T (A D),
exact refresh every 256 iterations) and the two-pass solver on the GPU against the C oracle on
the same fp32 A, after ITERS iterations (default 2048 = 8 refreshes).  Prints one JSON line (and
a heartbeat while the oracle runs).

Usage (GPU box, repo root): python3 tools/longrun_parity.py [ITERS] [CONFIG 1|2|3] > gpurun_out/longrun.json
"""
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    cfg = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    m, n, seed = {1: (8192, 65536, 41), 2: (8192, 524288, 42), 3: (1048576, 4096, 43)}[cfg]
    import numpy as np
    import torch
    from convex_optimization_amd.parameters import device_instance
    from oracle import oracle
    oracle.build()

    def rel(a, b):
        return float(np.linalg.norm(np.asarray(a) - np.asarray(b)) / np.linalg.norm(np.asarray(b)))

    gc, b, mu, _ = device_instance(m, n, 0.4, 1, TYPE="float", seed=seed, device=0)
    one = gc.run(b, mu, iters, record=True)
    st = {k: gc.solver_stat(k) for k in ("onepass", "refreshes", "fallbacks")}
    gc.set_tuning("onepass", 0)
    two = gc.run(b, mu, iters, record=True)
    A = np.ascontiguousarray(gc.A_b_gpu[0].cpu().numpy())
    bh = b.cpu().numpy()
    torch.cuda.synchronize()
    stop = threading.Event()

    def beat():
        while not stop.wait(30):
            print(f"# oracle running ({iters} iterations)", file=sys.stderr, flush=True)
    threading.Thread(target=beat, daemon=True).start()
    t0 = time.time()
    ref = oracle.run(A, bh, mu, 1, iters, nthreads=min(16, os.cpu_count() or 1))
    stop.set()

    rows = max(1, (1 << 28) // n)   # 2 GiB of fp64 at a time

    def f(x):   # fp64 objective, A converted `rows` rows at a time
        x = np.asarray(x, dtype=np.float64)
        r = np.concatenate([A[i:i + rows].astype(np.float64) @ x for i in range(0, A.shape[0], rows)]) - bh
        return 0.5 * float(r @ r) + mu * float(np.abs(x).sum())
    f_ref = f(ref["x"])
    out = {"workload": f"configs[{cfg}] {m}x{n} fp32, seed {seed}", "iters": iters, "onepass_stats": st,
           "oracle_s": round(time.time() - t0, 1),
           "onepass_vs_oracle_x_rel_l2": rel(one["x"], ref["x"]), "twopass_vs_oracle_x_rel_l2": rel(two["x"], ref["x"]),
           "onepass_vs_twopass_x_rel_l2": rel(one["x"], two["x"]),
           "onepass_objective_rel": abs(f(one["x"]) - f_ref) / f_ref, "twopass_objective_rel": abs(f(two["x"]) - f_ref) / f_ref,
           "err_iter_last": {"onepass": float(one["err_iter"][iters - 1]), "twopass": float(two["err_iter"][iters - 1]),
                             "oracle": float(ref["err_iter"][iters - 1])},
           "bound": "north_star 1e-5 relative l2 on x"}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
