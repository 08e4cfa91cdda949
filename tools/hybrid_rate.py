#!/usr/bin/env python3
"""PCIe-inclusive rate of the reference-style hybrid driver (lasso.ClassLasso: host vectors,
device GEMVs through GPU_Calculation's out-parameter calls, as lasso.py:173-292) beside the
device-resident loop (GPU_Calculation.run), same A and b, at configs[1]."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    import torch
    from convex_optimization_amd import lasso
    from convex_optimization_amd.parameters import device_instance
    m, n, iters = 8192, 65536, 40
    gc, b, mu, _ = device_instance(m, n, 0.4, 1, TYPE="float", seed=1, device=0)
    bh = b.cpu().numpy().reshape(-1, 1)
    d = gc.diag_ATA
    import types
    drv = lasso.ClassLasso(gc, d, types.SimpleNamespace(shape=(m, n)), bh, mu, 1, iters)
    drv.run(SILENCE=True)                     # warm
    t0 = time.perf_counter()
    drv.run(SILENCE=True)
    hyb = iters / (time.perf_counter() - t0)
    gc.solver_reset(b, mu)
    gc.solver_step(20)
    gc.stream.synchronize()
    t0 = time.perf_counter()
    gc.solver_step(200)
    gc.stream.synchronize()
    dev = 200 / (time.perf_counter() - t0)
    print(json.dumps({"m": m, "n": n, "hybrid_pcie_inclusive_iters_per_s": hyb, "device_loop_iters_per_s": dev}))


if __name__ == "__main__":
    main()
