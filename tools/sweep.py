#!/usr/bin/env python3
"""Tuning sweep on one GPU: iterations/s (graph replay) and per-kernel times
(eager + HIP events) of the device solver for launch-geometry variants.

  python tools/sweep.py --m 8192 --n 65536 --targets 1024,2048,4096 --reverse 0,1
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=8192)
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--block", type=int, default=1)
    ap.add_argument("--type", default="float")
    ap.add_argument("--targets", default="2048")
    ap.add_argument("--reverse", default="0")
    ap.add_argument("--nt", default="1")
    ap.add_argument("--tails", default="120")
    ap.add_argument("--colmodes", default="0")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    import torch
    from convex_optimization_amd.parameters import device_instance
    torch.cuda.set_device(0)
    out = []
    for tb in [int(v) for v in a.targets.split(",")]:
        os.environ["BPGL_TARGET_BLOCKS"] = str(tb)
        gc, b, mu, _ = device_instance(a.m, a.n, 0.4, a.block, TYPE=a.type, seed=1, device=0)
        geo = gc.geometry()
        for rev, nt, tail, cm in [(int(r), int(n), int(t), int(c))
                                  for r in a.reverse.split(",") for n in a.nt.split(",")
                                  for t in a.tails.split(",") for c in a.colmodes.split(",")]:
            gc.set_tuning("col_mode", cm)
            gc.set_tuning("reverse_rows", rev)
            gc.set_tuning("nt_loads", nt)
            gc.set_tuning("tail_permille", tail)
            best = 0.0
            for _ in range(a.rounds):
                gc.solver_reset(b, mu, use_graph=True)
                gc.solver_step(10)
                gc.stream.synchronize()
                t0 = time.perf_counter()
                gc.solver_step(a.steps)
                gc.stream.synchronize()
                best = max(best, a.steps / (time.perf_counter() - t0))
            gc.solver_reset(b, mu, use_graph=False)
            gc.solver_step(5)
            gc.set_kernel_timing(True)
            gc.solver_step(a.steps // 2)
            kt, _ = gc.kernel_times()
            gc.set_kernel_timing(False)
            rec = dict(target=tb, reverse=rev, nt=nt, tail=tail, col_mode=cm, geometry=geo,
                       iters_per_s=best,
                       kernel_us={k: round(v * 1e3, 2) for k, v in kt.items()})
            print(json.dumps(rec), flush=True)
            out.append(rec)
        del gc
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
