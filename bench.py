#!/usr/bin/env python3
"""Benchmark: ISTA (block best-response) iterations/s on dense fp32 A, 1..8 MI355X.

One "step" = one iteration of the hot path (reference lasso.py:102-157: the
shrink, s23 = A D, the exact line search, the x / Ax update and the next
gradient), all on the device, inputs resident in HBM before the timed region.
With one feature block (every default workload) the iteration streams A ONCE:
k_onepass forms s23 = A D and U = A^T s23 from one pass and the gradient is
carried as g += gamma U, with an exact g = A^T r every 256 iterations (folded
into the rate at its amortised cost, below); with several feature blocks, or
across column shards, it is the reference's two passes (A^T r, then A D).

  N = 1 : BASELINE configs[1]  m=8192 n=65536 fp32 A, one feature block.
  N > 1 : the metric's own unit on the metric's own matrix: iterations/s of the fixed
          8192 x 65536 fp32 problem split N ways (strong scaling, "scaling": "strong";
          speedup_vs_n1 = value / the N = 1 rate measured in the same run).  The split
          (--shard auto) follows the cost model of DESIGN.md section 6: one feature
          block -> rows (GPU g holds rows [g m/N, (g+1) m/N) of A, all columns,
          streams them once per iteration with k_onepass, and ONE RCCL all-reduce of
          n + 3 fp64 values per iteration carries U = A^T A D, the line-search dot
          products and the failure flag); several feature blocks -> columns (the
          reference's P-way split, cpu_calculation.py:23-27: two passes over A per
          iteration and one all-reduce of m + 2 + N fp64 on the residual side).
          Beside it, from the same run: "weak" (BASELINE configs[2]'s shape,
          m=8192 n=65536*N -- n = 524288 at N = 8 -- every GPU holding the 2 GiB of
          N = 1; unit block-iters/s = N x global iterations/s, with its own
          speedup_vs_n1), "columns" (the reference's column split of the same
          problem, and its weak form), each with its per-rank all-reduce times,
          "n1_same_run" (rank 0 alone on the N = 1 problem) and "rows_exchange_fp32"
          (the row split with the opt-in fp32 exchange).  --weak makes the weak
          problem the value line (the rounds 1-3 form).
  --config 2: configs[2]'s own problem (m=8192 n=524288) split over the N GPUs
          (strong scaling; at N = 1 the whole 16 GiB matrix on one GPU).
  --config 3 / 4: configs[3] (1048576 x 4096 fp32) / configs[4] (k = 128
          right-hand sides on bf16 A), one GPU.

Timing (every workload): W untimed warm-up iterations; an eager window of
max(K, 512) iterations (side legs: max(K, 128)) with HIP events around every kernel
on the solver stream (the per-kernel averages behind `roofline`, and the clock ramp
of a fresh box), lengthened on a one-pass leg until it contains an exact-gradient
refresh (a one-pass leg that timed none fails);
then `--windows` (default 5) windows of exactly K graph-replayed iterations, each
bracketed by a barrier and device synchronisation, max over ranks.  value and
ms_per_step come from the median window, with the one-pass exact-gradient refresh
(one A^T r pass every 256 iterations) folded in at its amortised rate: a window's
time minus the refreshes it happened to contain, plus K/256 refreshes, each at the
event-timed refresh cost.

N = 1 side legs (the same JSON line, each with its own ms_per_step, roofline and
kernel averages; a leg that fails records {"error": ...}): "config3" (configs[3],
1048576 x 4096 fp32), "config4" (configs[4], k = 128 right-hand sides on bf16 A,
the MFMA panel path) and "config2_one_gpu" (configs[2]'s whole 8192 x 524288
matrix on this one GPU).  --no-side-legs skips them.

Launch: python bench.py [--gpus N --steps K --warmup W].  For N > 1 under
torch.distributed.run (one process per GPU, RANK/LOCAL_RANK/WORLD_SIZE env) the
ranks run directly; without it (WORLD_SIZE unset) this process touches no GPU,
starts `python -m torch.distributed.run --nproc-per-node N bench.py <same args>`
as a child, relays its output and exits with its status.  Rank 0 prints one
JSON line.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

M, N_PER_GPU = 8192, 65536
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
METRIC = "ISTA iters/sec on dense A (8192×65536 fp32) at 1/2/4/8 MI355X; HBM-roofline %"


def alg_bytes_iter(m, w, sa=4, sv=8, k=1):
    """two passes over the active block + vector I/O."""
    return 2 * m * w * sa + sv * k * (5 * w + 5 * m)


def alg_bytes_iter_onepass(m, w, sa=4, sv=8):
    """The one-pass iteration (bpgl_onepass.h): the same vector I/O, A read once."""
    return m * w * sa + sv * (5 * w + 5 * m)


def alg_bytes_onepass(m, w, sa=4):
    """k_onepass per launch: read A_b (m x w) and D (w fp64), write s23 (m fp64) and
    U = A^T s23 (w fp64) once."""
    return m * w * sa + 8 * m + 16 * w


def alg_bytes_colpass(m, w, sa=4):
    """A^T s11 pass per launch (k_iter_a / k_colpass): read A_b (m x w) and s11
    (m fp64), produce g once (w fp64).  The shrink's x/D vector I/O is left out
    (conservative)."""
    return m * w * sa + 8 * m + 8 * w


def alg_bytes_rowpass(m, w, sa=4):
    """A D pass per launch (k_iter_b / k_rowpass): read A_b (m x w), D (w fp64),
    produce s23 once (m fp64)."""
    return m * w * sa + 8 * w + 8 * m


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=None, choices=[1, 2, 3, 4],
                    help="BASELINE.json configs[K]: 1 = 8192x65536 fp32 (default; weak scaling over N GPUs), "
                         "2 = 8192x524288 fp32 split over the N GPUs (strong), 3 = 1048576x4096 fp32, "
                         "4 = k=128 right-hand sides on bf16 A")
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=256,
                    help="iterations per timed window (default 256)")
    ap.add_argument("--warmup", type=int, default=200,
                    help="untimed iterations before the windows (default 200)")
    ap.add_argument("--ramp", type=int, default=512,
                    help="minimum length of the eager window with per-kernel events (default 512 iterations)")
    ap.add_argument("--windows", type=int, default=5,
                    help="timed windows of exactly --steps iterations; value uses the median (default 5)")
    ap.add_argument("--m", type=int, default=M)
    ap.add_argument("--n-per-gpu", type=int, default=N_PER_GPU)
    ap.add_argument("--block", type=int, default=1)
    ap.add_argument("--type", default="float", choices=["float", "double", "bf16"])
    ap.add_argument("--no-strong", action="store_true", help="skip the side legs of an N > 1 run")
    ap.add_argument("--weak", action="store_true",
                    help="N > 1: value = weak scaling (m=8192, n=65536 N, block-iters/s) instead of the default "
                         "strong scaling of the metric's 8192 x 65536 matrix")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline")
    ap.add_argument("--no-side-legs", action="store_true",
                    help="N = 1: skip the config3 / config4 / config2_one_gpu legs of the default line")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--seed", type=int, default=20190325)
    ap.add_argument("--onepass", type=int, default=-1, choices=[-1, 0, 1],
                    help="one pass over A per iteration: -1 (default) when eligible (1 block, 1 rank), 0 off, 1 required")
    ap.add_argument("--tail-row-blocks", type=int, default=-1, choices=[-1, 0, 1],
                    help="one-pass tail: residual update on blocks of its own (1, library default) or first in every block (0)")
    ap.add_argument("--graph-max", type=int, default=-1,
                    help="largest hipGraph of iterations replayed (power of two; -1: library default, 64)")
    ap.add_argument("--onepass-cache", type=int, default=-1,
                    help="permille of each one-pass row group read with cache-allocating loads (-1: library default)")
    ap.add_argument("--onepass-rows", type=int, default=-1, choices=[-1, 0, 1],
                    help="one-pass row groups: 1 interleaved rows, 0 consecutive (-1: library default)")
    ap.add_argument("--onepass-sb1", type=int, default=-1, choices=[-1, 0],
                    help="one segment block per row: the LDS-only row hand-off (-1: library default, on) or off (0)")
    ap.add_argument("--comm", action="store_true",
                    help="attach an RCCL communicator even at N = 1 (runs the sharded/all-reduce leg)")
    ap.add_argument("--shard", default="auto", choices=["auto", "rows", "columns"],
                    help="multi-GPU split (N > 1, or N = 1 with --comm): auto (default: rows for one feature block, "
                         "columns for several -- the cost model of DESIGN.md section 6), rows (one pass over A, "
                         "all-reduce of n + 3) or columns (the reference's split; two passes, all-reduce of m + 2 + N)")
    ap.add_argument("--exchange-fp32", type=int, default=0, choices=[0, 1],
                    help="RCCL row shards: the per-iteration all-reduce of [U | r.s23 | s23.s23 | failed] in fp32 "
                         "(1, opt-in: half the bytes, x within ~1e-6 of the fp64 exchange) or fp64 (0, default)")
    ap.add_argument("--rhs", type=int, default=1,
                    help="k > 1: configs[4] panel path (k right-hand sides, bf16 A, MFMA), 1 GPU")
    ap.add_argument("--kchunks", type=int, default=0, help="panel path split-K chunks (0 = auto)")
    ap.add_argument("--interleave", type=int, default=-1,
                    help="panel path mainloop variant 0/1/2 for both passes (-1: library defaults)")
    ap.add_argument("--interleave1", type=int, default=-1, help="panel path pass-1 mainloop variant (-1: default)")
    ap.add_argument("--interleave2", type=int, default=-1, help="panel path pass-2 mainloop variant (-1: default)")
    ap.add_argument("--d-split", type=int, default=-1, choices=[-1, 1, 2],
                    help="panel path: the direction enters the A D pass as a hi + lo bf16 pair (2) or as its "
                         "bf16 rounding (1); -1: library default")
    ap.add_argument("--carry-g", type=int, default=-1, choices=[-1, 0, 1],
                    help="panel path, one block: carry G += gamma A^T S (one bf16 product in pass 1) between exact "
                         "hi+lo gradients (1); -1: library default")
    ap.add_argument("--g-refresh", type=int, default=-1,
                    help="panel path with carry_g: exact gradient period (multiple of 8); -1: library default")
    ap.add_argument("--fuse-update", type=int, default=-1, choices=[-1, 0, 1],
                    help="panel path, one block with x deferred: reduce + line search + residual update in one "
                         "launch (1) or two (0); -1: library default")
    ap.add_argument("--fuse-grid", type=int, default=-1, choices=[-1, 256, 512, 1024],
                    help="panel path: blocks of the fused reduce + update launch (-1: library default)")
    ap.add_argument("--defer-x", type=int, default=-1, choices=[-1, 0, 1],
                    help="panel path, one block: apply x += gamma D in the next pass-1 epilogue (1) or in the "
                         "update kernel (0); -1: library default")
    a = ap.parse_args()
    a.strong_total = False
    if a.config == 2:
        world = int(os.environ.get("WORLD_SIZE", str(a.gpus)))
        a.m, a.strong_total = 8192, True
        if 524288 % world:
            raise SystemExit("--config 2 splits n = 524288 over the GPUs: N must divide it")
        a.n_per_gpu = 524288 // world
    elif a.config == 3:
        a.m, a.n_per_gpu = 1048576, 4096
        a.steps, a.warmup = min(a.steps, 30), min(a.warmup, 40)   # 2.7 ms per iteration
    elif a.config == 4:
        a.rhs = 128
    if a.shard == "auto":
        a.shard = "rows" if a.block == 1 else "columns"
    a.windows = max(1, a.windows)
    return a


def main_shape(args, G):
    """(n_total, scaling) of the value line: N = 1 -> the configured matrix ("none"); N > 1 -> the
    metric's named 8192 x 65536 matrix split N ways ("strong"), configs[2]'s own matrix split N ways
    with --config 2 ("strong"), or the weak problem m x 65536 N with --weak ("weak")"""
    if G == 1:
        return args.n_per_gpu, "none"
    if args.strong_total:
        return args.n_per_gpu * G, "strong"
    if args.weak:
        return args.n_per_gpu * G, "weak"
    return args.n_per_gpu, "strong"


def workload_label(args, G, m, n_total, ml, w, rows):
    """configs[K] label from the actual shape (BASELINE.json configs)."""
    if args.config == 2 or (m, n_total) == (8192, 524288):
        name = "configs[2]"
    elif args.config == 3 or (m, n_total) == (1048576, 4096):
        name = "configs[3]"
    elif (m, n_total) == (8192, 65536) and G == 1:
        name = "configs[1]"
    elif (m, n_total) == (8192, 65536):
        name = f"configs[1] matrix (the metric's 8192x65536) split {G} ways, strong scaling"
    elif m == 8192 and n_total == 65536 * G:
        name = "configs[2]-style weak scaling"
    else:
        name = "custom"
    s = f"{name}: m={m} n={n_total} {args.type} A, {args.block} feature block(s), {G} GPU(s)"
    if G > 1:
        s += (f", row-sharded {ml} rows/GPU, one RCCL all-reduce of n+3 fp64 per iteration" if rows else
              f", column-sharded {w} cols/GPU, one RCCL all-reduce of m+2+N fp64 per iteration")
    return s


class Ctx:
    def __init__(self, world):
        import torch
        import torch.distributed as dist
        self.rank = int(os.environ.get("RANK", "0"))
        self.world = int(os.environ.get("WORLD_SIZE", str(world)))
        self.local = int(os.environ.get("LOCAL_RANK", str(self.rank)))
        # rehearsal of the N > 1 code path on a one-GPU box (every rank on this device;
        # numbers meaningless): BPGL_BENCH_DEVICE=0.  RCCL refuses two ranks of one node on
        # one GPU, so each rank claims its own host id and the ranks talk over loopback sockets.
        # BPGL_BENCH_CU_PARTITION=1 with it: every rank's solver stream gets a disjoint,
        # XCD-symmetric 1/N of the CUs (distributed.xcd_symmetric_cu_mask), so each rank's
        # persistent one-pass grid is sized to its CUs and the default N > 1 path runs as
        # designed (the ranks still share one GPU's HBM: rates are not N-GPU rates).
        self.cu_mask = None
        if os.environ.get("BPGL_BENCH_DEVICE"):
            self.local = int(os.environ["BPGL_BENCH_DEVICE"])
            os.environ["NCCL_HOSTID"] = f"bpgl-rehearsal-{self.rank}"
            os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
            os.environ.setdefault("NCCL_IB_DISABLE", "1")
            if os.environ.get("BPGL_BENCH_CU_PARTITION") == "1" and self.world > 1:
                from convex_optimization_amd.distributed import xcd_symmetric_cu_mask
                cus = torch.cuda.get_device_properties(self.local).multi_processor_count
                self.cu_mask = xcd_symmetric_cu_mask(self.rank, self.world, cus)
        self.dist = dist
        if self.world > 1:
            dist.init_process_group("gloo")
        torch.cuda.set_device(self.local)

    def barrier(self):
        if self.world > 1:
            self.dist.barrier()

    def max(self, v):
        if self.world == 1:
            return v
        import torch
        t = torch.tensor([float(v)], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t[0])

    def gather(self, v):
        """every rank's float, in rank order (gloo)"""
        if self.world == 1:
            return [float(v)]
        import torch
        out = [torch.zeros(1, dtype=torch.float64) for _ in range(self.world)]
        self.dist.all_gather(out, torch.tensor([float(v)], dtype=torch.float64))
        return [float(t[0]) for t in out]


def build_problem(ctx, m, n_total, block, type_name, seed, force_comm=False, shard="rows"):
    import torch
    from convex_optimization_amd.distributed import RankComm, row_bounds, shard_bounds
    from convex_optimization_amd.parameters import device_instance
    comm = RankComm(ctx.rank, ctx.world) if (ctx.world > 1 or force_comm) else None
    col_range = row_range = None
    if comm is not None and shard == "rows":
        row_range = row_bounds(m, ctx.rank, ctx.world)
    elif ctx.world > 1:
        bounds = shard_bounds(n_total, block, ctx.rank, ctx.world)
        idx = torch.cat([torch.arange(s, e) for s, e in bounds]).to(f"cuda:{ctx.local}")
        col_range = idx
    gc, b, mu, _ = device_instance(m, n_total, 0.4, block, TYPE=type_name, seed=seed, device=ctx.local,
                                   comm=comm, col_range=col_range, row_range=row_range, cu_mask=ctx.cu_mask)
    torch.cuda.synchronize()
    return gc, b, mu


_T0 = time.time()


def progress(msg):
    """one line on stderr (rank 0): the phases of a long multi-leg run stay visible"""
    if int(os.environ.get("RANK", "0")) == 0:
        sys.stderr.write(f"# bench {time.time() - _T0:7.1f} s: {msg}\n")
        sys.stderr.flush()


def timed_window(ctx, sync, step, steps):
    """barrier + sync, exactly `steps` iterations, sync + barrier; max-over-ranks seconds."""
    ctx.barrier()
    sync()
    t0 = time.perf_counter()
    step(steps)
    sync()
    t1 = time.perf_counter()
    ctx.barrier()
    return ctx.max(t1 - t0)


class MeasureError(RuntimeError):
    """every timed window of a measurement was invalid (an Exception, so a side leg records it and
    every rank still reaches the closing barrier and rank 0 prints the line)"""


def median(v):
    v = sorted(v)
    k = len(v)
    return v[k // 2] if k % 2 else 0.5 * (v[k // 2 - 1] + v[k // 2])


def eager_window_len(steps, ramp, warmup, period, onepass):
    """iterations of the eager window: max(K, ramp), lengthened on a one-pass leg so that it
    contains an exact-gradient refresh (the refresh runs before iteration t when t is a positive
    multiple of `period`; the window covers iterations [warmup, warmup + n)), whose event-timed
    cost is folded into every window's rate"""
    n = max(steps, ramp)
    if onepass and period > 0:
        first = max(period, -(-warmup // period) * period)
        n = max(n, first - warmup + 1)
    return n


def measure(ctx, args, m, n_total):
    """W warm-up iterations, an eager window with per-kernel HIP events (max(K, 512) iterations),
    then `windows` graph windows of exactly K iterations (see the module docstring).  A window is
    valid when it ran the iteration the solve started with (one pass or two) and lost no
    iterations; if a one-pass launch failed before the windows (every window then runs on the
    two-pass kernels), the solver is reset and the whole sequence measured once more."""
    import torch
    progress(f"measure m={m} n={n_total} shard={args.shard} exchange_fp32={args.exchange_fp32}: building the instance")
    gc, b, mu = build_problem(ctx, m, n_total, args.block, args.type, args.seed, args.comm, args.shard)
    gc.set_tuning("onepass", args.onepass)
    if args.exchange_fp32:
        gc.set_tuning("exchange_fp32", -1)
    if args.tail_row_blocks >= 0:
        gc.set_tuning("tail_row_blocks", args.tail_row_blocks)
    if args.onepass_cache >= 0:
        gc.set_tuning("onepass_cache_permille", args.onepass_cache)
    if args.onepass_rows >= 0:
        gc.set_tuning("onepass_rows", args.onepass_rows)
    if args.onepass_sb1 >= 0:
        gc.set_tuning("onepass_sb1", args.onepass_sb1)
    if args.graph_max > 0:
        gc.set_tuning("graph_max", args.graph_max)

    def sync():
        gc.stream.synchronize()
        torch.cuda.synchronize()

    for attempt in range(2):
        progress(f"  attempt {attempt}: reset, {args.warmup} warm-up iterations")
        gc.solver_reset(b, mu, use_graph=True)
        op0 = gc.solver_stat("onepass")
        gc.solver_step(args.warmup)
        sync()
        # eager window: kernel averages (events on the solver stream) + clock ramp, and on a
        # one-pass leg at least one exact-gradient refresh
        n_ev = eager_window_len(args.steps, args.ramp, args.warmup, gc.solver_stat("refresh_period"), op0)
        progress(f"  eager window of {n_ev} iterations with kernel events")
        gc.set_kernel_timing(True)
        r0 = gc.solver_stat("refreshes")
        el_ev = timed_window(ctx, sync, gc.solver_step, n_ev)
        n_ref_ev = gc.solver_stat("refreshes") - r0
        times, samples = gc.kernel_times()
        gc.set_kernel_timing(False)
        refresh_ms = times["refresh"] * samples / n_ref_ev if n_ref_ev else 0.0
        refresh_ms = ctx.max(refresh_ms)
        st = gc.solver_status()   # completes any iteration a failed one-pass launch lost (outside the windows)
        eager_op = int(min(ctx.gather(gc.solver_stat("onepass"))))
        period = gc.solver_stat("refresh_period")
        if eager_op and period and not refresh_ms > 0.0:
            raise MeasureError(f"one-pass leg timed no exact-gradient refresh in its eager window "
                               f"({n_ev} iterations from {args.warmup}, period {period}): its rate would leave "
                               f"the refresh out")
        # graph windows; after each, the status call (outside the window) re-runs iterations a
        # failed one-pass launch lost -- such a window did not do its K iterations, and a window
        # after a fallback runs the two-pass kernels: neither counts toward the median
        wins = []
        progress(f"  {args.windows} graph windows of {args.steps} iterations")
        for _ in range(args.windows):
            r0 = gc.solver_stat("refreshes")
            rec0 = gc.solver_stat("fallbacks")
            el = timed_window(ctx, sync, gc.solver_step, args.steps)
            n_ref = ctx.max(gc.solver_stat("refreshes") - r0)
            st = gc.solver_status()
            lost = ctx.max(gc.solver_stat("fallbacks") - rec0) > 0
            op = int(min(ctx.gather(gc.solver_stat("onepass"))))
            adj = el - n_ref * refresh_ms * 1e-3 + (args.steps / period * refresh_ms * 1e-3 if period and op else 0.0)
            wins.append({"s": el, "refreshes": int(n_ref), "s_amortised": adj, "lost_iterations": bool(lost),
                         "onepass": op, "valid": (not lost) and op == op0})
        if any(w["valid"] for w in wins) and eager_op == op0:
            break
        if attempt == 1:
            raise MeasureError("every timed window lost one-pass iterations or fell back to two passes "
                               "(another process holds CUs?)")
    assert st["iters"] == args.warmup + n_ev + args.windows * args.steps or st["stopped"], st
    return dict(gc=gc, windows=wins, el_events=el_ev, n_events=n_ev, kernel_ms=times, samples=samples, status=st,
                refresh_ms=refresh_ms, refresh_period=period, w_local=gc.MAT_WIDTH, m_local=gc.MAT_HEIGHT,
                b=b, mu=mu, fallbacks=gc.solver_stat("fallbacks"), onepass=gc.solver_stat("onepass"),
                attempts=attempt + 1, cus=gc.solver_stat("cus"), onepass_rows=gc.solver_stat("onepass_rows"))


def window_rate(res, K):
    """iterations/s of the median valid window (the refresh folded in), and that window's raw time"""
    ok = [x for x in res["windows"] if x["valid"]]
    return K / median([x["s_amortised"] for x in ok]), median([x["s"] for x in ok]) / K


class SoloCtx:
    """rank 0 alone (no collectives): the N = 1 reference leg inside an N > 1 run"""

    def __init__(self, ctx):
        self.rank, self.world, self.local, self.cu_mask, self.dist = 0, 1, ctx.local, None, None

    def barrier(self):
        pass

    def max(self, v):
        return v

    def gather(self, v):
        return [float(v)]


def leg_summary(ctx, res, K, G, weak):
    """a secondary measurement of an N > 1 run (its own key in the JSON line)"""
    v, raw = window_rate(res, K)
    kms = res["kernel_ms"]
    return {"value": v * G if weak else v,
            "unit": "block-iters/s" if weak else "iters/s",
            "scaling": ("weak" if weak else "strong") if G > 1 else "none",
            "ms_per_step": 1e3 / v,
            "ms_per_step_raw_median": raw * 1e3,
            "config": f"{res['m_local']} rows x {res['w_local']} cols per GPU",
            "split": res["gc"].shard if G > 1 else "none",
            "iteration": "one pass over A" if kms.get("onepass", 0.0) > 0 else "two passes over A",
            "kernel_avg_ms": kms,
            "allreduce_ms_per_rank": ctx.gather(kms.get("allreduce", 0.0)),
            "onepass_fallbacks": res["fallbacks"], "cus_per_rank": res["cus"]}


def host_cores():
    """CPUs this process may use: the affinity mask, capped by a cgroup CPU quota and by
    OMP_NUM_THREADS when set (the GPU boxes give each job a share of a large host; os.cpu_count()
    counts the whole host).  Returns (threads, description)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, -(-int(q) // int(per)))
    except Exception:
        pass
    omp = os.environ.get("OMP_NUM_THREADS")
    n = aff
    if quota:
        n = min(n, quota)
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except Exception:
        pass
    return n, {"threads": n, "os_cpu_count": os.cpu_count(), "affinity": aff, "cgroup_quota_cpus": quota,
               "OMP_NUM_THREADS": omp, "model": model}


def cpu_pool_leg(cores):
    """The reference's own Pool-parallel CPU loop at configs[0] (oracle/pool_baseline.py).  Run
    before this process touches the GPU: the pool forks."""
    try:
        from oracle.pool_baseline import pool_baseline
        return pool_baseline(cores)
    except Exception as e:  # a reported baseline, never a reason to lose the GPU line
        return {"error": repr(e)}


def cpu_baseline(gc, b, mu, seconds, cores, cpu_info, share_note=""):
    """The oracle (C restatement of the reference iteration) on this host's cores,
    bounded sample of the same workload: the same A (copied back to host fp32),
    as many iterations as fit in about `seconds` of CPU time."""
    import numpy as np
    from oracle import oracle
    oracle.build()
    H, W = gc.MAT_HEIGHT, gc.MAT_WIDTH
    A = gc.A_b_gpu.permute(1, 0, 2).reshape(H, gc.Block * W).cpu().numpy()
    A = np.ascontiguousarray(A)
    bh = b.cpu().numpy()
    threads = cores
    t0 = time.perf_counter()
    oracle.run(A, bh, mu, gc.Block, 2, nthreads=threads)
    per = (time.perf_counter() - t0) / 2
    iters = int(max(3, min(200, seconds / max(per, 1e-6))))
    t0 = time.perf_counter()
    oracle.run(A, bh, mu, gc.Block, iters, nthreads=threads)
    el = time.perf_counter() - t0
    c_oracle = {"value": iters / el, "unit": "iters/s", "threads": threads,
                "sample": f"oracle/bpgl_oracle.c oracle_run, {iters} iterations from x=0 on the same "
                          f"{H}x{gc.Block * W} fp32 A and b{share_note}, {threads} OpenMP threads (fp64 arithmetic)"}
    out = {"host": cpu_info, "c_oracle": c_oracle}
    # SURVEY 8d also asks for the numpy restatement (OpenBLAS GEMVs, fp64) beside it: a few
    # iterations, bounded to about a third of the C sample's time
    # iterations only: diag(A^T A) (the set-up, as the reference excludes it: lasso.py:98) is
    # computed before the timed calls
    def numpy_rate(Ain, budget, **kw):
        oracle.run_numpy(Ain, bh, mu, gc.Block, 1, dg=dg, **kw)   # warm (first-touch of the operands)
        t0 = time.perf_counter()
        oracle.run_numpy(Ain, bh, mu, gc.Block, 2, dg=dg, **kw)
        per = (time.perf_counter() - t0) / 2
        n = int(max(2, min(100, budget / max(per, 1e-6))))
        t0 = time.perf_counter()
        oracle.run_numpy(Ain, bh, mu, gc.Block, n, dg=dg, **kw)
        return n / (time.perf_counter() - t0), n
    A64 = A.astype(np.float64)
    dg = np.square(A64).sum(axis=0)
    # three samples (the rate moves 12-40 it/s between boxes and runs on a shared host): the
    # median is the value, the three are reported as its range
    runs = [numpy_rate(A64, seconds / 9) for _ in range(3)]
    rates = sorted(r[0] for r in runs)
    v, n_np = rates[1], runs[0][1]
    out["numpy_fp64"] = {"value": v, "unit": "iters/s", "samples": [r[0] for r in runs],
                         "range": [rates[0], rates[2]],
                         "threads": "OpenBLAS default (OMP_NUM_THREADS=" + os.environ.get("OMP_NUM_THREADS", "unset") + ")",
                         "sample": f"oracle.run_numpy, median of 3 samples of {n_np} iterations from x=0 on the same A "
                                   "(as fp64), set-up excluded"}
    # the reported baseline: the reference's own CPU arithmetic (cpu_calculation.py's numpy GEMVs at
    # its default TYPE double, lasso.py:102-157) restated, on this job's cores -- the fastest of the
    # fp64 CPU paths timed here; the C oracle and the fp32-storage variant stay beside it
    out.update({"value": v, "unit": "iters/s", "cores": threads, "kind": "port", "range": [rates[0], rates[2]],
                "sample": f"oracle.run_numpy (the reference iteration in numpy, fp64 OpenBLAS GEMVs), median of 3 "
                          f"samples of {n_np} iterations from x=0 on the same {H}x{gc.Block * W} A and b{share_note}, "
                          f"set-up (diag) excluded, OpenBLAS on {threads} threads"})
    # and the fp32-storage variant (the reference's TYPE='float' CPU path: sgemv on fp32 A, fp64 elsewhere)
    del A64
    v, n_np = numpy_rate(A, seconds / 3, gemv_f32=True)
    out["numpy_fp32_storage"] = {"value": v, "unit": "iters/s", "threads": out["numpy_fp64"]["threads"],
                                 "sample": f"oracle.run_numpy(gemv_f32=True), {n_np} iterations from x=0 on the "
                                           "same fp32 A (fp32 GEMVs, fp64 vectors), set-up excluded"}
    return out


def vendor_yardstick(gc, reps=20):
    """Speed yardstick only (the reference's cuBLAS classes):
    PyTorch's ROCm GEMV (rocBLAS/hipBLASLt, fp32 accumulation) for the same two
    passes, A^T r and A d, on the same resident fp32 A.  Not parity-equivalent
    (fp32 accumulation); reported beside the solver, never as `value`."""
    import torch
    A = gc._A_dev
    if A.dim() != 2 or A.dtype != torch.float32:
        return None
    H, K = A.shape
    r = torch.randn(H, device=A.device)
    d = torch.randn(K, device=A.device)
    for _ in range(3):
        torch.mv(A.t(), r)
        torch.mv(A, d)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        torch.mv(A.t(), r)
    e1.record()
    torch.cuda.synchronize()
    t_mtv = e0.elapsed_time(e1) / reps
    e0.record()
    for _ in range(reps):
        torch.mv(A, d)
    e1.record()
    torch.cuda.synchronize()
    t_mv = e0.elapsed_time(e1) / reps
    return {"what": "torch.mv (rocBLAS/hipBLASLt) fp32 GEMV pair on the same A, fp32 accumulation",
            "mtv_ms": t_mtv, "mv_ms": t_mv,
            "mtv_GBps": H * K * 4 / t_mtv / 1e6, "mv_GBps": H * K * 4 / t_mv / 1e6}


def vendor_iteration_yardstick(gc, b, mu, iters=20):
    """The whole iteration on rocBLAS GEMVs (yardstick.VendorLasso): fp32
    GEMVs on the same resident A, fp64 elementwise; iterations/s, eager torch launches."""
    import torch
    from convex_optimization_amd.yardstick import VendorLasso
    A = gc._A_dev
    if A.dim() != 2 or A.dtype != torch.float32 or gc.Block != 1:
        return None
    v = VendorLasso.__new__(VendorLasso)
    v.Block, v.H, v.W, v.dtype, v.device = 1, A.shape[0], A.shape[1], torch.float32, A.device
    v.A_b = A.unsqueeze(0)                       # a view: no copy of A
    v.diag = (A.double() ** 2).sum(dim=0).unsqueeze(0) if A.numel() < (1 << 28) else \
        torch.stack([(A[:, j:j + 4096].double() ** 2).sum(dim=0) for j in range(0, A.shape[1], 4096)]).reshape(1, -1)
    v.rec = 1.0 / v.diag
    v.reset(b, mu)
    v.step(3)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    v.step(iters)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    return {"what": "yardstick.VendorLasso: the iteration with torch.mv (rocBLAS/hipBLASLt) fp32 GEMVs + torch "
                    "elementwise, fp64 vectors, eager launches", "iters_per_s": iters / el, "iters": iters}


def pmc_traffic(workload_key, kernel):
    """HBM bytes per launch of `kernel` from the committed PMC summary
    (profiles/pmc_traffic.json, written by tools/pmc_traffic.py), or None."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        return float(json.load(open(path))[workload_key][kernel]["hbm_bytes"])
    except Exception:
        return None


MFMA_BF16_DENSE_TFLOPS = 2500.0   # MI355X dense bf16 MFMA (MI355X_MICROARCH.md; no sparsity)


def mfma_counters(kernel, k):
    """MFMA utilisation of a panel pass from rocprofv3 counters (profiles/mfma_util.json, written by
    tools/mfma_util.py from tools/panel_mfma_pmc.sh): SQ_VALU_MFMA_BUSY_CYCLES over SIMDs x kernel
    cycles (GRBM_GUI_ACTIVE / 8), at the clock the chip ran and at the 2.4 GHz peak clock, or None"""
    try:
        e = json.load(open(os.path.join(ROOT, "profiles", "mfma_util.json")))[f"{kernel}_k{k}"]
    except Exception:
        return None
    return {"busy_cycles_per_launch": e["busy_cycles"], "mfma_instructions": e["mfma_instructions"],
            "busy_frac_at_running_clock": e["busy_frac_at_running_clock"],
            "busy_frac_at_peak_clock": e.get("busy_frac_at_peak_clock"),
            "running_clock_hz_est": e.get("running_clock_hz_est"),
            "source": "profiles/mfma_util.json (rocprofv3 SQ_VALU_MFMA_BUSY_CYCLES, SQ_INSTS_VALU_MFMA_BF16, "
                      "GRBM_GUI_ACTIVE; tools/panel_mfma_pmc.sh)"}


LDS_FILL_CAP_GBS = 9600.0   # best LDS-DMA fill rate measured on a panel pass, summed over CUs


def panel_bytes_pass(m, w, k):
    """One MFMA pass of the panel path: A_b in bf16 (m x w) once, the k-wide
    operand panel in (hi+lo bf16) and the fp32 split-K output once."""
    return 2 * m * w + 4 * k * (m + w) + 4 * k * (m + w)


def panel_fill_bytes(m, w, k, which, d_split=2, r_pieces=2):
    """Bytes through the CUs' LDS-DMA path per launch of panel pass `which` (1 or 2): every block
    streams its A tile and the k-wide operand over its K range -- pass 1: w/256 blocks, each the
    residual's hi + lo bf16 pieces over all m rows (r_pieces 2; with the carried gradient the bf16 S
    alone, 1 + 2 / g_refresh on average); pass 2: m/256 row blocks x the column chunks,
    together the direction's d_split pieces over all w columns once per row block."""
    if which == 1:
        return 2 * m * w + int((w // 256) * r_pieces * 2 * k * m)
    return 2 * m * w + (m // 256) * d_split * 2 * k * w


def main_panel(args):
    emit(measure_panel(args))


def measure_panel(args):
    """configs[4]: k right-hand sides on m x n bf16 A (PanelLasso, MFMA passes); the JSON line."""
    import torch
    from convex_optimization_amd.panel import PanelLasso
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        raise SystemExit("--rhs > 1 runs on one GPU (replicas only)")
    torch.cuda.set_device(0)
    m, n, k = args.m, args.n_per_gpu, args.rhs
    g = torch.Generator(device="cuda").manual_seed(args.seed)
    A = torch.randn(m, n, device="cuda", generator=g)
    A /= A.norm(dim=1, keepdim=True)
    Xt = torch.randn(n, k, device="cuda", generator=g) * (torch.rand(n, k, device="cuda", generator=g) < 0.4)
    pl = PanelLasso(A, args.block, nrhs=k, device=0, kchunks=args.kchunks)
    if args.interleave >= 0:
        pl.set_tuning("interleave", args.interleave)
    for q in (1, 2):
        if getattr(args, f"interleave{q}") >= 0:
            pl.set_tuning(f"interleave{q}", getattr(args, f"interleave{q}"))
    if args.d_split > 0:
        pl.set_tuning("d_split", args.d_split)
    if args.defer_x >= 0:
        pl.set_tuning("defer_x", args.defer_x)
    if args.fuse_update >= 0:
        pl.set_tuning("fuse_update", args.fuse_update)
    if args.fuse_grid > 0:
        pl.set_tuning("fuse_grid", args.fuse_grid)
    if args.carry_g >= 0:
        pl.set_tuning("carry_g", args.carry_g)
    if args.g_refresh >= 0:
        pl.set_tuning("g_refresh", args.g_refresh)
    d_split = pl.get_tuning("d_split")
    carry, g_period = pl.get_tuning("carry_g"), pl.get_tuning("g_refresh")
    del A
    Ab = pl.A_bf16.float()
    B = (Ab @ Xt + 0.01 * torch.randn(m, k, device="cuda", generator=g)).double()
    mu = (0.1 * (Ab.t() @ B.float()).abs().amax(dim=0)).double().cpu().numpy()
    del Ab
    torch.cuda.synchronize()

    def sync():
        pl.stream.synchronize()
        torch.cuda.synchronize()

    ctx = Ctx(1)
    pl.solver_reset(B, mu, use_graph=True)
    pl.solver_step(args.warmup)
    sync()
    n_ev = max(args.steps, args.ramp)          # eager window: kernel averages + clock ramp
    pl.set_kernel_timing(True)
    el_ev = timed_window(ctx, sync, pl.solver_step, n_ev)
    kms, samples = pl.kernel_times()
    pl.set_kernel_timing(False)
    wins = [timed_window(ctx, sync, pl.solver_step, args.steps) for _ in range(args.windows)]
    st = pl.solver_status()
    el_graph = median(wins)
    w = pl.MAT_WIDTH
    dom = max(("pass1_mfma", "pass2_mfma"), key=lambda q: kms[q])
    pb = panel_bytes_pass(m, w, k)
    achieved = pb / (kms[dom] * 1e-3) / 1e9
    # MFMA work of the dominant pass: the residual always enters as hi + lo, the direction
    # as hi + lo (d_split 2) or hi alone (d_split 1); with carry_g pass 1 runs the bf16 S product and,
    # every g_refresh iterations, the hi + lo residual products
    p1_products = (1 + 2 / g_period) if carry else 2
    fill_bytes = panel_fill_bytes(m, w, k, 1 if dom == "pass1_mfma" else 2, d_split, p1_products)
    flops = 2 * m * w * k * (p1_products if dom == "pass1_mfma" else d_split)
    tflops = flops / (kms[dom] * 1e-3) / 1e12
    iters_s = args.steps / el_graph
    alg_iter = 2 * m * w * 2 + 4 * k * 5 * (w + m)          # SURVEY.md 8d (c5: 2.336e9 B -> 3425 it/s)
    out = {
        "metric": METRIC.replace("fp32", "bf16") + f", {k} right-hand sides",
        "value": iters_s, "unit": f"iters/s ({k} right-hand sides per iteration)",
        "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": el_graph / args.steps * 1e3, "higher_is_better": True, "scaling": "none",
        "vs_baseline": None,
        "dtype": "bf16 (A) x hi+lo bf16 residual x " + ("hi+lo bf16" if d_split == 2 else "bf16") +
                 " direction, fp32 MFMA accumulate, fp64 reduce" +
                 (f"; gradient carried in fp32 (G += A^T bf16(V), V = gamma S + the previous rounding), exact every "
                  f"{g_period}" if carry else ""),
        "data": "synthetic (A ~ N(0,1) rows unit-norm, bf16 in HBM; X_true density 0.4; B = A X_true + 0.01 E)",
        "config": {
            "workload": f"configs[4]: k={k} right-hand sides, m={m} n={n} bf16 A, {args.block} feature block(s), 1 GPU",
            "m": m, "n": n, "nrhs": k, "feature_blocks": args.block, "kchunks": pl.kchunks,
            "interleave": args.interleave, "d_split": d_split, "defer_x": pl.get_tuning("defer_x"),
            "carry_g": carry, "g_refresh": g_period, "exact_gradients": pl.stat("exact_gradients"),
            "fuse_update": pl.get_tuning("fuse_update"), "fuse_grid": pl.get_tuning("fuse_grid"),
            "interleave12": [pl.get_tuning("interleave1"), pl.get_tuning("interleave2")],
            "alg_bytes_per_iter": alg_iter,
            "hbm_roofline_iters_per_s": HBM_PEAK_GBS * 1e9 / alg_iter,
            "iter_roofline_frac": iters_s * alg_iter / (HBM_PEAK_GBS * 1e9),
            "rhs_iters_per_s": iters_s * k,
            "iters_per_s_eager_with_events": n_ev / el_ev,
            "launch_mode": f"hipGraph replay, median of {args.windows} windows of {args.steps} iterations (value); "
                           f"eager + HIP events over {n_ev} iterations (kernel times)",
            "windows_s": wins,
            # the rate depends on the iterate: early in a solve x changes in every column and pass 1
            # stores all of X; later it skips the tiles the step left alone (pass 2 measured 201 µs at
            # iterations 5-517, 184 µs at 1500-2012)
            "windows_from_iteration": args.warmup + n_ev,
            "kernel_avg_ms": kms, "status": st,
        },
        "roofline": {
            "bound": "hbm", "kernel": {"pass1_mfma": "k_panel_pass1 (A^T V (carried) / A^T R (exact) panel GEMM + shrink)",
                                       "pass2_mfma": "k_panel_pass2 (A D panel GEMM)"}[dom],
            "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
            "traffic": pmc_traffic(f"panel_m{m}_n{n}_k{k}", {"pass1_mfma": "k_panel_pass1",
                                                              "pass2_mfma": "k_panel_pass2"}[dom]),
            "traffic_source": "profiles/pmc_traffic.json (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, per launch)",
            "alg_bytes_per_launch": pb,
            "avg_launch_ms": kms[dom],
            # whole iteration on the driver-visible clock: SURVEY 8d's bytes per iteration (the two
            # MFMA passes over A + the panel vector I/O) / ms_per_step / peak
            "iteration_frac_end_to_end": alg_iter / (el_graph / args.steps) / (HBM_PEAK_GBS * 1e9),
            "survey_two_pass_frac": alg_iter / (el_graph / args.steps) / (HBM_PEAK_GBS * 1e9),
            "mfma": {"achieved_tflops": tflops, "peak_tflops": MFMA_BF16_DENSE_TFLOPS,
                     "frac": tflops / MFMA_BF16_DENSE_TFLOPS, "flops_per_launch": flops,
                     "counters": mfma_counters({"pass1_mfma": "k_panel_pass1", "pass2_mfma": "k_panel_pass2"}[dom], k)},
            # the bound the k-sweep points at: every byte of A and of the k-wide
            # operand enters LDS through each CU's global_load_lds path; summed over the blocks of a
            # launch, against the best rate that path sustained in any panel pass (9.6 TB/s = 37.5 GB/s
            # per CU: pass 2 at k = 128, profiles/r02/final) -- an empirical cap, not a datasheet peak
            "lds_fill": {"bytes_per_launch": fill_bytes, "achieved_GBps": fill_bytes / (kms[dom] * 1e-3) / 1e9,
                         "empirical_cap_GBps": LDS_FILL_CAP_GBS,
                         "frac": fill_bytes / (kms[dom] * 1e-3) / 1e9 / LDS_FILL_CAP_GBS},
        },
    }
    return out


_JSON_OUT = None


def quiet_stdout():
    """Route fd 1 to stderr for the rest of the run (RCCL prints its version banner on
    stdout at communicator init); the JSON line goes to the original stdout via emit()."""
    global _JSON_OUT
    if _JSON_OUT is None:
        sys.stdout.flush()
        _JSON_OUT = os.fdopen(os.dup(1), "w")
        os.dup2(2, 1)


def emit(out):
    (_JSON_OUT or sys.stdout).write(json.dumps(out) + "\n")
    (_JSON_OUT or sys.stdout).flush()


def release():
    """drop the previous measurement's context, A and graphs before the next one"""
    import gc as _gc
    _gc.collect()
    try:
        import torch
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
    except Exception:
        pass


def side_legs_apply(args):
    """the N = 1 side legs ride on the default line only (configs[1], one block, fp32, no comm)"""
    return (not args.no_side_legs and args.config in (None, 1) and args.block == 1 and args.type == "float"
            and not args.comm and args.rhs == 1 and (args.m, args.n_per_gpu) == (M, N_PER_GPU))


def single_leg(ctx, args, m, n, label, steps_cap=None, ramp_cap=None):
    """one single-GPU measurement (measure()) summarised like the value line: value, ms_per_step,
    roofline (the dominant kernel's and the iteration's fractions) and the kernel averages"""
    a2 = argparse.Namespace(**vars(args))
    a2.m, a2.n_per_gpu, a2.comm = m, n, False
    if steps_cap:
        a2.steps = min(a2.steps, steps_cap)
    if ramp_cap:
        a2.ramp = min(a2.ramp, ramp_cap)
    res = measure(ctx, a2, m, n)
    K = a2.steps
    v, raw = window_rate(res, K)
    kms = res["kernel_ms"]
    ml, w = res["m_local"], res["w_local"]
    if kms.get("onepass", 0.0) > 0:
        dom, kname = "onepass", "k_onepass"
        dom_bytes, it_bytes = alg_bytes_onepass(ml, w), alg_bytes_iter_onepass(ml, w)
    else:
        dom = max(("colpass", "rowpass"), key=lambda q: kms[q])
        kname = "k_" + dom
        dom_bytes = (alg_bytes_colpass if dom == "colpass" else alg_bytes_rowpass)(ml, w)
        it_bytes = alg_bytes_iter(ml, w)
    ms = 1e3 / v
    achieved = dom_bytes / (kms[dom] * 1e-3) / 1e9
    traffic = pmc_traffic(f"m{m}_n{n}_b1_float_g1", kname)
    return {"workload": label, "value": v, "unit": "iters/s", "steps": K, "warmup": a2.warmup,
            "ms_per_step": ms, "ms_per_step_raw_median": raw * 1e3,
            "iteration": "one pass over A" if dom == "onepass" else "two passes over A",
            "windows": res["windows"], "refresh": {"period": res["refresh_period"], "ms_per_refresh": res["refresh_ms"]},
            "onepass_fallbacks": res["fallbacks"], "measure_attempts": res["attempts"],
            "kernel_avg_ms": kms, "status": res["status"],
            "roofline": {"bound": "hbm", "kernel": kname, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "alg_bytes_per_launch": dom_bytes,
                         "avg_launch_ms": kms[dom], "traffic": traffic,
                         "iteration_frac_end_to_end": it_bytes / (ms * 1e-3) / (HBM_PEAK_GBS * 1e9),
                         "survey_two_pass_frac": alg_bytes_iter(ml, w) / (ms * 1e-3) / (HBM_PEAK_GBS * 1e9)}}


def panel_leg(args):
    """configs[4] through measure_panel, summarised for the N = 1 line"""
    a2 = argparse.Namespace(**vars(args))
    a2.config, a2.rhs, a2.m, a2.n_per_gpu = 4, 128, M, N_PER_GPU
    # windows of whole 8-iteration graph replays, at least 64 iterations: a 20-iteration window ran
    # 4 of its iterations as eager launches (the panel graph holds 8), 5 % below the replayed rate
    a2.steps = max(64, -(-a2.steps // 8) * 8)
    p = measure_panel(a2)
    c = p["config"]
    return {"workload": c["workload"], "value": p["value"], "unit": p["unit"], "steps": p["steps"],
            "warmup": p["warmup"], "ms_per_step": p["ms_per_step"], "dtype": p["dtype"],
            "rhs_iters_per_s": c["rhs_iters_per_s"], "iter_roofline_frac": c["iter_roofline_frac"],
            "hbm_roofline_iters_per_s": c["hbm_roofline_iters_per_s"], "windows_s": c["windows_s"],
            "windows_from_iteration": c["windows_from_iteration"],
            "kernel_avg_ms": c["kernel_avg_ms"], "status": c["status"],
            "tuning": {q: c[q] for q in ("d_split", "carry_g", "g_refresh", "defer_x", "fuse_update", "kchunks",
                                         "interleave12")},
            "roofline": p["roofline"]}


def side_legs(ctx, args, out):
    """N = 1: configs[3], configs[4] and configs[2]'s whole matrix on this GPU, each on the driver's
    clock beside the value line (its own windows of --steps iterations, capped for the 2.7 ms
    iterations of configs[3] / [2]); a leg that raises records {"error": ...}"""
    legs = (("config3", lambda: single_leg(ctx, args, 1048576, 4096,
                                           "configs[3]: m=1048576 n=4096 float A, 1 feature block, 1 GPU",
                                           steps_cap=64, ramp_cap=128)),
            ("config4", lambda: panel_leg(args)),
            ("config2_one_gpu", lambda: single_leg(ctx, args, 8192, 524288,
                                                   "configs[2]'s whole matrix on one GPU: m=8192 n=524288 float A, "
                                                   "1 feature block", steps_cap=64, ramp_cap=128)))
    for key, run in legs:
        progress(f"side leg {key}")
        try:
            release()
            out[key] = run()
        except Exception as e:
            out[key] = {"error": f"{type(e).__name__}: {e}"[:400]}
        release()


def visible_gpu_count():
    """GPUs a child process would see, counted in a separate interpreter so that this one never
    loads HIP (torch.cuda.device_count() does not initialise the GPU on this image, but the
    launcher does not rely on that)."""
    import subprocess
    r = subprocess.run([sys.executable, "-c", "import torch; print(torch.cuda.device_count())"],
                       capture_output=True, text=True, timeout=600)
    try:
        return int(r.stdout.strip().splitlines()[-1])
    except Exception:
        return 0


def free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _spawn(cmd):
    """the rank launcher as a child process: its stdout / stderr are this process's (relayed as
    written), its exit status returned"""
    import subprocess
    return subprocess.call(cmd)


def needs_launch(args, env=None):
    """--gpus N > 1 outside torch.distributed.run (no WORLD_SIZE): this process launches the ranks"""
    return args.gpus > 1 and "WORLD_SIZE" not in (os.environ if env is None else env)


def launch_ranks(args, argv, spawn=None, count=None):
    """`python3 bench.py --gpus N` (N > 1) outside torch.distributed.run: start
    `python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1
    --master-port P bench.py <argv>` as a fresh child process (no exec: this process never touches
    the GPU) and return its exit status (128 + signal for a signalled child).  N above the visible
    GPU count fails at once with status 2, unless BPGL_BENCH_DEVICE puts every rank on one GPU
    (the rehearsal mode of Ctx)."""
    n = args.gpus
    if not os.environ.get("BPGL_BENCH_DEVICE"):
        have = (count or visible_gpu_count)()
        if have < n:
            sys.stderr.write(f"bench.py: --gpus {n} but only {have} GPU(s) visible; nothing launched\n")
            return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.join(ROOT, "bench.py")] + list(argv)
    progress(f"launching {n} ranks: {' '.join(cmd)}")
    sys.stdout.flush()
    sys.stderr.flush()
    rc = (spawn or _spawn)(cmd)
    return rc if rc >= 0 else 128 - rc


def main():
    args = parse()
    if needs_launch(args):
        # before quiet_stdout (the child inherits fd 1 for its JSON line) and before torch
        sys.exit(launch_ranks(args, sys.argv[1:]))
    quiet_stdout()
    rank = int(os.environ.get("RANK", "0"))
    cores, cpu_info = host_cores()
    pool = None
    if rank == 0 and not args.no_cpu and args.rhs == 1:
        pool = cpu_pool_leg(cores)     # forks worker processes: before anything touches the GPU
    if args.rhs > 1:
        return main_panel(args)
    import torch
    ctx = Ctx(args.gpus)
    G = ctx.world
    m = args.m
    n_total, scaling = main_shape(args, G)
    res = measure(ctx, args, m, n_total)
    w, ml = res["w_local"], res["m_local"]
    rows = res["gc"].shard == "rows"
    K = args.steps
    ok = [x for x in res["windows"] if x["valid"]]
    el_med = median([x["s_amortised"] for x in ok])
    el_raw = median([x["s"] for x in ok])
    iters_s = K / el_med
    iters_s_ev = res["n_events"] / res["el_events"]
    kms = res["kernel_ms"]
    sa = {"float": 4, "double": 8, "bf16": 2}[args.type]
    onepass = kms.get("onepass", 0.0) > 0
    if onepass:
        dom, dom_bytes, kname = "onepass", alg_bytes_onepass(ml, w, sa), "k_onepass"
        it_bytes = alg_bytes_iter_onepass(ml, w, sa)
    else:
        dom = max(("colpass", "rowpass"), key=lambda k: kms[k])
        dom_bytes = (alg_bytes_colpass if dom == "colpass" else alg_bytes_rowpass)(ml, w, sa)
        kname = "k_" + dom
        it_bytes = alg_bytes_iter(ml, w, sa)
    two_pass_bytes = alg_bytes_iter(ml, w, sa)
    achieved = dom_bytes / (kms[dom] * 1e-3) / 1e9
    workload_key = f"m{m}_n{n_total}_b{args.block}_{args.type}_g{G}" + ("_rows" if rows and G > 1 else "")
    traffic = pmc_traffic(workload_key, kname)
    weak = scaling == "weak"
    ms_step = el_med / K * 1e3
    allreduce_ms = ctx.gather(kms.get("allreduce", 0.0)) if G > 1 or args.comm else None
    out = {
        "metric": METRIC,
        "value": iters_s * G if weak else iters_s,
        "unit": "block-iters/s (1 block-iter = one iteration's worth of an 8192x65536 fp32 matrix, "
                "the per-GPU share; = N x global iterations/s)" if weak else "iters/s",
        "n_gpus": G,
        "steps": K,
        "warmup": args.warmup,
        "ms_per_step": ms_step,
        "higher_is_better": True,
        "scaling": scaling,
        # rounds 1-3 keyed the N > 1 value on the weak problem (block-iters/s); since round 4
        # it is the strong form (iters/s of the 8192 x 65536 matrix) unless --weak -- compare only lines
        # with the same "scaling"
        "value_semantics": {"none": "iters/s of the configured matrix on one GPU",
                            "strong": "iters/s of the fixed matrix split over the N GPUs (rounds >= 4)",
                            "weak": "block-iters/s = N x iters/s of m x 65536 N (the rounds 1-3 N > 1 value)"}[scaling],
        "vs_baseline": None,
        "dtype": "f64",
        "a_dtype": {"float": "fp32", "double": "fp64", "bf16": "bf16"}[args.type],
        "data": "synthetic (A ~ N(0,1) rows unit-norm, generated in HBM; x_true density 0.4; b = A x_true + 0.01 e)",
        "config": {
            "workload": workload_label(args, G, m, n_total, ml, w, rows),
            "m": m, "n": n_total, "m_local": ml, "n_local": w, "feature_blocks": args.block,
            "a_storage": args.type, "accumulate": "fp64",
            "parallelism": (f"{'row' if rows else 'column'}-shard x{G}" if G > 1 or args.comm else "single GPU"),
            "split": ("rows" if rows else "columns") if G > 1 or args.comm else "none",
            "split_rule": "auto: rows for one feature block (one pass over A, DESIGN.md section 6 cost model), "
                          "columns for several" if parse_shard_auto() else "--shard " + args.shard,
            "rccl": bool(G > 1 or args.comm),
            "exchange": ("fp32 (U rounded, scalars hi+lo)" if rows and (G > 1 or args.comm) and args.exchange_fp32
                         else "fp64"),
            "global_iters_per_s": iters_s,
            "iteration": ("one pass over A (k_onepass: s23 = A D and U = A^T s23 together; g += gamma U, "
                          "exact g = A^T r every 256 iterations)" + (
                              "; row shards: k_onepass_fold + RCCL all-reduce of [U | r.s23 | s23.s23 | failed]"
                              if rows and G > 1 else "") if onepass else
                          "two passes over A (A^T r, then A D)"),
            "alg_bytes_per_iter_per_gpu": it_bytes,
            "hbm_roofline_iters_per_s_per_gpu": HBM_PEAK_GBS * 1e9 / it_bytes,
            "iter_roofline_frac": iters_s * it_bytes / (HBM_PEAK_GBS * 1e9),
            "two_pass_alg_bytes_per_iter_per_gpu": two_pass_bytes,
            "two_pass_roofline_iters_per_s_per_gpu": HBM_PEAK_GBS * 1e9 / two_pass_bytes,
            "launch_mode": (f"hipGraph replay, median of {len(ok)} windows of exactly {K} iterations (value); "
                            f"eager + HIP events over {res['n_events']} iterations (kernel times)"),
            "windows": res["windows"],
            "ms_per_step_raw_median": el_raw / K * 1e3,
            "refresh": {"period": res["refresh_period"], "ms_per_refresh": res["refresh_ms"],
                        "folded": "window time - refreshes inside x ms_per_refresh + K/period x ms_per_refresh"},
            "onepass_fallbacks": res["fallbacks"],
            "iters_per_s_eager_with_events": iters_s_ev,
            "kernel_avg_ms": kms,
            "allreduce_ms_per_rank": allreduce_ms,
            "status": res["status"],
        },
        "roofline": {
            "bound": "hbm",
            "kernel": kname + ({"k_colpass": " (A^T s11 pass)", "k_rowpass": " (A D pass)",
                                "k_onepass": " (A D and A^T (A D) in one pass over A)"}[kname]),
            "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
            "traffic": traffic,
            "traffic_source": "profiles/pmc_traffic.json (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, per launch)"
            if traffic else None,
            "alg_bytes_per_launch": dom_bytes,
            "avg_launch_ms": kms[dom],
            # the whole iteration on the driver-visible clock (ms_per_step, per GPU): the bytes this
            # iteration must move / time / peak ...
            "iteration_frac_end_to_end": it_bytes / (ms_step * 1e-3) / (HBM_PEAK_GBS * 1e9),
            # ... and SURVEY 8d's two-pass bytes (2 m w s_A + 8 (5w + 5m)) over the same time: > 1
            # when one pass over A replaces two (8d's figure is superseded)
            "survey_two_pass_frac": two_pass_bytes / (ms_step * 1e-3) / (HBM_PEAK_GBS * 1e9),
        },
    }
    if ctx.rank == 0 and not args.no_cpu:
        progress("CPU baseline")
        note = "" if G == 1 else f" (rank 0's share of the {G}-GPU problem: {ml} x {w})"
        out["cpu_baseline"] = cpu_baseline(res["gc"], res["b"], res["mu"], args.cpu_seconds, cores, cpu_info, note)
        out["cpu_baseline"]["pool_configs0"] = pool
    out["config"]["measure_attempts"] = res["attempts"]
    out["config"]["cus_per_rank"] = res["cus"]
    out["config"]["onepass_rows"] = "interleaved" if res["onepass_rows"] else "consecutive"
    if G > 1 and not args.no_strong:
        # the other legs of one SCALE run: the other scaling form (weak:
        # configs[2]'s shape, or strong when --weak made the weak problem the value line), the
        # reference's column split (two passes, all-reduce of m + 2 + N on the residual side,
        # cpu_calculation.py:23-27) beside the row split, and rank 0 alone on the N = 1 problem --
        # so the split choice and both speedups come from one run
        def fresh():   # drop the previous leg's context, A and communicator before the next
            nonlocal res
            res = None
            import gc as _gc
            _gc.collect()
            torch.cuda.empty_cache()

        def leg(key, run, into=None):
            # a side leg that raises (the same way on every rank: shapes and eligibility are
            # rank-independent; MeasureError is an Exception) is recorded, not fatal -- `value`
            # above is already measured
            try:
                fresh()
                run()
            except Exception as e:
                (out if into is None else into)[key] = {"error": f"{type(e).__name__}: {e}"[:400]}

        other = None   # the other scaling form of the default problem: (key, n_total, weak)
        if not args.strong_total:
            other = ("strong", args.n_per_gpu, False) if weak else ("weak", args.n_per_gpu * G, True)

            def other_leg():
                r2 = measure(ctx, argparse.Namespace(**vars(args)), m, other[1])
                o = leg_summary(ctx, r2, K, G, other[2])
                o["config"] = (f"m={m} n={other[1]} " + ("(configs[2] shape at N = 8), " if other[2] else "") +
                               f"split {G} ways ({o['config']})")
                out[other[0]] = o
            leg(other[0], other_leg)
        if args.block == 1 and rows and not args.exchange_fp32:
            # the same row split with the opt-in fp32 exchange (half the all-reduce bytes): with the
            # fp64 line, the other leg and the column split, four message sizes per SCALE run for the
            # alpha / beta all-reduce model of DESIGN.md section 6.1
            def fp32_rows():
                a2 = argparse.Namespace(**vars(args))
                a2.exchange_fp32 = 1
                r2 = measure(ctx, a2, m, n_total)
                out["rows_exchange_fp32"] = leg_summary(ctx, r2, K, G, weak)
                out["rows_exchange_fp32"]["config"] = (f"m={m} n={n_total} row-sharded, all-reduce of n+5 fp32 "
                                                       f"({out['rows_exchange_fp32']['config']})")
            leg("rows_exchange_fp32", fp32_rows)
        if args.block == 1 and rows:
            a2 = argparse.Namespace(**vars(args))
            a2.shard = "columns"

            def columns():
                r2 = measure(ctx, a2, m, n_total)
                out["columns"] = leg_summary(ctx, r2, K, G, weak)
                out["columns"]["config"] = f"m={m} n={n_total} column-sharded ({out['columns']['config']})"
            leg("columns", columns)
            if other is not None and "error" not in out["columns"]:
                def columns_other():
                    r2 = measure(ctx, a2, m, other[1])
                    out["columns"][other[0]] = leg_summary(ctx, r2, K, G, other[2])
                leg(other[0], columns_other, into=out["columns"])
        if not args.strong_total:
            fresh()
            ctx.barrier()
            n1 = None
            if ctx.rank == 0:
                try:   # rank 0 alone: it must reach the barrier below whatever happens
                    a3 = argparse.Namespace(**vars(args))
                    a3.comm = False
                    solo = SoloCtx(ctx)
                    res = measure(solo, a3, m, args.n_per_gpu)
                    n1 = window_rate(res, K)[0]
                    o = leg_summary(solo, res, K, 1, False)
                except Exception as e:   # recorded; the barrier below is still reached
                    out["n1_same_run"] = {"error": f"{type(e).__name__}: {e}"[:400]}
            ctx.barrier()
            if ctx.rank == 0 and n1:
                o["config"] = f"m={m} n={args.n_per_gpu} on rank 0's GPU alone (no communicator), same run"
                out["n1_same_run"] = o
                speedups(out, n1, G)
    if G == 1 and args.type == "float" and res is not None:
        out["config"]["vendor_gemv_yardstick"] = vendor_yardstick(res["gc"])
        out["config"]["vendor_iteration_yardstick"] = vendor_iteration_yardstick(res["gc"], res["b"], res["mu"])
    if G == 1 and side_legs_apply(args):
        res = None
        side_legs(ctx, args, out)
    if ctx.rank == 0:
        emit(out)
    if ctx.world > 1:
        ctx.dist.destroy_process_group()


def speedups(out, n1, G):
    """speedup_vs_n1 of the value line and of every leg against the N = 1 rate of the same run: a
    strong line's iters/s / n1, a weak line's block-iters/s / n1 (= N x its efficiency); the weak
    forms also carry efficiency = speedup / N"""
    def put(o):
        if isinstance(o, dict) and "value" in o:
            o["speedup_vs_n1"] = o["value"] / n1
            if o.get("scaling") == "weak" or str(o.get("unit", "")).startswith("block"):
                o["efficiency_vs_n1"] = o["value"] / (G * n1)
    put(out)
    for key in ("strong", "weak", "rows_exchange_fp32"):
        put(out.get(key))
    col = out.get("columns")
    put(col)
    if isinstance(col, dict):
        for key in ("strong", "weak"):
            put(col.get(key))


def parse_shard_auto():
    return "--shard" not in sys.argv


if __name__ == "__main__":
    main()
