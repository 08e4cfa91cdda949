"""bench.py's algorithmic-byte figures against SURVEY.md 8d (CPU only; no GPU touched)."""
import importlib.util
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_iteration_bytes_match_survey():
    b = _bench()
    c2 = b.alg_bytes_iter(8192, 65536)
    assert c2 == 2 * 8192 * 65536 * 4 + 8 * (5 * 65536 + 5 * 8192)
    assert abs(b.HBM_PEAK_GBS * 1e9 / c2 - 1861) < 1.0          # "roofline 1861 it/s"
    c4 = b.alg_bytes_iter(1048576, 4096)
    assert abs(c4 - 3.440e10) < 0.001e10 and abs(b.HBM_PEAK_GBS * 1e9 / c4 - 232.5) < 0.5


def test_pass_bytes_and_panel_figures():
    b = _bench()
    assert b.alg_bytes_colpass(8192, 65536) == 8192 * 65536 * 4 + 8 * 8192 + 8 * 65536
    assert b.alg_bytes_rowpass(8192, 65536, 2) == 8192 * 65536 * 2 + 8 * 65536 + 8 * 8192
    # c5 per iteration: 2.336e9 B -> ~3425 it/s; flops 4 m w k = 2.749e11
    c5 = 2 * 8192 * 65536 * 2 + 4 * 128 * 5 * (65536 + 8192)
    assert abs(c5 - 2.336e9) < 0.001e9 and abs(8e12 / c5 - 3425) < 1.0
    assert b.panel_bytes_pass(8192, 65536, 128) == 2 * 8192 * 65536 + 8 * 128 * (8192 + 65536)


def test_panel_fill_bytes():
    """roofline.lds_fill of the configs[4] line: A plus every block's copy of the k-wide operand"""
    b = _bench()
    m, w, k = 8192, 65536, 128
    assert b.panel_fill_bytes(m, w, k, 1) == 2 * m * w + 256 * 4 * k * m == 2 ** 31
    assert b.panel_fill_bytes(m, w, k, 2) == 2 * m * w + 32 * 4 * k * w == 2 ** 31
    assert b.panel_fill_bytes(m, w, k, 2, d_split=1) == 2 * m * w + 32 * 2 * k * w
    assert b.panel_fill_bytes(m, w, 16, 1) < b.panel_fill_bytes(m, w, 128, 1)


def test_onepass_bytes():
    """one pass over A per iteration: the same vector I/O, A read once (roofline ~3720 it/s)"""
    b = _bench()
    it = b.alg_bytes_iter_onepass(8192, 65536)
    assert it == 8192 * 65536 * 4 + 8 * (5 * 65536 + 5 * 8192)
    assert it < b.alg_bytes_iter(8192, 65536) / 1.99
    assert abs(b.HBM_PEAK_GBS * 1e9 / it - 3720) < 1.0
    assert b.alg_bytes_onepass(8192, 65536) == 8192 * 65536 * 4 + 8 * 8192 + 16 * 65536


def test_default_arguments_are_the_headline_config():
    b = _bench()
    import sys
    argv = sys.argv
    try:
        sys.argv = ["bench.py"]
        a = b.parse()
    finally:
        sys.argv = argv
    assert (a.gpus, a.m, a.n_per_gpu, a.block, a.type, a.rhs) == (1, 8192, 65536, 1, "float", 1)
    assert a.onepass == -1   # the library's choice: one pass when eligible
    assert a.steps > 0 and a.warmup >= 0


def test_multi_gpu_defaults_keep_per_gpu_bytes():
    """N > 1: row shards by default; the weak-scaling shape (m = 8192, n = 65536 N) gives every
    GPU exactly the bytes of A of N = 1, and the rows cover m once"""
    b = _bench()
    from convex_optimization_amd.distributed import row_bounds
    import sys
    argv = sys.argv
    try:
        sys.argv = ["bench.py", "--gpus", "8"]
        a = b.parse()
    finally:
        sys.argv = argv
    assert a.shard == "rows"
    for G in (1, 2, 4, 8):
        n = a.n_per_gpu * G
        rows = [row_bounds(a.m, g, G) for g in range(G)]
        assert sum(e - s for s, e in rows) == a.m
        assert all((e - s) * n == a.m * a.n_per_gpu for s, e in rows)


def test_emit_writes_one_json_line():
    import io
    import json
    b = _bench()
    buf = io.StringIO()
    b._JSON_OUT = buf
    b.emit({"metric": "m", "value": 1.0})
    lines = buf.getvalue().splitlines()
    assert len(lines) == 1 and json.loads(lines[0])["value"] == 1.0


def _parse(b, argv):
    import sys
    old = sys.argv
    try:
        sys.argv = ["bench.py"] + argv
        return b.parse()
    finally:
        sys.argv = old


def test_config_mapping_and_split_rule():
    """--config 2 is configs[2]'s own problem (8192 x 524288) split over the GPUs (strong);
    --shard auto picks rows for one feature block and columns for several"""
    b = _bench()
    a = _parse(b, ["--config", "2", "--gpus", "8"])
    assert (a.m, a.n_per_gpu, a.strong_total, a.shard) == (8192, 65536, True, "rows")
    a = _parse(b, ["--config", "2"])
    assert (a.m, a.n_per_gpu) == (8192, 524288)
    assert _parse(b, ["--block", "2"]).shard == "columns"
    assert _parse(b, ["--block", "2", "--shard", "rows"]).shard == "rows"
    a = _parse(b, ["--config", "3"])
    assert (a.m, a.n_per_gpu) == (1048576, 4096)


def test_workload_labels_follow_the_shape():
    b = _bench()
    a = _parse(b, ["--config", "3"])
    assert b.workload_label(a, 1, 1048576, 4096, 1048576, 4096, False).startswith("configs[3]:")
    a = _parse(b, [])
    assert b.workload_label(a, 1, 8192, 65536, 8192, 65536, False).startswith("configs[1]:")
    assert "row-sharded 1024 rows/GPU" in b.workload_label(a, 8, 8192, 524288, 1024, 524288, True)
    a = _parse(b, ["--config", "2", "--gpus", "8"])
    assert b.workload_label(a, 8, 8192, 524288, 1024, 524288, True).startswith("configs[2]:")


def test_host_cores_and_window_median():
    b = _bench()
    n, info = b.host_cores()
    assert 1 <= n <= (os.cpu_count() or 1) and info["affinity"] >= 1 and info["threads"] == n
    assert b.median([3.0, 1.0, 2.0]) == 2.0 and b.median([4.0, 1.0, 2.0, 3.0]) == 2.5


def test_pool_baseline_matches_oracle():
    """the Pool-parallel CPU leg (the reference's ClassLassoCPU structure, oracle/pool_baseline.py)
    computes the reference iteration: same x as the C oracle with the same P-way split"""
    import numpy as np
    from oracle import oracle
    from oracle.pool_baseline import instance, largest_divisor_at_most, run_pool
    A, bb, mu = instance(128, 512, seed=3)
    x, el, _ = run_pool(A, bb, mu, 2, 4, 12)
    ref = oracle.run(A, bb, mu, 2, 12, P=4)["x"]
    assert np.linalg.norm(x - ref) <= 1e-10 * np.linalg.norm(ref)
    assert largest_divisor_at_most(2048, 12) == 8 and largest_divisor_at_most(2048, 64) == 64


def test_multi_gpu_legs_carry_both_splits():
    """the N > 1 line's side legs (bench.leg_summary): value in the leg's unit, per-rank all-reduce
    times, and the iteration form; window_rate takes the median of the valid windows only"""
    b = _bench()

    class FakeGC:
        shard = "columns"

    wins = [{"s": 0.1, "s_amortised": 0.1, "valid": True}, {"s": 0.5, "s_amortised": 0.5, "valid": False},
            {"s": 0.2, "s_amortised": 0.2, "valid": True}, {"s": 0.3, "s_amortised": 0.3, "valid": True}]
    res = {"windows": wins, "kernel_ms": {"colpass": 0.3, "rowpass": 0.3, "allreduce": 0.02, "onepass": 0.0},
           "m_local": 8192, "w_local": 65536, "gc": FakeGC(), "fallbacks": 0, "cus": 256}
    v, raw = b.window_rate(res, 100)
    assert abs(v - 100 / 0.2) < 1e-9 and abs(raw - 0.2 / 100) < 1e-12

    class TwoRanks(b.SoloCtx):
        def gather(self, x):
            return [float(x), float(x) + 1e-3]

    ctx = TwoRanks(type("C", (), {"local": 0})())
    weak = b.leg_summary(ctx, res, 100, 2, True)
    assert weak["value"] == 2 * v and weak["unit"] == "block-iters/s" and weak["split"] == "columns"
    assert weak["iteration"] == "two passes over A" and len(weak["allreduce_ms_per_rank"]) == 2
    strong = b.leg_summary(ctx, res, 100, 2, False)
    assert strong["value"] == v and strong["unit"] == "iters/s"
    solo = b.SoloCtx(type("C", (), {"local": 3})())
    assert (solo.rank, solo.world, solo.local) == (0, 1, 3) and solo.max(2.0) == 2.0 and solo.gather(1) == [1.0]


def test_multi_gpu_value_is_the_metric_unit():
    """N > 1: value is iterations/s of the metric's named 8192 x 65536 fp32 matrix split N ways
    (strong scaling); the weak problem (n = 65536 N, block-iters/s) is the side leg "weak", and
    --weak / --config 2 keep their own shapes; N = 1 reports "scaling": "none\""""
    b = _bench()
    for G in (2, 4, 8):
        a = _parse(b, ["--gpus", str(G)])
        assert (a.m, b.main_shape(a, G)) == (8192, (65536, "strong"))
        a = _parse(b, ["--gpus", str(G), "--weak"])
        assert b.main_shape(a, G) == (65536 * G, "weak")
    a = _parse(b, [])
    assert b.main_shape(a, 1) == (65536, "none")
    import os as _os
    _os.environ["WORLD_SIZE"] = "8"
    try:
        a = _parse(b, ["--config", "2", "--gpus", "8"])
    finally:
        del _os.environ["WORLD_SIZE"]
    assert b.main_shape(a, 8) == (524288, "strong")
    assert b.workload_label(_parse(b, []), 8, 8192, 65536, 1024, 65536, True).startswith(
        "configs[1] matrix (the metric's 8192x65536) split 8 ways")


def test_speedups_against_the_same_run_n1():
    """speedup_vs_n1 on the value line and every leg; efficiency only on the weak forms"""
    b = _bench()
    out = {"value": 1000.0, "scaling": "strong",
           "weak": {"value": 6000.0, "unit": "block-iters/s", "scaling": "weak"},
           "columns": {"value": 400.0, "unit": "iters/s", "scaling": "strong",
                       "weak": {"value": 2000.0, "unit": "block-iters/s", "scaling": "weak"}},
           "rows_exchange_fp32": {"error": "x"}}
    b.speedups(out, 250.0, 8)
    assert out["speedup_vs_n1"] == 4.0 and "efficiency_vs_n1" not in out
    assert out["weak"]["speedup_vs_n1"] == 24.0 and out["weak"]["efficiency_vs_n1"] == 3.0
    assert out["columns"]["speedup_vs_n1"] == 1.6 and out["columns"]["weak"]["speedup_vs_n1"] == 8.0
    assert "speedup_vs_n1" not in out["rows_exchange_fp32"]


def test_measure_error_is_an_exception():
    """a side leg whose windows are all invalid must be recorded, not end the run"""
    b = _bench()
    assert issubclass(b.MeasureError, Exception)


_LAUNCH_SCRIPT = r'''
import importlib.util, json, os, sys
root = sys.argv[1]
rc_child, have = int(sys.argv[2]), int(sys.argv[3])
sys.argv = ["bench.py", "--gpus", "2", "--steps", "20", "--warmup", "5"]
spec = importlib.util.spec_from_file_location("bench", os.path.join(root, "bench.py"))
b = importlib.util.module_from_spec(spec)
spec.loader.exec_module(b)
calls = []
b._spawn = lambda cmd: (calls.append(cmd), rc_child)[1]
b.visible_gpu_count = lambda: have
rc = None
try:
    b.main()
except SystemExit as e:
    rc = e.code
print(json.dumps({"rc": rc, "cmd": calls, "torch": "torch" in sys.modules,
                  "hip": [m for m in sys.modules if m.startswith("torch.cuda")]}))
'''


def _run_launcher(rc_child, have, extra_env=None):
    import json
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "BPGL_BENCH_DEVICE")}
    env.update(extra_env or {})
    r = subprocess.run([sys.executable, "-c", _LAUNCH_SCRIPT, ROOT, str(rc_child), str(have)],
                       capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 0, r.stderr
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_launcher_starts_ranks_as_a_child_without_touching_the_gpu():
    """`python3 bench.py --gpus 2` with no WORLD_SIZE (VERDICT r04 Missing #1): the parent starts
    torch.distributed.run as a child with the same arguments, never imports torch, and exits with
    the child's status"""
    o = _run_launcher(0, 8)
    assert o["rc"] == 0 and not o["torch"] and not o["hip"]
    (cmd,) = o["cmd"]
    i = cmd.index("torch.distributed.run")
    assert cmd[i - 1] == "-m" and "--nproc-per-node=2" in cmd and "--master-addr=127.0.0.1" in cmd
    assert "--nnodes=1" in cmd and any(c.startswith("--master-port=") for c in cmd)
    j = [k for k, c in enumerate(cmd) if c.endswith("bench.py")][-1]
    assert cmd[j + 1:] == ["--gpus", "2", "--steps", "20", "--warmup", "5"]
    assert _run_launcher(3, 8)["rc"] == 3          # the child's status is propagated
    assert _run_launcher(-9, 8)["rc"] == 137       # a signalled child: 128 + signal


def test_launcher_fails_fast_without_enough_gpus():
    o = _run_launcher(0, 1)
    assert o["rc"] == 2 and o["cmd"] == [] and not o["torch"]
    # the one-GPU rehearsal (every rank on BPGL_BENCH_DEVICE) skips the count
    o = _run_launcher(0, 1, {"BPGL_BENCH_DEVICE": "0"})
    assert o["rc"] == 0 and len(o["cmd"]) == 1


def test_launch_decision():
    b = _bench()
    a = _parse(b, ["--gpus", "2"])
    assert b.needs_launch(a, {}) and not b.needs_launch(a, {"WORLD_SIZE": "2"})
    assert not b.needs_launch(_parse(b, []), {})


def test_side_legs_ride_on_the_default_line_only():
    b = _bench()
    assert b.side_legs_apply(_parse(b, []))
    for argv in (["--no-side-legs"], ["--config", "3"], ["--type", "bf16"], ["--block", "2"], ["--comm"]):
        assert not b.side_legs_apply(_parse(b, argv)), argv


def test_one_pass_eager_window_always_times_a_refresh():
    """VERDICT r05 Weak #3: every one-pass leg folds the exact-gradient refresh into its rate, so
    its eager (event-timed) window must contain one (the refresh runs before iteration t when t is
    a positive multiple of the period); measure() raises MeasureError when a one-pass leg timed
    none.  Two-pass legs keep max(K, ramp)."""
    b = _bench()
    for period in (64, 256, 1000):
        for warmup in (0, 1, 5, 20, 40, 200, 255, 256, 257, 511, 700):
            for steps, ramp in ((20, 512), (64, 128), (256, 512), (30, 128), (1, 1)):
                n = b.eager_window_len(steps, ramp, warmup, period, 1)
                assert n >= max(steps, ramp)
                assert any(t % period == 0 for t in range(max(warmup, 1), warmup + n)), (period, warmup, n)
                assert b.eager_window_len(steps, ramp, warmup, period, 0) == max(steps, ramp)
                assert b.eager_window_len(steps, ramp, warmup, 0, 1) == max(steps, ramp)
    src = open(os.path.join(ROOT, "bench.py")).read()
    assert "timed no exact-gradient refresh" in src
