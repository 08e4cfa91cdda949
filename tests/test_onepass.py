"""One-pass iteration (bpgl_onepass.h): A streamed once per iteration, the gradient
carried as g += gamma A^T (A D).  Same algorithm as the two-pass iteration
(lasso.py:102-157); the arithmetic differs by summation order, by <= 1 ulp per hand-off
partial (the parity bit) and by the recurrence's accumulated rounding between exact
refreshes (every 256 iterations by default).  Tolerances, relative l2 on x:
  * a few iterations: <= 1e-12 against the two-pass path (measured ~1e-15);
  * 25 iterations of random problems: <= 1e-8 (measured 1e-15 .. 3e-9: these lasso
    trajectories amplify rounding -- the two-pass path itself drifts 6e-10 from the
    oracle on the worst shape);
  * the reference's own fixtures: <= 1e-9, as every other solver test;
  * north_star's bound 1e-5 at the full benchmark shape (measured ~1e-13).
Results are bitwise deterministic (graph = eager = split steps)."""
import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

from convex_optimization_amd import _native as N  # noqa: E402
from convex_optimization_amd.gpu_calculation import GPU_Calculation  # noqa: E402


def make_cls(type_name):
    return type("GC_" + type_name, (GPU_Calculation,), {"TYPE": type_name})


def rel(a, b):
    a, b = np.asarray(a).reshape(-1), np.asarray(b).reshape(-1)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300)


def both(gc, b, mu, iters, **kw):
    out = {}
    for op in (1, 0):
        gc.set_tuning("onepass", op)
        out[op] = gc.run(b, mu, iters, **kw)
    gc.set_tuning("onepass", -1)
    return out[1], out[0]


def used_onepass(gc, b, mu):
    """kernel timing shows which iteration ran"""
    gc.solver_reset(b, mu, use_graph=False)
    gc.set_kernel_timing(True)
    gc.solver_step(2)
    t, n = gc.kernel_times()
    gc.set_kernel_timing(False)
    return t["onepass"] > 0 and t["rowpass"] == 0 and t["colpass"] == 0


@pytest.mark.parametrize("case,type_name", [("c1_b1_p1_f32in", "float"), ("c1_b1_p1_f32in", "double"),
                                            ("c1_b1_p1_f64", "double")])
def test_reference_fixture(golden, case, type_name):
    fx = golden(case)
    A = oracle.fixture_A(fx)
    IT = int(fx["ITER_MAX"])
    gc = make_cls(type_name)(A, 1, device=0)
    eb = None if fx["err_bound"] < 0 else float(fx["err_bound"])
    assert used_onepass(gc, fx["b"], float(fx["mu"]))   # the default for one block on one rank
    one, two = both(gc, fx["b"], float(fx["mu"]), IT, err_bound=eb, record=True)
    for res in (one, two):
        assert res["t_last"] == int(fx["t_last"])
        assert res["stopped"] == bool(fx["stopped"])
        assert rel(res["x"], fx["x"]) <= 1e-9
    assert rel(one["x"], two["x"]) <= 1e-10, rel(one["x"], two["x"])
    T = int(fx["t_last"]) + 1
    np.testing.assert_allclose(one["err_iter"][:T], fx["err_iter"][:T], rtol=1e-6, atol=1e-9)


STOP_CASES = ["stop511_b1_p1_f32in", "stop257_b1_p4_f32in", "stop513_b1_p4_f32in"]


@pytest.mark.parametrize("use_graph", [True, False])
@pytest.mark.parametrize("type_name", ["float", "double"])
@pytest.mark.parametrize("case", STOP_CASES)
def test_stop_rule_pinned_to_reference(golden, case, type_name, use_graph):
    """ERR_BOUND on the default one-pass path (lasso.py:141-150, cpu_calculation.py:15-20).  The
    error criterion is evaluated on the carried g (g += gamma A^T (A D), exact A^T r every 256
    iterations); the reference's ClassLassoCPU evaluates it on the exact A^T r.  The fixtures stop
    where the carried g is oldest (t = 511) and right after a refresh (t = 257, 513): the stop
    iteration and the stopped flag must be the reference's exactly, x within 1e-9 and the
    err_iter trace within 1e-6 relative, with the one-pass kernel in use throughout."""
    fx = golden(case)
    A = oracle.fixture_A(fx)
    gc = make_cls(type_name)(A, 1, device=0)
    assert used_onepass(gc, fx["b"], float(fx["mu"]))
    res = gc.run(fx["b"], float(fx["mu"]), int(fx["ITER_MAX"]), err_bound=float(fx["err_bound"]),
                 record=True, use_graph=use_graph)
    assert gc.solver_stat("onepass") == 1 and gc.solver_stat("fallbacks") == 0
    T = int(fx["t_last"])
    assert bool(fx["stopped"]) and res["stopped"]
    assert res["t_last"] == T, (res["t_last"], T)
    assert rel(res["x"], fx["x"]) <= 1e-9, rel(res["x"], fx["x"])
    np.testing.assert_allclose(res["err_iter"][:T + 1], fx["err_iter"][:T + 1], rtol=1e-6)
    # the margin the carried g had: how far the stopping error sits below the bound, and the
    # smallest error before it above the bound
    eb = float(fx["err_bound"])
    print(f"{case} {type_name} graph={use_graph}: stop t={T}, err[T]/bound={res['err_iter'][T] / eb:.6f}, "
          f"min err[:T]/bound={res['err_iter'][:T].min() / eb:.6f}")


# (m, n, dtype): ragged widths (not a multiple of the 4096-column segment block), fewer
# rows than row groups, many row groups, 64 segment blocks per row, tiny problems
SHAPES = [(1000, 4100, "float"), (37, 9000, "float"), (4099, 1536, "float"), (256, 262144, "float"),
          (3, 5, "float"), (2048, 8192, "double"), (777, 3000, "double"), (1500, 10000, "bf16"),
          (300, 64 * 4096, "bf16"), (64, 2048 * 64, "double")]


@pytest.mark.parametrize("m,n,type_name", SHAPES)
def test_shapes_match_two_pass_and_oracle(m, n, type_name):
    rs = np.random.RandomState(m + 7 * n)
    A = rs.randn(m, n) / np.sqrt(n)
    x_true = np.where(rs.rand(n) < 0.3, rs.randn(n), 0.0)
    b = A @ x_true + 0.01 * rs.randn(m)
    mu = 0.1 * np.abs(A.T @ b).max()
    gc = make_cls(type_name)(A, 1, device=0)
    assert used_onepass(gc, b, mu)
    one, two = both(gc, b, mu, 5)
    assert rel(one["x"], two["x"]) <= 1e-12, rel(one["x"], two["x"])
    IT = 25
    one, two = both(gc, b, mu, IT)
    assert rel(one["x"], two["x"]) <= 1e-8, rel(one["x"], two["x"])
    assert one["t_last"] == two["t_last"]
    if m * n <= 4_000_000:
        Ah = gc.A_b_gpu[0, :, :n].to(torch.float64).cpu().numpy()
        ref = oracle.run(np.ascontiguousarray(Ah), b, mu, 1, IT)
        assert rel(one["x"], ref["x"]) <= 1e-8, rel(one["x"], ref["x"])


@pytest.mark.parametrize("m,n,type_name", [(1000, 4100, "float"), (37, 9000, "float"), (4099, 1536, "float"),
                                            (777, 3000, "double"), (1500, 10000, "bf16"), (300, 64 * 4096, "bf16")])
def test_interleaved_row_groups(m, n, type_name):
    """"onepass_rows" 1 (row group g owns rows g, g + ngroups, ...; the default at configs[1]) and 0
    (R consecutive rows) against the two-pass path, at the tolerances above (the U partials and the
    line-search shares sum other rows per group: rounding only); graph = eager bitwise; the stat
    reports the form in use; the stop rule stops at the same iteration"""
    rs = np.random.RandomState(m + 3 * n)
    A = rs.randn(m, n) / np.sqrt(n)
    b = A @ np.where(rs.rand(n) < 0.3, rs.randn(n), 0.0) + 0.01 * rs.randn(m)
    mu = 0.1 * np.abs(A.T @ b).max()
    gc = make_cls(type_name)(A, 1, device=0)
    gc.set_tuning("onepass", 0)
    two5, two25 = gc.run(b, mu, 5)["x"], gc.run(b, mu, 25)["x"]
    gc.set_tuning("onepass", 1)
    for rows in (1, 0):
        gc.set_tuning("onepass_rows", rows)
        r5 = gc.run(b, mu, 5)
        assert gc.solver_stat("onepass") == 1 and gc.solver_stat("onepass_rows") == rows
        assert rel(r5["x"], two5) <= 1e-12, (rows, rel(r5["x"], two5))
        g = gc.run(b, mu, 25, use_graph=True)["x"]
        e = gc.run(b, mu, 25, use_graph=False)["x"]
        np.testing.assert_array_equal(g, e)
        assert rel(g, two25) <= 1e-8, (rows, rel(g, two25))
    with pytest.raises(N.BpglError):
        gc.set_tuning("onepass_rows", 2)


@pytest.mark.parametrize("m,n,type_name", [(4099, 1536, "float"), (40000, 4096, "float"), (3, 5, "float"),
                                            (2000, 1000, "double"), (1500, 6000, "bf16")])
def test_one_segment_block_lds_hand_off(m, n, type_name):
    """One segment block per row (configs[3]'s shape class): phase 2 folds the row's 4 wave partials
    straight from LDS ("onepass_sb1", the default there) instead of a tagged granule through memory.
    Against the granule path: the same algorithm and the same fold order, the granule's parity bit
    aside (<= 1 ulp per row): <= 1e-12 after 5 iterations, <= 1e-8 after 25, the same stop iteration;
    graph = eager bitwise; the stat reports the path in use"""
    rs = np.random.RandomState(m + n)
    A = rs.randn(m, n) / np.sqrt(n)
    b = A @ np.where(rs.rand(n) < 0.3, rs.randn(n), 0.0) + 0.01 * rs.randn(m)
    mu = 0.1 * np.abs(A.T @ b).max()
    gc = make_cls(type_name)(A, 1, device=0)
    assert used_onepass(gc, b, mu)
    out = {}
    for sb1 in (-1, 0):
        gc.set_tuning("onepass_sb1", sb1)
        r5 = gc.run(b, mu, 5)
        assert gc.solver_stat("onepass_sb1") == (1 if sb1 else 0)
        g = gc.run(b, mu, 25, err_bound=1e-9, record=True, use_graph=True)
        e = gc.run(b, mu, 25, err_bound=1e-9, record=True, use_graph=False)
        np.testing.assert_array_equal(g["x"], e["x"])
        out[sb1] = (r5, g)
    assert rel(out[-1][0]["x"], out[0][0]["x"]) <= 1e-12, rel(out[-1][0]["x"], out[0][0]["x"])
    assert rel(out[-1][1]["x"], out[0][1]["x"]) <= 1e-8, rel(out[-1][1]["x"], out[0][1]["x"])
    assert out[-1][1]["t_last"] == out[0][1]["t_last"]
    with pytest.raises(N.BpglError):
        gc.set_tuning("onepass_sb1", 1)


def test_graph_eager_split_steps_bitwise():
    rs = np.random.RandomState(5)
    A = rs.randn(900, 5000)
    b = rs.randn(900)
    gc = make_cls("float")(A, 1, device=0)
    mu = 0.05 * float(np.abs(A.T @ b).max())
    a = gc.run(b, mu, 90, use_graph=True)["x"]
    e = gc.run(b, mu, 90, use_graph=False)["x"]
    c = gc.run(b, mu, 90, use_graph=True)["x"]
    np.testing.assert_array_equal(a, e)
    np.testing.assert_array_equal(a, c)
    gc.set_tuning("onepass_refresh", 64)
    gc.solver_reset(b, mu)
    for k in (3, 17, 8, 62):   # crosses the refresh points 64 and 0 in different graph phases
        gc.solver_step(k)
    np.testing.assert_array_equal(gc.solver_x(), gc.run(b, mu, 90)["x"])


@pytest.mark.parametrize("graph_max", [1, 2, 8, 64])
def test_graph_sizes_bitwise(graph_max):
    """hipGraphs of 1, 2, ... graph_max iterations: only the replay count changes"""
    rs = np.random.RandomState(11)
    A = rs.randn(700, 6000)
    b = rs.randn(700)
    gc = make_cls("float")(A, 1, device=0)
    mu = 0.05 * float(np.abs(A.T @ b).max())
    gc.set_tuning("onepass_refresh", 64)
    e = gc.run(b, mu, 150, use_graph=False)["x"]
    gc.set_tuning("graph_max", graph_max)
    gc.solver_reset(b, mu)
    for k in (1, 20, 63, 2, 64):   # 150 iterations in runs that straddle the refreshes at 64 and 128
        gc.solver_step(k)
    np.testing.assert_array_equal(gc.solver_x(), e)
    assert gc.solver_stat("enqueued") == 150 and gc.solver_stat("refreshes") == 2


def test_graph_max_rejects_bad_values():
    gc = make_cls("float")(np.ones((64, 256)), 1, device=0)
    for v in (0, 3, 128, -1):
        with pytest.raises(RuntimeError):
            gc.set_tuning("graph_max", v)


@pytest.mark.parametrize("m", [900, 3001])
def test_tail_row_blocks_bitwise_neutral(m):
    """where k_onepass_tail runs the residual update (blocks of its own, the default, or every block
    first) moves no bit: iterates, err record and the stop point are identical; graph and eager"""
    rs = np.random.RandomState(m)
    A = rs.randn(m, 5000)
    b = rs.randn(m)
    mu = 0.05 * float(np.abs(A.T @ b).max())
    gc = make_cls("float")(A, 1, device=0)
    out = {}
    for rb in (1, 0):
        gc.set_tuning("tail_row_blocks", rb)
        for graph in (True, False):
            out[rb, graph] = gc.run(b, mu, 120, err_bound=1e-6, record=True, use_graph=graph)
    for key in out:
        np.testing.assert_array_equal(out[key]["x"], out[1, True]["x"])
        np.testing.assert_array_equal(out[key]["err_iter"], out[1, True]["err_iter"])
        assert out[key]["t_last"] == out[1, True]["t_last"]
    with pytest.raises(Exception):
        gc.set_tuning("tail_row_blocks", 2)


@pytest.mark.parametrize("refresh", [0, 1, 5, 64])
def test_refresh_period(refresh):
    """the gradient recurrence with and without exact refreshes: same iterates to rounding"""
    rs = np.random.RandomState(9)
    A = rs.randn(1200, 6000)
    b = rs.randn(1200)
    mu = 0.05 * float(np.abs(A.T @ b).max())
    gc = make_cls("float")(A, 1, device=0)
    gc.set_tuning("onepass", 0)
    two = gc.run(b, mu, 150)
    gc.set_tuning("onepass", 1)
    gc.set_tuning("onepass_refresh", refresh)
    one = gc.run(b, mu, 150)
    assert rel(one["x"], two["x"]) <= 1e-8, rel(one["x"], two["x"])


def test_stop_rule_and_restart():
    """err_bound stop: same t_last as two-pass; a reset after a stop runs clean (fresh tags)"""
    rs = np.random.RandomState(4)
    A = rs.randn(600, 3000)
    b = A @ np.where(rs.rand(3000) < 0.1, rs.randn(3000), 0.0)
    mu = 0.1 * float(np.abs(A.T @ b).max())
    gc = make_cls("float")(A, 1, device=0)
    one, two = both(gc, b, mu, 400, err_bound=1e-3)
    assert one["stopped"] and two["stopped"] and one["t_last"] == two["t_last"]
    again = gc.run(b, mu, 400, err_bound=1e-3)
    np.testing.assert_array_equal(again["x"], one["x"])


def test_required_but_ineligible_raises():
    A = np.random.RandomState(0).randn(64, 256)
    gc = make_cls("float")(A, 2, device=0)      # two feature blocks
    gc.set_tuning("onepass", 1)
    with pytest.raises(N.BpglError, match="onepass=1"):
        gc.run(np.ones(64), 0.1, 3)
    gc.set_tuning("onepass", -1)
    assert gc.run(np.ones(64), 0.1, 3)["iters"] == 3   # auto falls back to two passes
    with pytest.raises(N.BpglError):
        gc.set_tuning("onepass", 2)


def test_full_size_matches_oracle():
    """configs[1] (8192 x 65536 fp32): one pass per iteration vs the oracle"""
    from convex_optimization_amd.parameters import device_instance
    gc, b, mu, _ = device_instance(8192, 65536, 0.4, 1, TYPE="float", seed=11, device=0)
    assert used_onepass(gc, b, mu)
    res = gc.run(b, mu, 8)
    assert gc.solver_stat("onepass_rows") == 1   # the default here: interleaved row groups
    A_host = gc.A_b_gpu[0].cpu().numpy()
    ref = oracle.run(np.ascontiguousarray(A_host), b.cpu().numpy(), mu, 1, 8, nthreads=16)
    assert rel(res["x"], ref["x"]) <= 1e-5
    assert rel(res["x"], ref["x"]) <= 1e-10, rel(res["x"], ref["x"])


@pytest.mark.parametrize("fail_at,use_graph", [(37, True), (0, False), (199, True)])
def test_hand_off_failure_falls_back_to_two_pass(golden, fail_at, use_graph):
    """A k_onepass launch whose row hand-off runs out of polls (its blocks were not all resident:
    another kernel or process held CUs) commits nothing -- the last block to arrive sees the
    failure and skips the line search, the tail skips the update -- and neither does any later
    iteration of the same step call.  bpgl_solver_status re-runs the lost iterations on the
    two-pass kernels for the rest of the solve.  The test hook "onepass_fail_at" makes the launch
    of iteration t report such a failure (once).  Result: the reference fixture within 1e-9 and
    the reference's err_iter trace, as every solver test; the next solve runs one pass again."""
    fx = golden("c1_b1_p1_f32in")
    A = oracle.fixture_A(fx)
    IT = int(fx["ITER_MAX"])
    gc = make_cls("float")(A, 1, device=0)
    gc.set_tuning("onepass", 1)
    gc.set_tuning("onepass_fail_at", fail_at)
    res = gc.run(fx["b"], float(fx["mu"]), IT, record=True, use_graph=use_graph)
    assert gc.solver_stat("fallbacks") == 1 and gc.solver_stat("onepass") == 0
    assert res["iters"] == IT and res["t_last"] == IT - 1
    assert rel(res["x"], fx["x"]) <= 1e-9, rel(res["x"], fx["x"])
    np.testing.assert_allclose(res["err_iter"][:IT], fx["err_iter"][:IT], rtol=1e-6, atol=1e-9)
    again = gc.run(fx["b"], float(fx["mu"]), IT)
    assert gc.solver_stat("fallbacks") == 0 and gc.solver_stat("onepass") == 1
    assert rel(again["x"], res["x"]) <= 1e-10, rel(again["x"], res["x"])


def test_failure_state_is_frozen_until_status():
    """iterations after a failed launch leave x, the residual and t untouched until the status
    call recovers them (split step calls, a failure in the middle of an 8-iteration graph)"""
    rs = np.random.RandomState(17)
    A = rs.randn(700, 9000)
    b = rs.randn(700)
    mu = 0.05 * float(np.abs(A.T @ b).max())
    gc = make_cls("float")(A, 1, device=0)
    clean = gc.run(b, mu, 60)
    gc.set_tuning("onepass_fail_at", 20)
    gc.solver_reset(b, mu)
    gc.solver_step(20)
    gc.stream.synchronize()
    x20 = gc._x.clone()
    r20 = gc._ctx_residual().clone()
    gc.solver_step(24)                 # iteration 20 fails: iterations 20..43 commit nothing
    gc.stream.synchronize()
    assert torch.equal(gc._x, x20) and torch.equal(gc._ctx_residual(), r20)
    st = gc.solver_status()            # recovers 20..43 on the two-pass kernels
    assert st["iters"] == 44 and gc.solver_stat("fallbacks") == 1
    gc.solver_step(16)
    assert gc.solver_status()["iters"] == 60
    assert rel(gc.solver_x(), clean["x"]) <= 1e-10, rel(gc.solver_x(), clean["x"])


def test_contention_with_a_concurrent_kernel():
    """the real failure mode: long GEMMs on another stream hold CUs while the solver runs.
    Whether or not a hand-off runs out of polls (it depends on the scheduler), the solve
    finishes with every iteration applied and the same iterates as an undisturbed run to
    rounding (a fallback changes the summation path: <= 1e-9)"""
    rs = np.random.RandomState(23)
    A = rs.randn(2048, 65536) / 256.0
    b = rs.randn(2048)
    mu = 0.05 * float(np.abs(A.T @ b).max())
    gc = make_cls("float")(A, 1, device=0)
    clean = gc.run(b, mu, 300)
    hog = torch.cuda.Stream(device=0)
    X = torch.randn(8192, 8192, device="cuda:0")
    with torch.cuda.stream(hog):
        for _ in range(12):
            X = torch.tanh(X @ X * 1e-4)
    gc.solver_reset(b, mu)
    gc.solver_step(300)
    st = gc.solver_status()
    torch.cuda.synchronize()
    print(f"contention: fallbacks {gc.solver_stat('fallbacks')}, iters {st['iters']}")
    assert st["iters"] == 300
    assert rel(gc.solver_x(), clean["x"]) <= 1e-9, rel(gc.solver_x(), clean["x"])


def test_iterate_recovers_without_iters_done(golden):
    """bpgl_iterate (the one-call C entry point) always goes through bpgl_solver_status, so a
    failed one-pass launch is re-run even when the caller passes iters_done = NULL (include/bpgl.h)"""
    fx = golden("c1_b1_p1_f32in")
    A = oracle.fixture_A(fx)
    IT = int(fx["ITER_MAX"])
    gc = make_cls("float")(A, 1, device=0)
    gc.set_tuning("onepass", 1)
    gc.set_tuning("onepass_fail_at", 37)
    b = torch.tensor(np.asarray(fx["b"]).reshape(-1), dtype=torch.float64, device="cuda:0")
    x = torch.zeros(gc.MAT_WIDTH_PAD, dtype=torch.float64, device="cuda:0")
    torch.cuda.synchronize()
    with gc._on_stream():
        N.check(N.lib().bpgl_iterate(gc._ctx, IT, None, float(fx["mu"]), N.ptr(b), N.ptr(x), None, None, -1.0,
                                     None), "bpgl_iterate")
    torch.cuda.synchronize()
    assert gc.solver_stat("fallbacks") == 1
    xr = x[:gc.MAT_WIDTH].cpu().numpy()
    assert rel(xr, fx["x"]) <= 1e-9, rel(xr, fx["x"])
