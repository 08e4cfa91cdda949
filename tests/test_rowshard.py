"""Row shards (include/bpgl.h bpgl_set_shard, bpgl_onepass.h k_onepass_fold): rank q holds
rows [m_q, m_{q+1}) of the single feature block, x is replicated, each iteration streams the
local A once and all-reduces [U | r.s23 | s23.s23] (w_pad + 2 fp64).

The reference has no row split (it shards columns, cpu_calculation.py:23-27); the iteration
it computes is the same (lasso.py:102-157), so parity is against the reference's fixtures and
the single-rank solver.  The multi-rank cases here run the ranks' kernels in one process on
one GPU with the exchange done by the test (phases 0/1 per iteration, 2/3 for the exact-gradient
refresh); the RCCL leg runs with one rank here and with two processes (each its own NCCL host id,
loopback sockets) in tests/test_rccl_ranks.py.
Tolerances (relative l2 on x): reference fixtures <= 1e-9 (as every solver test); rank
counts against each other and against the single-rank one-pass path <= 1e-10 (the sums over
ranks change the fp64 summation order only)."""
import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

from convex_optimization_amd import _native as N  # noqa: E402
from convex_optimization_amd import distributed as D  # noqa: E402
from convex_optimization_amd.gpu_calculation import GPU_Calculation  # noqa: E402


def make_cls(type_name):
    return type("GC_" + type_name, (GPU_Calculation,), {"TYPE": type_name})


def rel(a, b):
    a, b = np.asarray(a).reshape(-1), np.asarray(b).reshape(-1)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300)


def _exchange(ranks, fp32=False):
    torch.cuda.synchronize()
    total = sum(gc.exchange_buffer(fp32).clone() for gc in ranks)
    for gc in ranks:
        gc.exchange_buffer(fp32).copy_(total)
    torch.cuda.synchronize()


def run_external(A, b, mu, world, iters, type_name="float", err_bound=None, refresh=64, fp32=False, rows=-1):
    """`world` row-shard ranks on one GPU, the all-reduce done here (``fp32``: the fp32 wire
    format of phases 0/1, summed in fp32 like RCCL)."""
    ranks = []
    for g in range(world):
        gc = make_cls(type_name)(D.shard_rows(A, g, world), 1, device=0, shard="rows")
        gc.set_ranks(g, world)
        gc.set_tuning("onepass_refresh", refresh)
        gc.set_tuning("exchange_fp32", 1 if fp32 else 0)
        gc.set_tuning("onepass_rows", rows)
        ranks.append(gc)
    diag = sum(gc._diag.clone() for gc in ranks)   # column norms: sums over ranks
    for g, gc in enumerate(ranks):
        gc.set_diag(diag)
        s, e = D.row_bounds(A.shape[0], g, world)
        gc.solver_reset(np.asarray(b).reshape(-1)[s:e], mu, err_bound=err_bound, record_len=iters,
                        use_graph=False)

    def refresh_g():
        for gc in ranks:
            gc.solver_phase(2)
        _exchange(ranks)
        for gc in ranks:
            gc.solver_phase(3)

    refresh_g()
    for t in range(iters):
        if refresh and t and t % refresh == 0:
            refresh_g()
        for gc in ranks:
            gc.solver_phase(0)
        _exchange(ranks, fp32)
        for gc in ranks:
            gc.solver_phase(1)
    return ranks


def test_external_row_ranks_fp32_exchange_eight_ranks():
    """the opt-in fp32 wire format across 8 row ranks -- configs[2]'s rank count -- summed in
    fp32: every rank's x bit-identical, within 5e-6 of the fp64 exchange and 1e-5 of the oracle
    (measured 1.5e-6: each rank's partial U is rounded before the cross-rank cancellation)"""
    rs = np.random.RandomState(21)
    m, n = 1024, 20000
    A = rs.randn(m, n) / np.sqrt(n)
    b = A @ np.where(rs.rand(n) < 0.3, rs.randn(n), 0.0) + 0.01 * rs.randn(m)
    mu = 0.1 * float(np.abs(A.T @ b).max())
    f32 = run_external(A, b, mu, 8, 120, fp32=True)
    f64 = run_external(A, b, mu, 8, 120, fp32=False)
    xs = [gc.solver_x() for gc in f32]
    for x in xs[1:]:
        np.testing.assert_array_equal(x, xs[0])
    orc = oracle.run(A.astype(np.float32).astype(np.float64), b, mu, 1, 120)["x"]
    print(f"8 ranks fp32 exchange: vs fp64 {rel(xs[0], f64[0].solver_x()):.2e}, vs oracle {rel(xs[0], orc):.2e}")
    assert rel(xs[0], f64[0].solver_x()) <= 5e-6
    assert rel(xs[0], orc) <= 1e-5


@pytest.mark.parametrize("case,world,type_name", [("c1_b1_p1_f32in", 2, "float"), ("c1_b1_p1_f32in", 4, "float"),
                                                  ("c1_b1_p1_f64", 3, "double")])
def test_external_row_ranks_match_reference(golden, case, world, type_name):
    fx = golden(case)
    A = oracle.fixture_A(fx)
    IT = int(fx["ITER_MAX"])
    ranks = run_external(A, fx["b"], float(fx["mu"]), world, IT, type_name=type_name)
    xs = [gc.solver_x() for gc in ranks]
    for x in xs[1:]:
        np.testing.assert_array_equal(x, xs[0])          # x is replicated bit for bit
    assert rel(xs[0], fx["x"]) <= 1e-9, rel(xs[0], fx["x"])
    errs = [gc.solver_records()[0] for gc in ranks]
    np.testing.assert_array_equal(errs[0], errs[-1])
    np.testing.assert_allclose(errs[0][:IT], fx["err_iter"][:IT], rtol=1e-6, atol=1e-9)


@pytest.mark.parametrize("world", [2, 3])
def test_external_row_ranks_interleaved_row_groups(world):
    """every rank's row groups on interleaved rows ("onepass_rows" 1; 3 ranks: ragged shards of 3001
    rows, 5 segment blocks per row, ~50 row groups of ~20 rows per rank): ranks bit-identical, within
    1e-10 of the consecutive-row form and of the single-rank solver, and 1e-8 of the oracle"""
    rs = np.random.RandomState(31)
    m, n = 3001, 20000
    A = rs.randn(m, n) / np.sqrt(n)
    b = A @ np.where(rs.rand(n) < 0.3, rs.randn(n), 0.0) + 0.01 * rs.randn(m)
    mu = 0.1 * float(np.abs(A.T @ b).max())
    IT = 25
    ilv = run_external(A, b, mu, world, IT, rows=1)
    con = run_external(A, b, mu, world, IT, rows=0)
    assert all(gc.solver_stat("onepass_rows") == 1 for gc in ilv)
    assert all(gc.solver_stat("onepass_rows") == 0 for gc in con)
    xs = [gc.solver_x() for gc in ilv]
    for x in xs[1:]:
        np.testing.assert_array_equal(x, xs[0])
    single = make_cls("float")(A, 1, device=0).run(b, mu, IT)["x"]
    orc = oracle.run(A.astype(np.float32).astype(np.float64), b, mu, 1, IT)["x"]
    assert rel(xs[0], con[0].solver_x()) <= 1e-10, rel(xs[0], con[0].solver_x())
    assert rel(xs[0], single) <= 1e-10, rel(xs[0], single)
    assert rel(xs[0], orc) <= 1e-8, rel(xs[0], orc)


def test_external_row_ranks_ragged_and_stop():
    """rows not divisible by the rank count; the err_bound stop fires on every rank at the same t"""
    rs = np.random.RandomState(21)
    m, n = 1001, 5000
    A = rs.randn(m, n) / np.sqrt(n)
    b = A @ np.where(rs.rand(n) < 0.1, rs.randn(n), 0.0) + 0.01 * rs.randn(m)
    mu = 0.1 * float(np.abs(A.T @ b).max())
    single = make_cls("float")(A, 1, device=0)
    ref = single.run(b, mu, 300, err_bound=1e-4)
    ranks = run_external(A, b, mu, 3, 300, err_bound=1e-4)
    st = [gc.solver_status() for gc in ranks]
    assert ref["stopped"] and all(s["stopped"] for s in st)
    assert all(s["t_last"] == ref["t_last"] for s in st), (ref["t_last"], [s["t_last"] for s in st])
    assert rel(ranks[0].solver_x(), ref["x"]) <= 1e-10, rel(ranks[0].solver_x(), ref["x"])


def test_single_rank_rccl_rows_matches_onepass():
    """the RCCL leg (comm init, all-reduce of [U | r.s23 | s23.s23] inside the graph, the
    w-sized diag and gradient all-reduces) with one rank: same iterates as the plain solver"""
    rs = np.random.RandomState(8)
    m, n = 1500, 12000
    A = rs.randn(m, n) / np.sqrt(n)
    b = A @ np.where(rs.rand(n) < 0.3, rs.randn(n), 0.0) + 0.01 * rs.randn(m)
    mu = 0.1 * float(np.abs(A.T @ b).max())
    plain = make_cls("float")(A, 1, device=0).run(b, mu, 150)
    rows = make_cls("float")(A, 1, device=0, comm=D.RankComm(0, 1), shard="rows")
    np.testing.assert_allclose(rows.diag_ATA, make_cls("float")(A, 1, device=0).diag_ATA, rtol=1e-15)
    rows.set_tuning("exchange_fp32", 0)            # the fp64 exchange: the same sums as one rank
    g1 = rows.run(b, mu, 150, use_graph=True)
    g0 = rows.run(b, mu, 150, use_graph=False)
    np.testing.assert_array_equal(g1["x"], g0["x"])
    assert g1["iters"] == 150
    assert rel(g1["x"], plain["x"]) <= 1e-10, rel(g1["x"], plain["x"])


def test_single_rank_rccl_rows_fp32_exchange():
    """the opt-in fp32 RCCL row exchange (U rounded, the line-search scalars as hi + lo
    pairs): graph = eager bitwise, within 1e-6 of the fp64 exchange and within the north_star
    1e-5 of the oracle (measured 1.8e-7 after 300 iterations, the size of the trajectory's
    rounding-order sensitivity)"""
    rs = np.random.RandomState(8)
    m, n = 1500, 12000
    A = rs.randn(m, n) / np.sqrt(n)
    b = A @ np.where(rs.rand(n) < 0.3, rs.randn(n), 0.0) + 0.01 * rs.randn(m)
    mu = 0.1 * float(np.abs(A.T @ b).max())
    rows = make_cls("float")(A, 1, device=0, comm=D.RankComm(0, 1), shard="rows")
    rows.set_tuning("exchange_fp32", -1)           # fp32 with an RCCL communicator
    f1 = rows.run(b, mu, 300, use_graph=True)
    f0 = rows.run(b, mu, 300, use_graph=False)
    np.testing.assert_array_equal(f1["x"], f0["x"])
    rows.set_tuning("exchange_fp32", 0)
    d = rows.run(b, mu, 300)
    A32 = A.astype(np.float32).astype(np.float64)
    orc = oracle.run(A32, b, mu, 1, 300)["x"]
    print(f"fp32 exchange: vs fp64 exchange {rel(f1['x'], d['x']):.2e}, vs oracle {rel(f1['x'], orc):.2e}")
    assert rel(f1["x"], d["x"]) <= 1e-6, rel(f1["x"], d["x"])
    assert rel(f1["x"], orc) <= 1e-5, rel(f1["x"], orc)


def test_two_granules_per_lane_width():
    """SB > 64 segment blocks per row (two hand-off granules per lane), the per-GPU shape of
    configs[2] under row shards at 8 GPUs (1024 x 524288 fp32), one rank"""
    from convex_optimization_amd.parameters import device_instance
    gc, b, mu, _ = device_instance(1024, 524288, 0.4, 1, TYPE="float", seed=3, device=0)
    gc.set_tuning("onepass", 1)
    one = gc.run(b, mu, 10)
    gc.set_tuning("onepass", 0)
    two = gc.run(b, mu, 10)
    assert rel(one["x"], two["x"]) <= 1e-10, rel(one["x"], two["x"])
    rows = make_cls("float")(gc._A_dev, 1, device=0, comm=D.RankComm(0, 1), shard="rows")
    rows.set_tuning("exchange_fp32", 0)
    r = rows.run(b, mu, 10)
    assert rel(r["x"], one["x"]) <= 1e-12, rel(r["x"], one["x"])


def test_row_shard_argument_errors():
    A = np.random.RandomState(0).randn(64, 256)
    with pytest.raises(N.BpglError, match="one feature block"):
        make_cls("float")(A, 2, device=0, shard="rows")
    with pytest.raises(ValueError):
        make_cls("float")(A, 1, device=0, shard="diagonal")
    gc = make_cls("float")(A, 1, device=0, shard="rows")
    gc.set_ranks(0, 2)                             # external exchange: one pass only
    gc.set_tuning("onepass", 0)
    with pytest.raises(N.BpglError, match="external row shards run the one-pass iteration only"):
        gc.solver_reset(np.ones(64), 0.1)
    gc = make_cls("float")(A, 1, device=0, shard="rows")
    gc.set_tuning("onepass", -1)
    gc.solver_reset(np.ones(64), 0.1)
    with pytest.raises(N.BpglError, match="external row shards"):
        gc.solver_phase(2)
    # bind already happened: the layout is fixed
    with pytest.raises(N.BpglError, match="precede"):
        N.check(N.lib().bpgl_set_shard(gc._ctx, N.BPGL_SHARD_COLUMNS), "bpgl_set_shard")


@pytest.mark.parametrize("type_name,world", [("double", 2), ("bf16", 3)])
def test_external_row_ranks_storage_types(type_name, world):
    """fp64 and bf16 storage of the row shards (the bf16 case against the one-rank solver on the
    same bf16-rounded A): every rank's x bit-identical, <= 1e-10 from one rank"""
    rs = np.random.RandomState(30 + world)
    m, n = 700, 9000
    A = rs.randn(m, n) / np.sqrt(n)
    b = A @ np.where(rs.rand(n) < 0.2, rs.randn(n), 0.0) + 0.01 * rs.randn(m)
    mu = 0.1 * float(np.abs(A.T @ b).max())
    ref = make_cls(type_name)(A, 1, device=0).run(b, mu, 120)
    ranks = run_external(A, b, mu, world, 120, type_name=type_name)
    xs = [gc.solver_x() for gc in ranks]
    for x in xs[1:]:
        np.testing.assert_array_equal(x, xs[0])
    assert rel(xs[0], ref["x"]) <= 1e-10, rel(xs[0], ref["x"])


def test_two_granules_ragged_width_with_records():
    """SB = 97 segment blocks (w = 395000, not a multiple of the 4096-column block), err_iter /
    time_iter recording and the err_bound rule through the one-rank RCCL row path"""
    rs = np.random.RandomState(12)
    m, n = 96, 395000
    A = rs.randn(m, n) / np.sqrt(n)
    b = A @ np.where(rs.rand(n) < 0.05, rs.randn(n), 0.0) + 0.01 * rs.randn(m)
    mu = 0.1 * float(np.abs(A.T @ b).max())
    plain = make_cls("float")(A, 1, device=0)
    plain.set_tuning("onepass", 0)
    two = plain.run(b, mu, 60, err_bound=1e-3, record=True)
    rows = make_cls("float")(A, 1, device=0, comm=D.RankComm(0, 1), shard="rows")
    rows.set_tuning("exchange_fp32", 0)
    one = rows.run(b, mu, 60, err_bound=1e-3, record=True)
    assert one["t_last"] == two["t_last"] and one["stopped"] == two["stopped"]
    assert rel(one["x"], two["x"]) <= 1e-10, rel(one["x"], two["x"])
    T = one["t_last"] + 1
    np.testing.assert_allclose(one["err_iter"][:T], two["err_iter"][:T], rtol=1e-8, atol=1e-12)
    # times of the completed iterations increase; the stopping iteration records none, as the
    # reference breaks before time_record (lasso.py:147-157)
    assert np.all(np.diff(one["time_iter"][:T]) > 0) and one["time_iter"][T] == 0.0


def test_rccl_rows_failure_falls_back_to_two_pass_rows():
    """row shards: a failed k_onepass launch (test hook "onepass_fail_at") raises the failure
    slot of the exchange, so every rank skips that iteration and the ones after it; the status
    call re-runs them on the two-pass row iteration (exact g = sum_q A_q^T r_q every iteration,
    s23 on the local rows, an all-reduce of 3 scalars) for the rest of the solve.  Same iterates
    as an undisturbed run to rounding (<= 1e-10)"""
    rs = np.random.RandomState(8)
    m, n = 1500, 12000
    A = rs.randn(m, n) / np.sqrt(n)
    b = A @ np.where(rs.rand(n) < 0.3, rs.randn(n), 0.0) + 0.01 * rs.randn(m)
    mu = 0.1 * float(np.abs(A.T @ b).max())
    rows = make_cls("float")(A, 1, device=0, comm=D.RankComm(0, 1), shard="rows")
    rows.set_tuning("exchange_fp32", 0)
    clean = rows.run(b, mu, 150)
    for fp32 in (0, -1):
        rows.set_tuning("exchange_fp32", fp32)
        rows.set_tuning("onepass_fail_at", 45)
        res = rows.run(b, mu, 150)
        assert res["iters"] == 150
        assert rows.solver_stat("fallbacks") == 1 and rows.solver_stat("onepass") == 0
        tol = 1e-10 if fp32 == 0 else 1e-6    # fp32 exchange before the failure: its own drift
        assert rel(res["x"], clean["x"]) <= tol, (fp32, rel(res["x"], clean["x"]))


@pytest.mark.parametrize("fp32", [False, True])
def test_external_rows_failure_on_one_rank(fp32):
    """caller-side exchange: rank 0's launch fails at t = 5; the summed failure slot makes both
    ranks skip the iteration, bpgl_solver_status reports BPGL_E_EXCHANGE on every rank with the
    state intact, and the caller re-runs the iteration.  x stays bit-identical across ranks and
    within 1e-12 of the undisturbed run (the re-run launch walks its rows in the other direction,
    launches alternate it, so the U partial sums change order)"""
    rs = np.random.RandomState(21)
    m, n = 1001, 5000
    A = rs.randn(m, n) / np.sqrt(n)
    b = A @ np.where(rs.rand(n) < 0.1, rs.randn(n), 0.0) + 0.01 * rs.randn(m)
    mu = 0.1 * float(np.abs(A.T @ b).max())
    ref = run_external(A, b, mu, 2, 40, fp32=fp32)
    ranks = []
    for g in range(2):
        gc = make_cls("float")(D.shard_rows(A, g, 2), 1, device=0, shard="rows")
        gc.set_ranks(g, 2)
        gc.set_tuning("onepass_refresh", 64)
        gc.set_tuning("exchange_fp32", 1 if fp32 else 0)
        ranks.append(gc)
    ranks[0].set_tuning("onepass_fail_at", 5)
    diag = sum(gc._diag.clone() for gc in ranks)
    for g, gc in enumerate(ranks):
        gc.set_diag(diag)
        s, e = D.row_bounds(m, g, 2)
        gc.solver_reset(np.asarray(b).reshape(-1)[s:e], mu, use_graph=False)
    for gc in ranks:
        gc.solver_phase(2)
    _exchange(ranks)
    for gc in ranks:
        gc.solver_phase(3)

    def one_iteration():
        for gc in ranks:
            gc.solver_phase(0)
        _exchange(ranks, fp32)
        for gc in ranks:
            gc.solver_phase(1)

    for t in range(40):
        one_iteration()
        if t == 5:
            for gc in ranks:
                with pytest.raises(N.BpglError, match="state is intact"):
                    gc.solver_status()
            one_iteration()            # the lost iteration again
    xs = [gc.solver_x() for gc in ranks]
    np.testing.assert_array_equal(xs[0], xs[1])
    assert rel(xs[0], ref[0].solver_x()) <= 1e-12, rel(xs[0], ref[0].solver_x())
    assert all(gc.solver_status()["iters"] == 40 for gc in ranks)


def test_two_pass_row_iteration_matches_plain_solver():
    """"onepass" = 0 on a row-shard context: the two-pass row iteration (the fallback after a
    failed hand-off) -- one rank without a communicator and the one-rank RCCL leg, graph and
    eager -- gives the plain solver's iterates (<= 1e-10; exact g every iteration, so no
    recurrence), with the stop rule at the same t"""
    rs = np.random.RandomState(8)
    m, n = 1500, 12000
    A = rs.randn(m, n) / np.sqrt(n)
    b = A @ np.where(rs.rand(n) < 0.3, rs.randn(n), 0.0) + 0.01 * rs.randn(m)
    mu = 0.1 * float(np.abs(A.T @ b).max())
    plain = make_cls("float")(A, 1, device=0)
    plain.set_tuning("onepass", 0)
    ref = plain.run(b, mu, 120, err_bound=1e-4, record=True)
    for comm in (None, D.RankComm(0, 1)):
        rows = make_cls("float")(A, 1, device=0, comm=comm, shard="rows")
        rows.set_tuning("onepass", 0)
        g1 = rows.run(b, mu, 120, err_bound=1e-4, record=True, use_graph=True)
        assert rows.solver_stat("onepass") == 0
        g0 = rows.run(b, mu, 120, err_bound=1e-4, use_graph=False)
        np.testing.assert_array_equal(g1["x"], g0["x"])
        assert g1["t_last"] == ref["t_last"] and g1["stopped"] == ref["stopped"]
        assert rel(g1["x"], ref["x"]) <= 1e-10, rel(g1["x"], ref["x"])
        T = ref["t_last"] + 1
        np.testing.assert_allclose(g1["err_iter"][:T], ref["err_iter"][:T], rtol=1e-8, atol=1e-12)
