"""GPU parity tests: the HIP path (through the C ABI) against the oracle and the
reference's golden outputs.  Run on the MI355X box with ``-m gpu``.

Tolerances: every device computation accumulates in fp64 over A's stored
values, so on identical (A, b, mu) the device result differs from the fp64
oracle only by summation order: <= 1e-9 relative l2 on x after 200 iterations
at the golden sizes (measured ~1e-12), and <= 1e-5 (north_star's stated bound)
at the full benchmark shapes.
"""
import os

import numpy as np
import pytest

from conftest import golden_cases
from oracle import oracle

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

from convex_optimization_amd import _native as N  # noqa: E402
from convex_optimization_amd import lasso  # noqa: E402
from convex_optimization_amd.gpu_calculation import GPU_Calculation  # noqa: E402

NT = min(16, os.cpu_count() or 1)


def make_cls(type_name):
    return type("GC_" + type_name, (GPU_Calculation,), {"TYPE": type_name})


def stored(A, type_name):
    """A as the device stores it, returned as fp64 (the exact values the kernels see)."""
    if type_name == "double":
        return A.astype(np.float64)
    if type_name == "float":
        return A.astype(np.float32).astype(np.float64)
    t = torch.from_numpy(np.ascontiguousarray(A, dtype=np.float32)).to(torch.bfloat16)
    return t.to(torch.float64).numpy()


def rel(a, b):
    return np.linalg.norm(np.asarray(a).reshape(-1) - np.asarray(b).reshape(-1)) / max(
        np.linalg.norm(np.asarray(b).reshape(-1)), 1e-300)


# ---------------------------------------------------------------------------
# kernels one by one: diag(A^T A), A^T r, A d
# ---------------------------------------------------------------------------
SHAPES = [(77, 120, 3), (512, 2048, 2), (1000, 4100, 1), (3, 5, 1), (129, 1002, 2), (4099, 1536, 3)]


@pytest.mark.parametrize("type_name", ["double", "float", "bf16"])
@pytest.mark.parametrize("shape", SHAPES)
def test_kernels_match_oracle(type_name, shape):
    H, K, B = shape
    rs = np.random.RandomState(H * 7 + K)
    A = rs.randn(H, K)
    As = stored(A, type_name)
    gc = make_cls(type_name)(A, B, device=0)
    W = K // B
    np.testing.assert_allclose(gc.diag_ATA, oracle.diag_ata(As, B), rtol=1e-12)
    r = rs.randn(H, 1)
    d = rs.randn(W, 1)
    for m in range(B):
        g = np.zeros((W, 1))
        gc.mat_tMulVec_DiffSize(g, m, r)
        ref = oracle.mtv(As, m * W, W, r)
        np.testing.assert_allclose(g.reshape(-1), ref, rtol=1e-11, atol=1e-12 * np.abs(ref).max())
        s = np.zeros((H, 1))
        gc.matMulVec_DiffSize(s, m, d)
        ref = oracle.mv(As, m * W, W, d)
        np.testing.assert_allclose(s.reshape(-1), ref, rtol=1e-11, atol=1e-12 * np.abs(ref).max())


def test_gemv_device_tensors_no_host_copy():
    rs = np.random.RandomState(1)
    A = rs.randn(300, 800).astype(np.float32)
    gc = make_cls("float")(torch.from_numpy(A).cuda(), 2)
    r = torch.randn(300, dtype=torch.float64, device="cuda")
    g = torch.empty(400, dtype=torch.float64, device="cuda")
    gc.mat_tMulVec_DiffSize(g, 1, r)
    ref = oracle.mtv(A.astype(np.float64), 400, 400, r.cpu().numpy())
    np.testing.assert_allclose(g.cpu().numpy(), ref, rtol=1e-12, atol=1e-12)


def test_bad_block_index_raises():
    gc = make_cls("float")(np.ones((8, 16)), 2)
    with pytest.raises(IndexError):
        gc.mat_tMulVec_DiffSize(np.zeros((8, 1)), 2, np.zeros((8, 1)))
    with pytest.raises(ValueError):
        make_cls("float")(np.ones((8, 15)), 2)


# ---------------------------------------------------------------------------
# the device-resident solver against the reference's own runs
# ---------------------------------------------------------------------------
def _fixture_case_types():
    out = []
    for c in golden_cases():
        out.append((c, "double"))
        if c.endswith("f32in"):
            out.append((c, "float"))
    return out


@pytest.mark.parametrize("case,type_name", _fixture_case_types())
def test_solver_matches_reference_run(golden, case, type_name):
    fx = golden(case)
    A = oracle.fixture_A(fx)
    BLOCK, IT = int(fx["BLOCK"]), int(fx["ITER_MAX"])
    gc = make_cls(type_name)(A, BLOCK, device=0)
    order = fx["order"] if bool(fx["random_order"]) else None
    eb = None if fx["err_bound"] < 0 else float(fx["err_bound"])
    res = gc.run(fx["b"], float(fx["mu"]), IT, err_bound=eb, order=order, record=True)
    x = fx["x"].reshape(-1)
    assert res["t_last"] == int(fx["t_last"])
    assert res["stopped"] == bool(fx["stopped"])
    assert rel(res["x"], x) <= 1e-9, rel(res["x"], x)
    T = int(fx["t_last"]) + 1
    np.testing.assert_allclose(res["err_iter"][:T], fx["err_iter"][:T], rtol=1e-6, atol=1e-9)
    assert np.all(np.diff(res["time_iter"][:T]) >= 0)


@pytest.mark.parametrize("case", ["c1_b2_p4_f32in", "random_b4_p1_f32in", "bound_b4_p2_f32in", "stop511_b1_p1_f32in",
                                  "stop257_b1_p4_f32in", "randbound231_b4_p2_f32in", "randbound545_b4_p1_f32in"])
def test_drivers_on_device(golden, case):
    fx = golden(case)
    A = oracle.fixture_A(fx)
    BLOCK, IT = int(fx["BLOCK"]), int(fx["ITER_MAX"])
    gc = make_cls("float")(A, BLOCK, device=0)
    d = gc.diag_ATA
    eb = None if fx["err_bound"] < 0 else float(fx["err_bound"])
    x = fx["x"].reshape(-1)
    import random
    py_seed = int(fx.get("py_seed", 5))
    for cls in ((lasso.ClassLassoR,) if bool(fx["random_order"]) else (lasso.ClassLasso, lasso.ClassLassoDevice)):
        random.seed(py_seed)
        drv = cls(gc, d, A, fx["b"], float(fx["mu"]), BLOCK, IT)
        err_iter = np.zeros(IT)
        drv.run(ERR_BOUND=eb, err_iter=err_iter, SILENCE=True)
        assert drv.iters == int(fx["t_last"]) + 1, cls
        assert rel(drv.x, x) <= 1e-9, (cls, rel(drv.x, x))
    if bool(fx["random_order"]):
        class DevR(lasso.ClassLassoDevice):
            def __init__(self, *a):
                lasso.ClassLassoDevice.__init__(self, *a)
                self.idx_shuffle = np.arange(self.BLOCK)
            index_get = lasso.ClassLassoR.index_get
        random.seed(py_seed)
        drv = DevR(gc, d, A, fx["b"], float(fx["mu"]), BLOCK, IT)
        drv.run(ERR_BOUND=eb, SILENCE=True)
        assert drv.iters == int(fx["t_last"]) + 1
        assert rel(drv.x, x) <= 1e-9


def test_graph_and_eager_identical_and_deterministic(golden):
    fx = golden("c1_b2_p4_f32in")
    A = oracle.fixture_A(fx)
    gc = make_cls("float")(A, 2, device=0)
    a = gc.run(fx["b"], float(fx["mu"]), 120, use_graph=True)["x"]
    b = gc.run(fx["b"], float(fx["mu"]), 120, use_graph=False)["x"]
    c = gc.run(fx["b"], float(fx["mu"]), 120, use_graph=True)["x"]
    np.testing.assert_array_equal(a, b)
    np.testing.assert_array_equal(a, c)


def test_warm_start_and_split_steps(golden):
    """x0 warm start and step() in pieces equal one long run."""
    fx = golden("c1_b1_p1_f32in")
    A = oracle.fixture_A(fx)
    gc = make_cls("float")(A, 1, device=0)
    full = gc.run(fx["b"], float(fx["mu"]), 60)["x"]
    gc.solver_reset(fx["b"], float(fx["mu"]))
    for k in (7, 13, 40):
        gc.solver_step(k)
    np.testing.assert_array_equal(gc.solver_x(), full)
    half = gc.run(fx["b"], float(fx["mu"]), 30)["x"]
    warm = oracle.run(A, fx["b"], float(fx["mu"]), 1, 30, x0=half)["x"]
    dev = gc.run(fx["b"], float(fx["mu"]), 30, x0=half)["x"]
    assert rel(dev, warm) <= 1e-9


def test_zero_problem_gamma_zero():
    """b = 0: D = 0, r2 = 0, the step is 0 (the reference would raise at t = 0)."""
    gc = make_cls("float")(np.random.RandomState(0).randn(64, 128), 2)
    res = gc.run(np.zeros(64), 0.1, 10)
    assert np.all(res["x"] == 0) and res["gamma"] == 0.0


# ---------------------------------------------------------------------------
# benchmark shapes: parity against the oracle on the same fp32 A, and
# size-independent properties of the iteration
# ---------------------------------------------------------------------------
def _device_problem(H, K, B, seed=11):
    from convex_optimization_amd.parameters import device_instance
    return device_instance(H, K, 0.4, B, TYPE="float", seed=seed, device=0)


@pytest.mark.parametrize("H,K,B,IT", [(8192, 65536, 1, 8), (262144, 4096, 1, 6), (8192, 16384, 4, 8)])
def test_benchmark_shapes_match_oracle(H, K, B, IT):
    gc, b, mu, _ = _device_problem(H, K, B)
    res = gc.run(b, mu, IT)
    A_host = gc.A_b_gpu.permute(1, 0, 2).reshape(H, K).cpu().numpy() if B > 1 else \
        gc.A_b_gpu[0].cpu().numpy()
    ref = oracle.run(np.ascontiguousarray(A_host), b.cpu().numpy(), mu, B, IT, nthreads=NT)
    assert rel(res["x"], ref["x"]) <= 1e-5, rel(res["x"], ref["x"])
    assert rel(res["x"], ref["x"]) <= 1e-10   # what fp64 accumulation actually gives


def test_objective_monotone_at_full_size():
    """Exact line search => F(x_t) = 1/2 ||A x_t - b||^2 + mu ||x_t||_1 never increases."""
    H, K = 8192, 65536
    gc, b, mu, _ = _device_problem(H, K, 1, seed=3)
    gc.solver_reset(b, mu)
    res = gc._ctx_residual()
    objs = []
    for _ in range(12):
        gc.solver_step(1)
        gc.stream.synchronize()
        objs.append(0.5 * float(torch.square(res).sum()) + mu * float(gc.solver_x_device().abs().sum()))
    assert all(b2 <= a2 * (1 + 1e-12) for a2, b2 in zip(objs, objs[1:])), objs
    assert objs[-1] < objs[0]


# ---------------------------------------------------------------------------
# column-sharded multi-rank kernels, with the all-reduce done by the test
# (RCCL refuses two ranks on one GPU; the RCCL leg differs only by the call)
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("case,world", [("c1_b2_p4_f32in", 2), ("c1_b1_p1_f32in", 4), ("ragged_b3_p2_f32in", 2)])
def test_external_exchange_ranks_match_single(golden, case, world):
    from convex_optimization_amd import distributed as D
    fx = golden(case)
    A = oracle.fixture_A(fx)
    B, IT = int(fx["BLOCK"]), int(fx["ITER_MAX"])
    ranks = []
    for g in range(world):
        gc = make_cls("float")(D.shard_columns(A, B, g, world), B, device=0)
        gc.set_ranks(g, world)
        gc.solver_reset(fx["b"], float(fx["mu"]), record_len=IT, use_graph=False)
        ranks.append(gc)
    for _ in range(IT):
        for gc in ranks:
            gc.solver_phase(0)
        torch.cuda.synchronize()
        total = sum(gc.exchange_buffer().clone() for gc in ranks)
        for gc in ranks:
            gc.exchange_buffer().copy_(total)
        torch.cuda.synchronize()
        for gc in ranks:
            gc.solver_phase(1)
    x = D.assemble_x([gc.solver_x() for gc in ranks], B)
    ref = fx["x"].reshape(-1)
    assert rel(x, ref) <= 1e-9, rel(x, ref)
    errs = [gc.solver_records()[0] for gc in ranks]
    np.testing.assert_array_equal(errs[0], errs[1])
    np.testing.assert_allclose(errs[0][:IT], fx["err_iter"][:IT], rtol=1e-6, atol=1e-9)


@pytest.mark.parametrize("case", ["c1_b2_p4_f32in", "bound_b4_p2_f32in", "ragged_b3_p2_f32in"])
def test_single_rank_rccl_path(golden, case):
    """The RCCL leg (comm init, all-reduce captured in the graph, k_step) with one rank on one GPU:
    same answers as the reference run and as the communicator-free solver."""
    from convex_optimization_amd import distributed as D
    fx = golden(case)
    A = oracle.fixture_A(fx)
    B, IT = int(fx["BLOCK"]), int(fx["ITER_MAX"])
    eb = None if fx["err_bound"] < 0 else float(fx["err_bound"])
    plain = make_cls("float")(A, B, device=0)
    ref = plain.run(fx["b"], float(fx["mu"]), IT, err_bound=eb, record=True)
    gc = make_cls("float")(A, B, device=0, comm=D.RankComm(0, 1))
    for graph in (True, False):
        res = gc.run(fx["b"], float(fx["mu"]), IT, err_bound=eb, record=True, use_graph=graph)
        assert res["t_last"] == int(fx["t_last"]) and res["stopped"] == bool(fx["stopped"])
        assert rel(res["x"], fx["x"].reshape(-1)) <= 1e-9
        assert rel(res["x"], ref["x"]) <= 1e-12, rel(res["x"], ref["x"])
        T = int(fx["t_last"]) + 1
        np.testing.assert_allclose(res["err_iter"][:T], ref["err_iter"][:T], rtol=1e-12, atol=1e-15)


@pytest.mark.parametrize("case", ["c1_b1_p1_f64", "c1_b2_p4_f64", "ragged_b3_p2_f32in"])
def test_vendor_yardstick_reproduces_reference(golden, case):
    """The rocBLAS-GEMV yardstick (yardstick.VendorLasso, fp64) runs the same iteration."""
    from convex_optimization_amd.yardstick import VendorLasso
    fx = golden(case)
    A = oracle.fixture_A(fx)
    B, IT = int(fx["BLOCK"]), int(fx["ITER_MAX"])
    v = VendorLasso(A, B, dtype=torch.float64, device=0)
    v.reset(fx["b"], float(fx["mu"]))
    v.step(IT)
    assert rel(v.solution(), fx["x"].reshape(-1)) <= 1e-9


def test_tuning_knobs_do_not_change_results(golden):
    fx = golden("c1_b2_p4_f32in")
    A = oracle.fixture_A(fx)
    gc = make_cls("float")(A, 2, device=0)
    base = gc.run(fx["b"], float(fx["mu"]), 50)["x"]
    for key, val in [("nt_loads", 0), ("tail_permille", 0), ("reverse_rows", 1), ("tail_permille", 1000),
                     ("nt_loads", 1), ("col_mode", 1), ("col_mode", 2), ("col_mode", 0)]:
        gc.set_tuning(key, val)
        np.testing.assert_array_equal(gc.run(fx["b"], float(fx["mu"]), 50)["x"], base)
    for gone in ("fused", "onepass_fold", "onepass_variant"):   # removed in round 5
        with pytest.raises(Exception):
            gc.set_tuning(gone, 0)
