"""Parity at BASELINE.json's full single-GPU sizes, against the oracle on the same fp32 A.

  * configs[1] (8192 x 65536 fp32), 640 iterations: the one-pass iteration's carried gradient
    (g += gamma A^T (A D)) with its default exact refresh every 256 iterations crosses two
    refreshes; bound: north_star's 1e-5 relative l2 on x.
  * configs[3] (1048576 x 4096 fp32 = 2^32 elements, 16 GiB): past 2^31 elements, where the
    reference's `int` offsets overflow (gpu_calculation.py:49,86,266,282).  A few iterations
    against the oracle (int64 indexing on both sides), then size-independent properties over a
    longer run: the objective never increases (exact line search, lasso.py:129-136) and the
    one-pass and two-pass iterations agree.

Tolerances are the north_star bound (1e-5) for the long run; the short runs against the oracle
are held to 1e-9 (measured ~1e-14: the paths differ by summation order only), one pass against
two passes over 30 iterations to 1e-8 (as tests/test_onepass.py at 25 iterations).

  * configs[3] on the BASELINE Gaussian recipe (rows N(0,1), unit norm; the instance generated in
    HBM by torch) for 260 iterations -- across the one-pass exact-gradient refresh at 256 -- against
    the reference iteration restated in torch fp64 on the GPU (tests/torch_restatement.py, pinned to
    the C oracle on a small instance in the same test).  Bound: north_star's 1e-5 on x.
  * configs[3] and configs[2] on the same recipe as oracle/gauss_instance.c generates it (bit-identical
    on every host) against the C oracle's own 300 iterations, run once in the build container
    (tests/golden/gauss_configs{3,2}.npz, tests/golden/make_gauss.py)."""
import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

from convex_optimization_amd.parameters import device_instance  # noqa: E402


def rel(a, b):
    a, b = np.asarray(a).reshape(-1), np.asarray(b).reshape(-1)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300)


def objective(gc, mu):
    """1/2 ||A x - b||^2 + mu ||x||_1 from the solver's residual (lasso.py:47-48)"""
    r = gc._ctx_residual()
    return 0.5 * float(torch.dot(r, r)) + mu * float(gc.solver_x_device().abs().sum())


@pytest.mark.timeout(900)
def test_config1_long_horizon_crosses_two_refreshes():
    gc, b, mu, _ = device_instance(8192, 65536, 0.4, 1, TYPE="float", seed=29, device=0)
    IT = 640
    res = gc.run(b, mu, IT, record=True)
    assert gc.solver_stat("onepass") == 1 and gc.solver_stat("refreshes") == IT // 256
    assert res["iters"] == IT
    A = np.ascontiguousarray(gc.A_b_gpu[0].cpu().numpy())
    ref = oracle.run(A, b.cpu().numpy(), mu, 1, IT, nthreads=16)
    e = rel(res["x"], ref["x"])
    print(f"configs[1], {IT} iterations: rel l2 vs oracle {e:.3e}")
    assert e <= 1e-5, e
    # the error criterion falls toward 0; its late values carry the trajectory's rounding
    # sensitivity (measured: within 3.1e-8 absolute of the oracle's, first value 0.98)
    np.testing.assert_allclose(res["err_iter"][:IT], ref["err_iter"][:IT], rtol=1e-4, atol=1e-6 * ref["err_iter"][0])


@pytest.mark.timeout(900)
def test_config3_full_size_past_2_31_elements():
    m, n = 1048576, 4096
    assert m * n == 1 << 32
    gc, b, mu, _ = device_instance(m, n, 0.4, 1, TYPE="float", seed=31, device=0)
    IT = 4
    one = gc.run(b, mu, IT)
    assert gc.solver_stat("onepass") == 1
    A = np.ascontiguousarray(gc.A_b_gpu[0].cpu().numpy())
    bh = b.cpu().numpy()
    # the last rows and columns are reached (int64 offsets): the oracle's A.d on the same A
    d = np.random.RandomState(1).randn(n)
    s = torch.empty(m, dtype=torch.float64, device="cuda:0")
    gc.matMulVec_DiffSize(s, 0, torch.from_numpy(d).cuda())
    s_ref = oracle.mv(A, 0, n, d, nthreads=16)
    assert rel(s.cpu().numpy(), s_ref) <= 1e-12 and rel(s.cpu().numpy()[-1024:], s_ref[-1024:]) <= 1e-12
    ref = oracle.run(A, bh, mu, 1, IT, nthreads=16)
    del A
    e = rel(one["x"], ref["x"])
    print(f"configs[3] {m}x{n}, {IT} iterations: one pass vs oracle {e:.3e}")
    assert e <= 1e-9, e
    # size-independent properties over a longer run: monotone objective, one pass = two passes
    objs = []
    gc.solver_reset(b, mu)
    objs.append(objective(gc, mu))
    for _ in range(6):
        gc.solver_step(5)
        gc.solver_status()
        objs.append(objective(gc, mu))
    x1 = gc.solver_x()
    print("objective:", " ".join(f"{o:.10e}" for o in objs))
    assert all(objs[k + 1] <= objs[k] * (1 + 1e-12) for k in range(len(objs) - 1)), objs
    gc.set_tuning("onepass", 0)
    x2 = gc.run(b, mu, 30)["x"]
    e2 = rel(x1, x2)
    print(f"configs[3], 30 iterations: one pass vs two passes {e2:.3e}")
    assert e2 <= 1e-8, e2   # measured 1.0e-9 (near convergence; the paths differ in summation order)


def _external_rows(A_dev, b, mu, world, iters, refresh=256):
    """`world` row-shard contexts on this GPU over slices of one device A (bound in place, no
    copy), the per-iteration exchange summed here: exactly the per-rank shapes and the exchange
    protocol of an N = world run (only the transport differs from RCCL)."""
    from convex_optimization_amd import distributed as D
    from convex_optimization_amd.gpu_calculation import GPU_Calculation
    cls = type("GC_float", (GPU_Calculation,), {"TYPE": "float"})
    m = A_dev.shape[0]
    ranks = []
    for g in range(world):
        s, e = D.row_bounds(m, g, world)
        gc = cls(A_dev[s:e], 1, device=0, shard="rows")
        assert gc._A_dev.data_ptr() == A_dev[s:e].data_ptr()      # bound in place
        gc.set_ranks(g, world)
        gc.set_tuning("onepass_refresh", refresh)
        ranks.append(gc)
    diag = sum(gc._diag.clone() for gc in ranks)
    for g, gc in enumerate(ranks):
        s, e = D.row_bounds(m, g, world)
        gc.set_diag(diag)
        gc.solver_reset(b[s:e], mu, use_graph=False)

    def exchange():
        torch.cuda.synchronize()
        total = sum(gc.exchange_buffer().clone() for gc in ranks)
        for gc in ranks:
            gc.exchange_buffer().copy_(total)
        torch.cuda.synchronize()

    for phases in ((2, 3),) + ((0, 1),) * iters:
        for gc in ranks:
            gc.solver_phase(phases[0])
        exchange()
        for gc in ranks:
            gc.solver_phase(phases[1])
    return ranks


@pytest.mark.timeout(900)
def test_config2_full_problem_one_gpu_and_eight_row_ranks():
    """configs[2] (8192 x 524288 fp32, 16 GiB): the whole problem on one GPU (one pass, 128
    segment blocks per row = two hand-off granules per lane) against the oracle, and the
    eight per-rank shapes of the N = 8 row split (1024 x 524288 each, the caller-summed
    exchange of [U | r.s23 | s23.s23 | failed]) against the one-GPU run"""
    m, n, IT = 8192, 524288, 4
    gc, b, mu, _ = device_instance(m, n, 0.4, 1, TYPE="float", seed=37, device=0)
    one = gc.run(b, mu, IT)
    assert gc.solver_stat("onepass") == 1
    ranks = _external_rows(gc._A_dev, b, mu, 8, IT)
    xs = [r.solver_x() for r in ranks]
    for x in xs[1:]:
        np.testing.assert_array_equal(x, xs[0])
    e8 = rel(xs[0], one["x"])
    del ranks
    A = np.ascontiguousarray(gc.A_b_gpu[0].cpu().numpy())
    ref = oracle.run(A, b.cpu().numpy(), mu, 1, IT, nthreads=16)
    e1 = rel(one["x"], ref["x"])
    print(f"configs[2] {m}x{n}, {IT} iterations: one GPU vs oracle {e1:.3e}, 8 row ranks vs one GPU {e8:.3e}")
    assert e1 <= 1e-9, e1
    assert e8 <= 1e-10, e8


def _pin_torch_restatement():
    """the torch fp64 restatement equals the C oracle (same algorithm; summation order only)"""
    from torch_restatement import run_torch
    rs = np.random.RandomState(3)
    A = rs.randn(512, 2048)
    A /= np.linalg.norm(A, axis=1, keepdims=True)
    A = A.astype(np.float32)
    b = rs.randn(512)
    mu = 0.1 * float(np.abs(A.astype(np.float64).T @ b).max())
    ref = oracle.run(A, b, mu, 1, 40, nthreads=16)
    got = run_torch(torch.from_numpy(A).cuda(), torch.from_numpy(b).cuda(), mu, 40)
    assert rel(got["x"].cpu().numpy(), ref["x"]) <= 1e-12
    np.testing.assert_allclose(got["err_iter"].cpu().numpy(), ref["err_iter"], rtol=1e-10, atol=1e-14)


@pytest.mark.timeout(900)
@pytest.mark.parametrize("m,n,seed", [(1048576, 4096, 41)])
def test_gaussian_recipe_260_iterations_full_size(m, n, seed):
    """configs[3] at full size (2^32 elements) on the BASELINE Gaussian recipe (configs[2]'s case moved
    to the C-oracle fixture below in round 6),
    260 iterations through the product path (one pass over A, exact gradient refresh at 256),
    against the torch fp64 restatement: x within 1e-5 relative l2, the error criterion trace within
    1e-4 relative (or 1e-6 of its first value absolute)."""
    from torch_restatement import run_torch
    _pin_torch_restatement()
    IT = 260
    gc, b, mu, _ = device_instance(m, n, 0.4, 1, TYPE="float", seed=seed, device=0)
    res = gc.run(b, mu, IT, record=True)
    assert gc.solver_stat("onepass") == 1 and gc.solver_stat("refreshes") == 1
    ref = run_torch(gc._A_dev, b, mu, IT)
    e = rel(res["x"], ref["x"].cpu().numpy())
    print(f"{m}x{n} Gaussian recipe, {IT} iterations: rel l2 vs torch fp64 restatement {e:.3e}")
    assert e <= 1e-5, e
    er = ref["err_iter"].cpu().numpy()
    np.testing.assert_allclose(res["err_iter"][:IT], er, rtol=1e-4, atol=1e-6 * er[0])


GOLDEN = __import__("os").path.join(__import__("os").path.dirname(__file__), "golden")


@pytest.mark.timeout(900)
@pytest.mark.parametrize("name", ["gauss_configs3", "gauss_configs2"])
def test_gaussian_recipe_against_c_oracle_fixture(name):
    """configs[3] (1048576 x 4096 fp32) and configs[2] (8192 x 524288 fp32), 2^32 elements each, on
    the reference's instance recipe (parameters.py:17-33; rows N(0, 1) with unit norm -- the
    Irwin-Hall draws of oracle/gauss_instance.c, bit-identical on every host) against the C oracle at
    full size: the instance is rebuilt here and proved identical to the build container's (A at 4096
    sample points, SHA-256 of b, mu), then 300 iterations through the product path (one pass over A,
    the exact gradient refresh at 256) are compared with the oracle's 300 (tests/golden/make_gauss.py):
    x within north_star's 1e-5 relative l2, the error-criterion trace within 1e-4 relative (or 1e-6
    of its first value absolute), the objective within 1e-10 relative."""
    import hashlib
    from convex_optimization_amd.gpu_calculation import GPU_Calculation
    fx = dict(np.load(__import__("os").path.join(GOLDEN, name + ".npz")))
    m, n, IT = int(fx["m"]), int(fx["n"]), int(fx["iters"])
    A, b, mu, _ = oracle.gauss_instance(int(fx["seed"]), m, n, float(fx["den"]), nthreads=16)
    assert np.array_equal(A[fx["A_rows"], fx["A_cols"]], fx["A_samples"])
    assert hashlib.sha256(b.tobytes()).digest() == bytes(fx["b_sha256"])
    assert mu == float(fx["mu"])
    Ad = torch.from_numpy(A).to("cuda:0")
    del A
    cls = type("GC_float", (GPU_Calculation,), {"TYPE": "float"})
    gc = cls(Ad, 1, device=0)
    bd = torch.from_numpy(b).to("cuda:0")
    res = gc.run(bd, mu, IT, record=True)
    assert gc.solver_stat("onepass") == 1 and gc.solver_stat("refreshes") == (IT - 1) // 256
    e = rel(res["x"], fx["x"])
    f = objective(gc, mu)
    print(f"{name}: {m} x {n} Gaussian recipe vs C oracle fixture, {IT} iterations: rel l2 {e:.3e}, "
          f"objective {abs(f - float(fx['objective'])) / float(fx['objective']):.3e}")
    assert e <= 1e-5, e
    assert abs(f - float(fx["objective"])) <= 1e-10 * float(fx["objective"])
    er = fx["err_iter"]
    np.testing.assert_allclose(res["err_iter"][:IT], er[:IT], rtol=1e-4, atol=1e-6 * er[0])
