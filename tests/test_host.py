"""Host-side logic of the package (no GPU): cpu_calculation mirror, block orders,
instance generator, drivers over a numpy stand-in for GPU_Calculation."""
import random

import numpy as np
import pytest

from conftest import golden_cases
from convex_optimization_amd import cpu_calculation as cc
from convex_optimization_amd import lasso, parameters
from oracle import oracle


def test_cpu_calculation_kats(golden):
    k = golden("kats")
    np.testing.assert_array_equal(cc.soft_thresholding(k["t"], float(k["tau"])), k["soft"])
    np.testing.assert_array_equal(cc.element_proj(k["v"], -0.3, 0.5), k["proj"])
    assert cc.error_crit(k["g"], k["x"], float(k["mu"])) == float(k["err"])
    A_bp = cc.A_bp_get(k["A"], int(k["BLOCK"]), int(k["P"]))
    np.testing.assert_array_equal(A_bp, k["A_bp"])
    P = int(k["P"])
    np.testing.assert_allclose(np.stack([cc.fun_s12(A_bp[0, p], k["s11"]) for p in range(P)]), k["s12"],
                               rtol=1e-13)
    np.testing.assert_allclose(cc.fun_diag_ATA(A_bp), k["diag"], rtol=1e-13)
    dd = cc.fun_dd_p(P, k["d"])
    np.testing.assert_array_equal(dd, k["dd_p"])
    np.testing.assert_allclose(np.stack([cc.fun_s22(A_bp[1, p], dd[p]) for p in range(P)]), k["s22"],
                               rtol=1e-12, atol=1e-14)


def test_A_bp_get_rejects_ragged():
    with pytest.raises(ValueError):
        cc.A_bp_get(np.zeros((4, 10)), 3, 1)


def test_shuffled_order_matches_reference(golden):
    fx = golden("random_b4_p1_f32in")
    order = lasso.shuffled_order(int(fx["BLOCK"]), int(fx["ITER_MAX"]), random.Random(5))
    np.testing.assert_array_equal(order, fx["order"])


def test_cyclic_order():
    np.testing.assert_array_equal(lasso.cyclic_order(3, 7), [0, 1, 2, 0, 1, 2, 0])


@pytest.mark.parametrize("case", ["c1_b1_p1_f64", "c1_b2_p4_f64"])
def test_parameters_reproduce_reference_instance(golden, case):
    fx = golden(case)
    A, x_true, b, mu = parameters.parameters(int(fx["N"]), int(fx["K"]), float(fx["den"]), SILENCE=True,
                                             seed=int(fx["seed"]))
    np.testing.assert_array_equal(b, fx["b"])
    assert mu == float(fx["mu"])


def test_parameters_text_roundtrip(tmp_path):
    A, x_true, b, mu = parameters.parameters(12, 24, 0.5, SAVE_FLAG=True, SILENCE=True, seed=3,
                                             directory=str(tmp_path))
    A2, x2, b2, mu2 = parameters.parameters(0, 0, 0, READ_FLAG=True, SILENCE=True, directory=str(tmp_path))
    np.testing.assert_allclose(A2, A, rtol=1e-15)
    np.testing.assert_allclose(b2, b, rtol=1e-15)
    assert abs(mu2 - mu) <= 1e-15 * mu


class NumpyGemv:
    """Test double with GPU_Calculation's GEMV surface, computed by the oracle."""

    def __init__(self, A, Block):
        self.A = A
        self.Block = Block
        self.MAT_HEIGHT, self.MAT_WIDTH = A.shape[0], A.shape[1] // Block

    def mat_tMulVec_DiffSize(self, s13, m, s11):
        W = self.MAT_WIDTH
        s13[...] = oracle.mtv(self.A, m * W, W, s11).reshape(s13.shape)

    def matMulVec_DiffSize(self, s23, m, d):
        W = self.MAT_WIDTH
        s23[...] = oracle.mv(self.A, m * W, W, d).reshape(s23.shape)


@pytest.mark.parametrize("case", golden_cases())
def test_hybrid_driver_semantics(golden, case):
    """lasso.ClassLasso(R) over a numpy GEMV stand-in reproduces the reference run."""
    fx = golden(case)
    A = oracle.fixture_A(fx)
    BLOCK, IT = int(fx["BLOCK"]), int(fx["ITER_MAX"])
    gc = NumpyGemv(A, BLOCK)
    d = oracle.diag_ata(A, BLOCK)
    if bool(fx["random_order"]):
        random.seed(int(fx.get("py_seed", 5)))
        drv = lasso.ClassLassoR(gc, d, A, fx["b"], float(fx["mu"]), BLOCK, IT)
    else:
        drv = lasso.ClassLasso(gc, d, A, fx["b"], float(fx["mu"]), BLOCK, IT)
    err_iter, time_iter = np.zeros(IT), np.zeros(IT + 1)
    eb = None if fx["err_bound"] < 0 else float(fx["err_bound"])
    drv.run(ERR_BOUND=eb, err_iter=err_iter, time_iter=time_iter, SILENCE=True)
    x = fx["x"].reshape(-1)
    assert drv.iters == int(fx["t_last"]) + 1
    assert np.linalg.norm(drv.x.reshape(-1) - x) <= 1e-9 * np.linalg.norm(x)
    T = drv.iters
    np.testing.assert_allclose(err_iter[:T], fx["err_iter"][:T], rtol=1e-4, atol=1e-10)


def test_results_files_roundtrip_and_figure(tmp_path):
    from convex_optimization_amd import results
    IT = 10
    time_iter = np.linspace(0, 1, IT + 1)
    err_iter = np.logspace(0, -5, IT)
    results.save_performance("GPU", time_iter, err_iter, directory=str(tmp_path), iters=7)
    results.save_performance("CPU", time_iter * 3, err_iter, directory=str(tmp_path))
    data = results.load_performance(str(tmp_path))
    np.testing.assert_array_equal(data["gpu_time"], time_iter[1:8])
    np.testing.assert_array_equal(data["gpu_errors"], err_iter[:7])
    assert data["cpu_time"].shape == (IT,)
    png = results.compare_figure(str(tmp_path))
    assert (tmp_path / "compare.png").exists() and png.endswith("compare.png")

