"""The oracle (C + numpy restatements) pinned against the reference's own outputs.

Fixtures: tests/golden/*.npz, written by tests/golden/make_golden.py, which ran
the reference's ClassLassoCPU (lasso.py:25-169) and cpu_calculation.py in the
build container.
"""
import numpy as np
import pytest

from conftest import golden_cases
from oracle import oracle

# The reference sums with OpenBLAS dgemv / numpy pairwise order; the restatement
# sums in a fixed row order.  Both are fp64: the measured gap is <= 1e-10.
X_TOL = 1e-9


def _run_args(fx):
    order = fx["order"] if bool(fx["random_order"]) else None
    if order is not None and len(order) < int(fx["ITER_MAX"]):
        # a run that stopped early captured only the blocks it updated; the padding (the last block,
        # as the device reads a short order) is never reached when the stop is reproduced
        order = np.concatenate([order, np.full(int(fx["ITER_MAX"]) - len(order), order[-1], dtype=order.dtype)])
    eb = None if fx["err_bound"] < 0 else float(fx["err_bound"])
    return order, eb


@pytest.mark.parametrize("case", golden_cases())
def test_c_oracle_matches_reference(golden, case):
    fx = golden(case)
    A = oracle.fixture_A(fx)
    order, eb = _run_args(fx)
    res = oracle.run(A, fx["b"], fx["mu"], int(fx["BLOCK"]), int(fx["ITER_MAX"]), P=int(fx["P"]),
                     order=order, err_bound=eb)
    x = fx["x"].reshape(-1)
    assert res["t_last"] == int(fx["t_last"])
    assert np.linalg.norm(res["x"] - x) <= X_TOL * np.linalg.norm(x)
    T = int(fx["t_last"]) + 1
    np.testing.assert_allclose(res["err_iter"][:T], fx["err_iter"][:T], rtol=1e-4, atol=1e-10)


@pytest.mark.parametrize("case", golden_cases())
def test_numpy_oracle_matches_reference(golden, case):
    fx = golden(case)
    A = oracle.fixture_A(fx)
    order, eb = _run_args(fx)
    res = oracle.run_numpy(A, fx["b"], fx["mu"], int(fx["BLOCK"]), int(fx["ITER_MAX"]),
                           order=order, err_bound=eb)
    x = fx["x"].reshape(-1)
    assert res["t_last"] == int(fx["t_last"])
    assert np.linalg.norm(res["x"] - x) <= X_TOL * np.linalg.norm(x)


@pytest.mark.parametrize("case", ["c1_b1_p1_f32in", "c1_b2_p4_f32in"])
def test_numpy_fp32_gemv_variant_within_stated_tolerance(golden, case):
    """the CPU-baseline variant with fp32 GEMVs (the reference's TYPE='float' CPU path):
    x within the north_star 1e-5 of the reference run (SURVEY 8c measured 1.6-2.4e-6 for fp32 storage)"""
    fx = golden(case)
    A = oracle.fixture_A(fx).astype(np.float32)
    res = oracle.run_numpy(A, fx["b"], fx["mu"], int(fx["BLOCK"]), int(fx["ITER_MAX"]), gemv_f32=True)
    x = fx["x"].reshape(-1)
    assert np.linalg.norm(res["x"] - x) <= 1e-5 * np.linalg.norm(x), np.linalg.norm(res["x"] - x) / np.linalg.norm(x)


@pytest.mark.parametrize("case", ["c1_b1_p1_f32in", "ragged_b3_p2_f32in"])
def test_c_oracle_fp32_storage_is_exact(golden, case):
    """fp32-rounded fixtures: storing A as float32 changes nothing (same values)."""
    fx = golden(case)
    A = oracle.fixture_A(fx)
    r64 = oracle.run(A, fx["b"], fx["mu"], int(fx["BLOCK"]), 40, P=int(fx["P"]))
    r32 = oracle.run(A.astype(np.float32), fx["b"], fx["mu"], int(fx["BLOCK"]), 40, P=int(fx["P"]))
    np.testing.assert_array_equal(r64["x"], r32["x"])


def test_c_oracle_thread_count_invariant(golden):
    fx = golden("c1_b2_p4_f64")
    A = oracle.fixture_A(fx)
    a = oracle.run(A, fx["b"], fx["mu"], 2, 30, P=4, nthreads=1)
    b = oracle.run(A, fx["b"], fx["mu"], 2, 30, P=4, nthreads=5)
    np.testing.assert_array_equal(a["x"], b["x"])


def test_oracle_kernels_match_reference_kats(golden):
    k = golden("kats")
    A, BLOCK, P = k["A"], int(k["BLOCK"]), int(k["P"])
    K = A.shape[1]
    w, ws = K // BLOCK, K // (BLOCK * P)
    # fun_diag_ATA
    np.testing.assert_allclose(oracle.diag_ata(A, BLOCK), k["diag"], rtol=1e-13)
    # fun_s12 per shard of block 0
    for p in range(P):
        np.testing.assert_allclose(oracle.mtv(A, p * ws, ws, k["s11"]), k["s12"][p].reshape(-1), rtol=1e-12)
    # sum over shards of fun_s22 of block 1 == oracle mv with P shards
    s = oracle.mv(A, w, w, k["d"], P=P)
    np.testing.assert_allclose(s, k["s22"].sum(axis=0).reshape(-1), rtol=1e-12, atol=1e-14)


def test_sharded_decomposition_equals_single(golden):
    """The P-shard (future multi-GPU) decomposition is numerically the single-shard algorithm."""
    fx = golden("c1_b1_p1_f32in")
    A = oracle.fixture_A(fx)
    a = oracle.run(A, fx["b"], fx["mu"], 1, 100, P=1)
    b = oracle.run(A, fx["b"], fx["mu"], 1, 100, P=8)
    assert np.linalg.norm(a["x"] - b["x"]) <= 1e-10 * np.linalg.norm(a["x"])


def test_dropin_run_of_reference_driver_is_bitwise():
    """tests/golden/dropin/*.npz: the reference's unmodified ClassLassoCPU (lasso.py:25-169, its
    Pool included) run with sys.modules["cpu_calculation"] bound to this repository's
    convex_optimization_amd.cpu_calculation (tests/golden/dropin_proof.py, build container only).
    Every array -- x, err_iter, t_last, the block order, d_ATA, b, mu -- equals the fixture of the
    run on the reference's own cpu_calculation.py bit for bit."""
    import os
    import numpy as np
    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    names = sorted(f for f in os.listdir(os.path.join(here, "dropin")) if f.endswith(".npz"))
    # every reference-run case (rounds 1-5: 7; round 6: + 3 one-pass stop pins, 2 shuffled-order stops, a ragged stop)
    assert names == sorted(c + ".npz" for c in golden_cases())
    for name in names:
        a = np.load(os.path.join(here, "dropin", name))
        b = np.load(os.path.join(here, name))
        assert sorted(a.files) == sorted(b.files)
        for k in b.files:
            np.testing.assert_array_equal(a[k], b[k], err_msg=f"{name}:{k}")


def test_gauss_instance_is_deterministic_and_gaussian():
    """oracle/gauss_instance.c (the Gaussian-recipe instance of the full-size fixture): the same bits
    for any thread count and from the row-slice generator, rows of unit l2 norm, N(0, 1)-like
    entries (Irwin-Hall: mean 0, kurtosis 2.9 against 3), density 0.4 of x_true"""
    A1, b1, mu1, x1 = oracle.gauss_instance(7, 512, 1024, nthreads=1)
    A2, b2, mu2, x2 = oracle.gauss_instance(7, 512, 1024, nthreads=5)
    assert np.array_equal(A1, A2) and np.array_equal(b1, b2) and mu1 == mu2 and np.array_equal(x1, x2)
    assert np.array_equal(oracle.gauss_rows(7, 100, 3, 1024), A1[100:103])
    np.testing.assert_allclose(np.linalg.norm(A1.astype(np.float64), axis=1), 1.0, rtol=1e-6)
    z = A1.astype(np.float64).reshape(-1) * np.sqrt(1024)
    assert abs(z.mean()) < 0.01 and abs(z.var() - 1) < 0.01
    assert 2.8 < ((z - z.mean()) ** 4).mean() / z.var() ** 2 < 3.0
    assert abs((x1 != 0).mean() - 0.4) < 0.05
    assert not np.array_equal(A1, oracle.gauss_instance(8, 512, 1024)[0])


@pytest.mark.parametrize("name", ["gauss_configs3", "gauss_configs2"])
def test_gauss_fixture_samples_match_the_generator(name):
    """tests/golden/gauss_configs{3,2}.npz (configs[3] / configs[2] at full size, C oracle,
    tests/golden/make_gauss.py) were made from this generator: their stored A samples of 64 rows are
    regenerated bit for bit"""
    import os
    path = os.path.join(os.path.dirname(__file__), "golden", name + ".npz")
    fx = dict(np.load(path))
    n, seed = int(fx["n"]), int(fx["seed"])
    for r, c, v in list(zip(fx["A_rows"], fx["A_cols"], fx["A_samples"]))[:64]:
        assert oracle.gauss_rows(seed, int(r), 1, n)[0, int(c)] == v
    assert fx["x"].shape == (n,) and int(fx["iters"]) >= 260 and np.isfinite(fx["objective"])
