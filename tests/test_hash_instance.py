"""The long-horizon fixtures' instance generator (tests/hash_instance.py): numpy and torch build the
same A and b bit for bit, b is exact whatever the summation order, and every committed
tests/golden/longrun_*.npz matches the generator at its stored sample points (CPU only)."""
import glob
import os

import numpy as np

import hash_instance as H

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_numpy_and_torch_agree_bitwise():
    import torch
    A = H.np_A(300, 1000)
    b = H.np_b(A)
    At = H.torch_A(300, 1000, "cpu")
    assert torch.equal(At, torch.from_numpy(A))
    assert np.array_equal(H.torch_b(At).numpy(), b)
    rows, cols = H.sample_points(300, 1000, k=64)
    assert np.array_equal(H.np_entries(rows, cols, 1000), A[rows, cols])
    Ab = H.np_A_bf16(300, 1000)
    assert torch.equal(H.torch_A_bf16(300, 1000, "cpu"), torch.from_numpy(Ab))
    assert np.array_equal(H.np_entries_bf16(rows, cols, 1000), Ab[rows, cols])
    assert torch.equal(torch.from_numpy(Ab).to(torch.bfloat16).float(), torch.from_numpy(Ab))   # exact in bf16
    B = H.torch_B(torch.from_numpy(Ab), 3)
    assert all(np.array_equal(B[:, r].numpy(), H.np_b_rhs(Ab, r)) for r in range(3))


def test_row_shards_are_slices_of_the_instance():
    """torch_A / torch_b of a row shard (the RCCL long-horizon test's ranks build only their rows) are
    the rows of the whole instance's A and b, bit for bit"""
    import torch
    A = H.np_A(300, 1000)
    b = H.np_b(A)
    for r0, r1 in ((0, 150), (150, 300), (7, 11)):
        As = H.torch_A(r1 - r0, 1000, "cpu", chunk_rows=3, row0=r0)
        assert torch.equal(As, torch.from_numpy(A[r0:r1]))
        assert np.array_equal(H.torch_b(As, row0=r0, m_total=300).numpy(), b[r0:r1])


def test_b_is_exact_in_any_order():
    A = H.np_A(200, 4096)
    x = H.np_x_true(4096)
    b1 = H.np_b(A)
    b2 = A.astype(np.float64)[:, ::-1] @ x[::-1] + H.np_e(200)
    b3 = np.array([sum(float(a) * float(c) for a, c in zip(row[x != 0], x[x != 0])) for row in A[:5]])
    assert np.array_equal(b1, b2)
    assert np.array_equal(b1[:5] - H.np_e(200)[:5], b3)
    assert 0.3 < np.count_nonzero(x) / x.size < 0.5


def test_committed_fixtures_match_the_generator():
    for path in sorted(glob.glob(os.path.join(GOLD, "longrun_*.npz"))):
        fx = dict(np.load(path))
        n = int(fx["n"])
        assert int(fx["iters"]) >= 260, path
        if "rhs" in fx:   # configs[4]: bf16 A, the oracle's RHS
            assert np.array_equal(H.np_entries_bf16(fx["A_rows"], fx["A_cols"], n), fx["A_samples"]), path
            for r in fx["rhs"]:
                x = fx[f"x_{r}"]
                assert x.shape == (n,) and np.isfinite(x).all()
                assert fx[f"err_iter_{r}"][-1] < fx[f"err_iter_{r}"][0]
            continue
        assert np.array_equal(H.np_entries(fx["A_rows"], fx["A_cols"], n), fx["A_samples"]), path
        assert fx["x"].shape == (n,) and np.isfinite(fx["x"]).all()
        assert fx["err_iter"][-1] < fx["err_iter"][0]
