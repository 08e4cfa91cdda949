"""The drop-in boundary used from plain C (examples/bpgl_solve.c): no Python, no PyTorch in the caller.

The program allocates device memory itself, binds A in the reference's np.hsplit layout
(gpu_calculation.py:172-173), computes diag(A^T A) and runs bpgl_iterate with the reference's
ERR_BOUND rule -- the calls a non-Python binding of GPU_Calculation / ClassLassoCB_v2 would make
(INTEGRATION.md).  CPU: it builds, links libbpgl.so and the HIP runtime and nothing of Python or
torch, and rejects a bad command line before touching the GPU.  GPU: on reference-run fixtures
(one block with an ERR_BOUND stop on the one-pass path; two blocks on the two-pass path) x within
1e-9 of the reference, the stop iteration exact, the error record within 1e-6 relative.
"""
import os
import subprocess

import numpy as np
import pytest

from oracle import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "examples", "bpgl_solve")


def _build():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "examples")], check=True)
    return EXE


def test_c_caller_builds_and_links_only_the_library():
    exe = _build()
    libs = subprocess.run(["ldd", exe], capture_output=True, text=True, check=True).stdout
    assert "libbpgl.so" in libs and "libamdhip64" in libs
    assert "torch" not in libs and "python" not in libs
    p = subprocess.run([exe], capture_output=True, text=True)
    assert p.returncode == 2 and "usage" in p.stderr
    p = subprocess.run([exe, "A", "b", "4", "6", "4", "0.1", "10", "-1", "x", "e"], capture_output=True, text=True)
    assert p.returncode == 2 and "bad shape" in p.stderr      # n % nblock != 0


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["stop511_b1_p1_f32in", "c1_b2_p4_f32in"])
def test_c_caller_reproduces_reference_run(golden, case, tmp_path):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    fx = golden(case)
    A = oracle.fixture_A(fx).astype(np.float32)
    m, n = A.shape
    IT, BLOCK = int(fx["ITER_MAX"]), int(fx["BLOCK"])
    A.tofile(tmp_path / "A.f32")
    np.asarray(fx["b"], dtype=np.float64).reshape(-1).tofile(tmp_path / "b.f64")
    p = subprocess.run([_build(), str(tmp_path / "A.f32"), str(tmp_path / "b.f64"), str(m), str(n), str(BLOCK),
                        repr(float(fx["mu"])), str(IT), repr(float(fx["err_bound"])), str(tmp_path / "x.f64"),
                        str(tmp_path / "e.f64")], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    done, stopped, t_last = (int(v) for v in p.stdout.split())
    assert t_last == int(fx["t_last"]) and bool(stopped) == bool(fx["stopped"]) and done == t_last + 1
    x = np.fromfile(tmp_path / "x.f64")
    ref = fx["x"].reshape(-1)
    assert np.linalg.norm(x - ref) <= 1e-9 * np.linalg.norm(ref)
    err = np.fromfile(tmp_path / "e.f64")
    np.testing.assert_allclose(err[:t_last + 1], fx["err_iter"][:t_last + 1], rtol=1e-6, atol=1e-12)
