"""The C-ABI library loads and exports every symbol include/bpgl.h declares.

CPU-only: no call here reaches the GPU (argument validation happens before any
HIP call, so invalid arguments are rejected on a machine without a device).
"""
import ctypes
import os

import pytest

from convex_optimization_amd import _native as N
from convex_optimization_amd import panel  # noqa: F401  (registers the bpgl_panel_* signatures)


def test_library_present_and_loads():
    assert os.path.exists(N.LIB_PATH), "run __graft_entry__.build() first"
    assert N.lib().bpgl_version() >= 200


def test_every_header_symbol_exported():
    names = N.header_functions()
    assert len(names) >= 20
    L = ctypes.CDLL(N.LIB_PATH)
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    # and the Python binding declares a signature for each of them
    assert set(names) == set(N._SIGS), set(names) ^ set(N._SIGS)


@pytest.mark.parametrize("args,code", [
    ((0, 9, 64, 64, 1), -1),     # unknown dtype
    ((0, 0, 0, 64, 1), -1),      # m == 0
    ((0, 0, 64, 65, 2), -1),     # n_local not divisible by nblock
    ((0, 0, 64, 64, 0), -1),     # nblock == 0
])
def test_create_rejects_bad_arguments(args, code):
    ctx = ctypes.c_void_p()
    rc = N.lib().bpgl_create(ctypes.byref(ctx), *args, None)
    assert rc == code
    assert ctx.value is None
    assert N.lib().bpgl_last_error().decode()


@pytest.mark.parametrize("args", [
    (0, 256, 256, 1, 48, 0),            # nrhs not 16 / 32 / 64 / 128
    (0, 200, 256, 1, 16, 0),            # m not a multiple of 256
    (0, 256, 512, 3, 16, 0),            # n not divisible by nblock
    (0, 256, 384, 1, 16, 0),            # block width not a multiple of 256
    (0, 256, 512, 1, 16, 3),            # w not a multiple of 64 * kchunks
    (0, 256, 1 << 24, 1, 128, 0),       # nrhs * w reaches 2^31
])
def test_panel_create_rejects_bad_arguments(args):
    """bpgl_panel_create checks its shape contract before any HIP call (include/bpgl.h)"""
    ctx = ctypes.c_void_p()
    rc = N.lib().bpgl_panel_create(ctypes.byref(ctx), *args, None)
    assert rc == -1
    assert ctx.value is None
    assert N.lib().bpgl_last_error().decode()


def test_null_context_is_an_error_not_a_crash():
    assert N.lib().bpgl_mtv(None, 0, None, None) == -1
    assert N.lib().bpgl_solver_step(None, 1) == -1
    assert N.lib().bpgl_scratch_bytes(None) == -1
    L = N.lib()
    assert L.bpgl_panel_scratch_bytes(None) == -1
    assert L.bpgl_panel_bind(None, None, 0, None, 0) == -1
    assert L.bpgl_panel_diag(None, None) == -1
    assert L.bpgl_panel_step(None, 1) == -1
    assert L.bpgl_panel_reset(None, None, None, None, 0, 0) == -1
    v = ctypes.c_int64()
    assert L.bpgl_panel_get_tuning(None, b"interleave1", ctypes.byref(v)) == -1
    assert L.bpgl_panel_set_tuning(None, b"interleave", 0) == -1


def test_dtype_names():
    assert N.dtype_code("double") == N.BPGL_F64
    assert N.dtype_code("float") == N.BPGL_F32
    assert N.dtype_code("bf16") == N.BPGL_BF16
    with pytest.raises(ValueError):
        N.dtype_code("int8")
