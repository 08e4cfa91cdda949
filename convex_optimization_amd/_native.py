"""ctypes binding of libbpgl.so (the C ABI declared in include/bpgl.h).

The HIP kernels are the only compute path of this package: if the in-tree
library is missing or fails to load, every GPU entry point raises instead of
falling back to anything else.

torch is imported before the library is loaded so that the HIP runtime and
RCCL the library links against (sonames libamdhip64.so.7 / librccl.so.1) are
resolved to the copies PyTorch already loaded -- one runtime per process.
"""
import ctypes
import os
import re

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

_HERE = os.path.dirname(os.path.abspath(__file__))
# BPGL_LIB: another in-tree build of the same library (diagnostic builds under build_diag/)
LIB_PATH = os.environ.get("BPGL_LIB") or os.path.join(_HERE, "_lib", "libbpgl.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "bpgl.h")

BPGL_F32, BPGL_F64, BPGL_BF16 = 0, 1, 2
BPGL_SHARD_COLUMNS, BPGL_SHARD_ROWS = 0, 1
_DTYPES = {
    "float": BPGL_F32, "float32": BPGL_F32, "f32": BPGL_F32,
    "double": BPGL_F64, "float64": BPGL_F64, "f64": BPGL_F64,
    "bf16": BPGL_BF16, "bfloat16": BPGL_BF16,
}
TORCH_DTYPE = {BPGL_F32: torch.float32, BPGL_F64: torch.float64, BPGL_BF16: torch.bfloat16}
VEC_ELEMS = {BPGL_F32: 4, BPGL_F64: 2, BPGL_BF16: 8}

_p = ctypes.c_void_p
_i64 = ctypes.c_int64
_i32 = ctypes.c_int32
_int = ctypes.c_int
_f64 = ctypes.c_double
_pp = ctypes.POINTER(ctypes.c_void_p)

_SIGS = {
    "bpgl_last_error": (ctypes.c_char_p, []),
    "bpgl_version": (_int, []),
    "bpgl_stream_create": (_int, [_int, ctypes.POINTER(ctypes.c_uint32), _i32, _pp]),
    "bpgl_stream_destroy": (_int, [_p]),
    "bpgl_create": (_int, [_pp, _int, _int, _i64, _i64, _i32, _p]),
    "bpgl_destroy": (None, [_p]),
    "bpgl_stream": (_p, [_p]),
    "bpgl_scratch_bytes": (_i64, [_p]),
    "bpgl_block_width_padded": (_i64, [_p]),
    "bpgl_bind": (_int, [_p, _p, _i64, _i64, _p, _i64]),
    "bpgl_diag_ata": (_int, [_p, _p]),
    "bpgl_set_diag": (_int, [_p, _p]),
    "bpgl_set_shard": (_int, [_p, _int]),
    "bpgl_mtv": (_int, [_p, _i32, _p, _p]),
    "bpgl_mv": (_int, [_p, _i32, _p, _p]),
    "bpgl_comm_unique_id": (_int, [_p]),
    "bpgl_comm_init": (_int, [_p, _p, _int, _int]),
    "bpgl_set_ranks": (_int, [_p, _int, _int]),
    "bpgl_solver_phase": (_int, [_p, _int]),
    "bpgl_solver_exchange_buffer": (_p, [_p, ctypes.POINTER(_i64)]),
    "bpgl_solver_reset": (_int, [_p, _p, _f64, _p, _p, _i64, _f64, _p, _p, _i64, _int]),
    "bpgl_solver_step": (_int, [_p, _i64]),
    "bpgl_solver_status": (_int, [_p, ctypes.POINTER(_i64), ctypes.POINTER(_int), ctypes.POINTER(_i64),
                                  ctypes.POINTER(_f64), ctypes.POINTER(_f64)]),
    "bpgl_solver_stat": (_int, [_p, ctypes.c_char_p, ctypes.POINTER(_i64)]),
    "bpgl_solver_residual": (_p, [_p]),
    "bpgl_iterate": (_int, [_p, _i64, _p, _f64, _p, _p, _p, _p, _f64, ctypes.POINTER(_i64)]),
    "bpgl_set_kernel_timing": (_int, [_p, _int]),
    "bpgl_set_tuning": (_int, [_p, ctypes.c_char_p, _i64]),
    "bpgl_kernel_times": (_int, [_p, ctypes.POINTER(_f64), ctypes.POINTER(_i64)]),
    "bpgl_geometry": (_int, [_p, ctypes.POINTER(_i32), ctypes.POINTER(_i32), ctypes.POINTER(_i32),
                             ctypes.POINTER(_i32)]),
}

_lib = None


def lib():
    """Load libbpgl.so once; raise loudly when it is absent."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                "(or `make -C convex_optimization_amd/csrc`). There is no fallback path.")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


class BpglError(RuntimeError):
    pass


def check(rc, what=""):
    if rc != 0:
        msg = lib().bpgl_last_error().decode(errors="replace")
        raise BpglError(f"{what} failed ({rc}): {msg}")


def dtype_code(type_name):
    key = str(type_name).lower().replace("torch.", "")
    if key not in _DTYPES:
        raise ValueError(f"unsupported TYPE {type_name!r}; use one of {sorted(_DTYPES)}")
    return _DTYPES[key]


def header_functions(path=HEADER_PATH):
    """Names of every function declared in include/bpgl.h."""
    text = open(path).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(bpgl_[a-z0-9_]+)\s*\(", text)))


def ptr(t):
    """Device/host address of a tensor (None -> NULL)."""
    return None if t is None else ctypes.c_void_p(t.data_ptr())
