#!/usr/bin/env python3
"""Run tools/onepass5_probe.hip at configs[1] size: S = A D and U = A^T S in one HBM pass
(deep register delay line, one-hop exchange), checked against torch fp64; timed."""
import ctypes
import json
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    import torch
    so = os.path.join(HERE, "_onepass5_probe.so")
    if not os.path.exists(so):
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                        "-o", so, os.path.join(HERE, "onepass5_probe.hip")], check=True)
    L = ctypes.CDLL(so)
    L.onepass5_run.restype = ctypes.c_double
    L.onepass5_run.argtypes = [ctypes.c_void_p, ctypes.c_longlong, ctypes.c_longlong, ctypes.c_longlong, ctypes.c_int,
                               ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                               ctypes.c_void_p, ctypes.c_int, ctypes.c_uint, ctypes.c_int,
                               ctypes.POINTER(ctypes.c_int)]
    m, n = 8192, 65536
    nseg = n // 1024
    g = torch.Generator(device="cuda").manual_seed(3)
    A = torch.randn(m, n, device="cuda", generator=g)
    D = torch.randn(n, device="cuda", dtype=torch.float64, generator=g)
    Sref = A.double() @ D
    Uref = A.double().t() @ Sref
    PG = torch.zeros(2 * m * 64, device="cuda", dtype=torch.int64)
    err = torch.zeros(1, device="cuda", dtype=torch.int32)
    res = ctypes.c_int()
    tag = 1
    for variant in range(10):
        nchunk = 4
        S = torch.zeros(m, device="cuda", dtype=torch.float64)
        Us = torch.zeros(nchunk * 4 * n, device="cuda", dtype=torch.float64)
        err.zero_()
        ms = L.onepass5_run(A.data_ptr(), n, m, n, nchunk, D.data_ptr(), PG.data_ptr(),
                            S.data_ptr(), Us.data_ptr(), err.data_ptr(), 10, tag, variant, ctypes.byref(res))
        tag += 20
        torch.cuda.synchronize()
        U = Us.view(-1, n).sum(dim=0)
        print(json.dumps({"variant": variant, "nchunk": nchunk, "resident_blocks": res.value, "ms": ms,
                          "err": int(err.item()), "GBps_one_pass": m * n * 4 / ms / 1e6 if ms > 0 else None,
                          "S_rel": float((S - Sref).norm() / Sref.norm()),
                          "U_rel": float((U - Uref).norm() / Uref.norm())}), flush=True)


if __name__ == "__main__":
    main()
