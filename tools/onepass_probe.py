#!/usr/bin/env python3
"""Run tools/onepass_probe.hip at configs[1] size: check S = A D and U = A^T S against torch
fp64 and time the single pass (compare: two streamed passes ~630 us)."""
import ctypes
import json
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    import torch
    so = os.path.join(HERE, "_onepass_probe.so")
    if not os.path.exists(so):
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                        "-o", so, os.path.join(HERE, "onepass_probe.hip")], check=True)
    L = ctypes.CDLL(so)
    L.onepass_run.restype = ctypes.c_double
    L.onepass_run.argtypes = [ctypes.c_void_p, ctypes.c_longlong, ctypes.c_longlong, ctypes.c_void_p, ctypes.c_void_p,
                              ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_uint,
                              ctypes.c_int]
    m, n = 8192, 65536
    g = torch.Generator(device="cuda").manual_seed(3)
    A = torch.randn(m, n, device="cuda", generator=g)
    D = torch.randn(n, device="cuda", dtype=torch.float64, generator=g)
    S = torch.zeros(m, device="cuda", dtype=torch.float64)
    Ug = torch.zeros(8, n, device="cuda", dtype=torch.float64)
    gran = torch.zeros(m * 32 * 2, device="cuda", dtype=torch.int64)
    err = torch.zeros(1, device="cuda", dtype=torch.int32)
    torch.cuda.synchronize()
    Sref = A.double() @ D
    Uref = A.double().t() @ Sref
    tag = 1
    for variant in range(7):
        gran.zero_(); err.zero_(); S.zero_(); Ug.zero_()
        ms = L.onepass_run(A.data_ptr(), n, m, D.data_ptr(), S.data_ptr(), Ug.data_ptr(), gran.data_ptr(),
                           err.data_ptr(), 10, tag, variant)
        tag += 20
        torch.cuda.synchronize()
        U = Ug.sum(dim=0)
        out = {"variant": variant, "ms": ms, "err": int(err.item()),
               "S_rel": float((S - Sref).norm() / Sref.norm()), "U_rel": float((U - Uref).norm() / Uref.norm()),
               "hbm_GBps_one_pass": m * n * 4 / ms / 1e6}
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
