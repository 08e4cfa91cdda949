#!/usr/bin/env python3
"""Run tools/regpass_probe.hip at configs[1] size for several register-pipeline shapes and tile
counts; check the two products against torch (stand-in s = 1e-3 x row partial)."""
import ctypes
import json
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    import torch
    so = os.path.join(HERE, "_regpass_probe.so")
    if not os.path.exists(so):
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                        "-o", so, os.path.join(HERE, "regpass_probe.hip")], check=True)
    L = ctypes.CDLL(so)
    L.regpass_run.restype = ctypes.c_double
    L.regpass_run.argtypes = [ctypes.c_void_p, ctypes.c_longlong, ctypes.c_longlong, ctypes.c_longlong, ctypes.c_int,
                              ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    m, n = 8192, 65536
    nseg = n // 1024
    g = torch.Generator(device="cuda").manual_seed(3)
    A = torch.randn(m, n, device="cuda", generator=g)
    D = torch.randn(n, device="cuda", dtype=torch.float64, generator=g)
    Ad = A.double()
    partref = (Ad.view(m, nseg, 1024) * D.view(1, nseg, 1024)).sum(dim=2)          # [m][nseg]
    for nchunk in (4, 8):
        part = torch.zeros(m * nseg, device="cuda", dtype=torch.float64)
        Us = torch.zeros(nchunk * 4 * n, device="cuda", dtype=torch.float64)
        for variant in range(4):
            ms = L.regpass_run(A.data_ptr(), n, m, n, nchunk, D.data_ptr(), part.data_ptr(), Us.data_ptr(), 10, variant)
            torch.cuda.synchronize()
            pr = part.view(m, nseg)
            U = Us.view(nchunk * 4, n).sum(dim=0)
            # stand-in s for (row, seg) = 1e-3 * partial of that row and segment
            Uref = (Ad.view(m, nseg, 1024) * (1e-3 * partref).view(m, nseg, 1)).sum(dim=0).reshape(-1)
            print(json.dumps({"nchunk": nchunk, "variant": variant, "ms": ms, "GBps": m * n * 4 / ms / 1e6,
                              "part_rel": float((pr - partref).norm() / partref.norm()),
                              "U_rel": float((U - Uref).norm() / Uref.norm())}), flush=True)


if __name__ == "__main__":
    main()
