#!/usr/bin/env python3
"""Run tools/onepass6_probe.hip at configs[1] size: S = A D and U = A^T S in one HBM pass
(block-combined partials, XCD-local row groups), checked against torch fp64; timed."""
import ctypes
import json
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    import torch
    so = os.path.join(HERE, "_onepass6_probe.so")
    if not os.path.exists(so):
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                        "-o", so, os.path.join(HERE, "onepass6_probe.hip")], check=True)
    L = ctypes.CDLL(so)
    L.onepass6_run.restype = ctypes.c_double
    L.onepass6_run.argtypes = [ctypes.c_void_p, ctypes.c_longlong, ctypes.c_longlong, ctypes.c_longlong,
                               ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                               ctypes.c_int, ctypes.c_uint, ctypes.c_int, ctypes.POINTER(ctypes.c_int),
                               ctypes.c_void_p]
    m, n = 8192, 65536
    g = torch.Generator(device="cuda").manual_seed(3)
    A = torch.randn(m, n, device="cuda", generator=g)
    D = torch.randn(n, device="cuda", dtype=torch.float64, generator=g)
    Sref = A.double() @ D
    Uref = A.double().t() @ Sref
    PG = torch.zeros(m * 16, device="cuda", dtype=torch.int64)
    err = torch.zeros(1, device="cuda", dtype=torch.int32)
    res = ctypes.c_int()
    stats = torch.zeros(8, device="cuda", dtype=torch.int64)
    tag = 1
    for rep in range(2):
        for variant in range(8):
            S = torch.zeros(m, device="cuda", dtype=torch.float64)
            Us = torch.zeros(16 * n, device="cuda", dtype=torch.float64)
            err.zero_()
            stats.zero_()
            ms = L.onepass6_run(A.data_ptr(), n, m, n, D.data_ptr(), PG.data_ptr(), S.data_ptr(), Us.data_ptr(),
                                err.data_ptr(), 10, tag, variant, ctypes.byref(res), stats.data_ptr())
            tag += 20
            torch.cuda.synchronize()
            U = Us.view(-1, n).sum(dim=0)
            st = stats.tolist()
            nw = 12 * 1024
            print(json.dumps({"variant": variant, "rep": rep, "resident_blocks": res.value, "ms": ms,
                              "err": int(err.item()), "GBps_one_pass": m * n * 4 / ms / 1e6 if ms > 0 else None,
                              "S_rel": float((S - Sref).norm() / Sref.norm()),
                              "U_rel": float((U - Uref).norm() / Uref.norm()),
                              # per wave and launch (12 launches); realtime ticks are 10 ns
                              "late_per_wave": st[0] / nw, "late_wait_us_per_wave": st[1] / nw / 100,
                              "pubspin_per_wave": st[2] / nw, "pubspin_us_per_wave": st[3] / nw / 100,
                              "wave_us_avg": st[4] / nw / 100, "wave_us_max": st[5] / 100}), flush=True)


if __name__ == "__main__":
    main()
