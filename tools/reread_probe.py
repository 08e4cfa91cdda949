#!/usr/bin/env python3
"""Run tools/reread_probe.hip on an 8192 x 65536 fp32 matrix: time of one streamed read of A
vs a read plus an immediate re-read of each tile, for several tile heights."""
import ctypes
import json
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    import torch
    so = os.path.join(HERE, "_reread_probe.so")
    if not os.path.exists(so):
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared", "-o", so,
                        os.path.join(HERE, "reread_probe.hip")], check=True)
    L = ctypes.CDLL(so)
    L.reread_run.restype = ctypes.c_double
    L.reread_run.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_longlong, ctypes.c_longlong,
                             ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
    m, lda = 8192, 65536
    a = torch.randn(m * lda, device="cuda")
    sink = torch.zeros(1 << 22, dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    nbytes = m * lda * 4
    for rows in (8, 16, 32, 64, 128, 512):
        for kind in (0, 1, 2, 3, 4):
            ms = L.reread_run(kind, 1024, a.data_ptr(), lda, m, rows, sink.data_ptr(), 10)
            print(json.dumps(dict(rows=rows, tile_KiB=rows * 4, kind=kind, ms=round(ms, 4),
                                  hbm_GBps_once=round(nbytes / ms / 1e6, 1))), flush=True)


if __name__ == "__main__":
    main()
