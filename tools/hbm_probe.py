#!/usr/bin/env python3
"""Run the HBM read-ceiling probe (tools/hbm_probe.hip) on a 2 GiB buffer."""
import ctypes
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    import torch
    so = os.path.join(HERE, "_hbm_probe.so")
    if not os.path.exists(so):
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared", "-o", so,
                        os.path.join(HERE, "hbm_probe.hip")], check=True)
    L = ctypes.CDLL(so)
    L.probe_run.restype = ctypes.c_double
    L.probe_run.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                            ctypes.c_longlong, ctypes.c_void_p, ctypes.c_longlong, ctypes.c_int]
    nbytes = 8192 * 65536 * 4
    a = torch.randn(nbytes // 4, device="cuda")
    o = torch.empty_like(a) if "--copy" in sys.argv else a
    sink = torch.zeros(1 << 22, dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    for kind, unr, blocks in [(0, 4, 2048), (0, 8, 2048), (0, 16, 2048), (0, 8, 1024), (0, 8, 4096), (0, 8, 8192),
                              (1, 4, 2048), (1, 8, 2048), (1, 8, 4096), (2, 8, 2048), (2, 8, 4096),
                              (3, 4, 1024), (3, 4, 2048), (3, 4, 4096), (4, 4, 2048), (4, 8, 4096)]:
        if kind == 4 and o is a:
            continue
        ms = L.probe_run(kind, unr, blocks, a.data_ptr(), o.data_ptr(), nbytes, sink.data_ptr(), 65536, 10)
        moved = nbytes * (2 if kind == 4 else 1)
        print(json.dumps(dict(kind=kind, unroll=unr, blocks=blocks, ms=round(ms, 4),
                              GBps=round(moved / ms / 1e6, 1))), flush=True)


if __name__ == "__main__":
    main()
