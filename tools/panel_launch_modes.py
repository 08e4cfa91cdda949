"""Panel path (configs[4] shape): iterations/s under the three launch modes -- hipGraph replay,
plain eager launches, eager launches with HIP events around every kernel -- on one A.
Usage (GPU box): python tools/panel_launch_modes.py [steps]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from convex_optimization_amd.panel import PanelLasso  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 96
    m, n, k = 8192, 65536, 128
    torch.cuda.set_device(0)
    g = torch.Generator(device="cuda").manual_seed(20190325)
    A = torch.randn(m, n, device="cuda", generator=g)
    A /= A.norm(dim=1, keepdim=True)
    Xt = torch.randn(n, k, device="cuda", generator=g) * (torch.rand(n, k, device="cuda", generator=g) < 0.4)
    pl = PanelLasso(A, 1, nrhs=k, device=0)
    del A
    Ab = pl.A_bf16.float()
    B = (Ab @ Xt + 0.01 * torch.randn(m, k, device="cuda", generator=g)).double()
    mu = (0.1 * (Ab.t() @ B.float()).abs().amax(dim=0)).double().cpu().numpy()
    del Ab
    out = {}
    for mode in ("graph", "eager", "events", "graph", "eager"):
        pl.solver_reset(B, mu, use_graph=(mode == "graph"))
        pl.set_kernel_timing(mode == "events")
        pl.solver_step(8)
        pl.stream.synchronize()
        t0 = time.perf_counter()
        pl.solver_step(steps)
        pl.stream.synchronize()
        el = time.perf_counter() - t0
        out.setdefault(mode, []).append(round(steps / el, 1))
        if mode == "events":
            out["events_kernel_ms"] = {a: round(b, 4) for a, b in pl.kernel_times()[0].items()}
        pl.set_kernel_timing(False)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
