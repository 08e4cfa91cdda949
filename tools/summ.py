"""Print one line per bench JSON (value, ms/step and the per-kernel event averages in us)."""
import glob
import json
import sys

for pat in sys.argv[1:]:
    for f in sorted(glob.glob(pat)):
        try:
            d = json.loads(open(f).readline())
        except Exception:
            print(f, "no JSON line")
            continue
        c = d.get("config", {})
        k = c.get("kernel_avg_ms", {})
        ks = " ".join(f"{n} {v * 1e3:.1f}" for n, v in k.items() if v)
        print(f"{f.split('/')[-1]:40s} {d['value']:9.1f} it/s  {d['ms_per_step'] * 1e3:8.1f} us/step  "
              f"frac {d.get('roofline', {}).get('frac', 0):.3f}  | {ks}")
