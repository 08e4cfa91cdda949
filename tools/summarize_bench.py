"""One line per bench JSON file: workload, it/s, iteration roofline fraction, dominant kernel."""
import json
import sys

for path in sys.argv[1:]:
    try:
        d = json.load(open(path))
    except Exception as e:   # noqa: BLE001
        print(f"{path}: unreadable ({e})")
        continue
    c, r = d["config"], d["roofline"]
    frac = c.get("iter_roofline_frac")
    km = {k: round(v * 1e3, 1) for k, v in c.get("kernel_avg_ms", {}).items() if isinstance(v, float) and v}
    print(f"{path.split('/')[-1]:32s} {d['value']:10.1f} {d['unit'][:14]:14s} iter_frac={frac if frac is None else round(frac, 3)} "
          f"{r['kernel'].split()[0]} {r['frac']:.3f} us={km}")
