"""Summarise tools/wide_sweep.sh: per run the iteration time and the k_onepass event average."""
import glob
import json
import os
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/wide_sweep"
for f in sorted(glob.glob(os.path.join(d, "*.json"))):
    try:
        j = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:   # noqa: BLE001
        print(os.path.basename(f), "unreadable", e)
        continue
    k = j["config"].get("kernel_avg_ms", {})
    print(f"{os.path.basename(f)[:-5]:28s} us/it {1e3 * j['ms_per_step']:8.2f}  onepass {1e3 * k.get('onepass', 0):8.2f}"
          f"  fold {1e3 * k.get('rowreduce', 0):6.2f}  tail {1e3 * k.get('update', 0):6.2f}"
          f"  fallbacks {j['config'].get('onepass_fallbacks')}")
