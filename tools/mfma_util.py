#!/usr/bin/env python3
"""MFMA utilisation of the panel passes from the counters of tools/panel_mfma_pmc.sh.

Usage: python tools/mfma_util.py OUTDIR > profiles/mfma_util.json
For each pass: SQ_VALU_MFMA_BUSY_CYCLES / (SIMDs x kernel cycles), kernel cycles = GRBM_GUI_ACTIVE / 8
(rocprofv3 sums it over the 8 XCDs, MI355X_MICROARCH.md "DVFS give-back"); the same busy cycles
against the 2.4 GHz peak clock over the kernel-trace duration (= the flop-based fraction of the
2.5 PF dense bf16 peak); and the instruction count x 16 cycles per v_mfma_f32_16x16x32_bf16
(guide: per-instruction table) as a cross-check of the busy counter."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

SIMDS = 1024            # 256 CUs x 4
PEAK_HZ = 2.4e9         # the clock of the 2.5 PF dense bf16 figure (1024 flops / cycle / SIMD)
CYC_PER_MFMA = 16       # v_mfma_f32_16x16x32_bf16, cycles per SIMD


def counters(d):
    v = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = "k_panel_pass1" if "pass1" in r["Kernel_Name"] else "k_panel_pass2"
            v[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: sum(x) / len(x) for c, x in cs.items()} for k, cs in v.items()}


def durations(d):
    """average launch duration per pass over all of its instantiations (the carried-gradient pass 1
    runs two: the carried form and, every g_refresh iterations, the exact one), weighted by calls"""
    tot, calls = defaultdict(float), defaultdict(int)
    for f in glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            for k in ("k_panel_pass1", "k_panel_pass2"):
                if k in r["Name"]:
                    tot[k] += float(r["TotalDurationNs"]) * 1e-9
                    calls[k] += int(r["Calls"])
    return {k: tot[k] / calls[k] for k in tot if calls[k]}


def main():
    root = sys.argv[1]
    dur = durations(os.path.join(root, "trace"))
    res = {"source": os.environ.get("MFMA_SOURCE", "tools/profile.sh (rocprofv3 --pmc, one pass per k) + kernel trace of bench.py --config 4"),
           "simds": SIMDS, "peak_clock_hz": PEAK_HZ}
    for kdir in sorted(glob.glob(os.path.join(root, "k*"))):
        k = os.path.basename(kdir)
        for name, c in sorted(counters(kdir).items()):
            busy = c["SQ_VALU_MFMA_BUSY_CYCLES"]
            cyc = c["GRBM_GUI_ACTIVE"] / 8
            e = {"mfma_instructions": c["SQ_INSTS_VALU_MFMA_BF16"], "mfma_flops": c["SQ_INSTS_VALU_MFMA_MOPS_BF16"] * 512,
                 "busy_cycles": busy, "busy_from_count": c["SQ_INSTS_VALU_MFMA_BF16"] * CYC_PER_MFMA,
                 "kernel_cycles": cyc, "busy_frac_at_running_clock": busy / (SIMDS * cyc)}
            if k == "k128" and name in dur:
                e["trace_avg_s"] = dur[name]
                e["running_clock_hz_est"] = cyc / dur[name]
                e["busy_frac_at_peak_clock"] = busy / (SIMDS * PEAK_HZ * dur[name])
                e["tflops"] = e["mfma_flops"] / dur[name] / 1e12
            res[f"{name}_{k}"] = e
    json.dump(res, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
