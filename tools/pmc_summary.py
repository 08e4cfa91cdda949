#!/usr/bin/env python3
"""Average every PMC counter per kernel over the counter_collection CSVs under DIR.

Usage: python tools/pmc_summary.py DIR [DIR ...]
Prints kernel -> {counter: mean per dispatch}; FETCH_SIZE / WRITE_SIZE are also
shown as bytes with the gfx950 corrections of MI355X_MICROARCH.md (KiB units;
FETCH_SIZE x2 for 16-B/lane streaming reads).
"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def short(name):
    m = re.search(r"(k_[a-z0-9_]+)", name)
    base = m.group(1) if m else name[:40]
    t = re.search(r"ILi(\d+)E(?:Li(\d+)E)?(?:Li(\d+)E)?", name)
    return base + ("<" + ",".join(g for g in t.groups() if g) + ">" if t else "")


def main():
    vals = defaultdict(lambda: defaultdict(list))
    files = [f for root in sys.argv[1:] for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"),
                                                           recursive=True)]
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                vals[short(row.get("Kernel_Name", ""))][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for k in sorted(vals):
        print(k)
        for c in sorted(vals[k]):
            v = vals[k][c]
            mean = sum(v) / len(v)
            extra = ""
            if c == "FETCH_SIZE":
                extra = f"  -> {2 * mean * 1024 / 1e9:.4f} GB corrected"
            elif c == "WRITE_SIZE":
                extra = f"  -> {mean * 1024 / 1e9:.4f} GB"
            print(f"  {c:28s} {mean:16.1f}  (n={len(v)}){extra}")


if __name__ == "__main__":
    main()
