#!/usr/bin/env python3
"""Per-launch HBM traffic of the hot kernels from rocprofv3 PMC passes.

Usage: python tools/pmc_traffic.py FETCH_DIR WRITE_DIR WORKLOAD_KEY [ALG_BYTES_PER_LAUNCH]

Reads the counter_collection CSVs of two separate `rocprofv3 --pmc FETCH_SIZE`
and `--pmc WRITE_SIZE` passes (FETCH_SIZE and WRITE_SIZE do not fit one pass
on gfx950) and applies MI355X_MICROARCH.md's HBM corrections:
  * FETCH_SIZE and WRITE_SIZE are in KiB;
  * on gfx950 FETCH_SIZE reports exactly half the bytes of a wide (16 B/lane)
    coalesced streaming read, so it is doubled.
Writes/updates profiles/pmc_traffic.json: {WORKLOAD_KEY: {kernel: bytes/launch, ...}}.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_launch(dirname, counter):
    files = glob.glob(os.path.join(dirname, "**", "*counter_collection.csv"), recursive=True)
    vals = defaultdict(list)
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                name = row.get("Kernel_Name", "")
                if "k_iter_a" in name:
                    key = "k_iter_a"
                elif "k_iter_b" in name:
                    key = "k_iter_b"
                elif "k_colpass" in name and ("Li0E" in name or ", 0," in name or "<float, 0" in name):
                    key = "k_colpass"
                elif "k_rowpass" in name:
                    key = "k_rowpass"
                elif "k_onepass<" in name:      # not k_onepass_tail / k_onepass_fold
                    key = "k_onepass"
                elif "k_panel_pass1" in name:
                    key = "k_panel_pass1"
                elif "k_panel_pass2" in name:
                    key = "k_panel_pass2"
                else:
                    continue
                vals[key].append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items() if v}, {k: len(v) for k, v in vals.items()}


def main():
    fdir, wdir, key = sys.argv[1], sys.argv[2], sys.argv[3]
    alg = float(sys.argv[4]) if len(sys.argv) > 4 else None
    fetch, nf = per_launch(fdir, "FETCH_SIZE")
    write, nw = per_launch(wdir, "WRITE_SIZE")
    out = {}
    for k in sorted(set(fetch) | set(write)):
        fb = 2.0 * fetch.get(k, 0.0) * 1024.0
        wb = write.get(k, 0.0) * 1024.0
        out[k] = {"fetch_bytes_corrected": fb, "write_bytes": wb, "hbm_bytes": fb + wb,
                  "dispatches": [nf.get(k, 0), nw.get(k, 0)]}
        if alg:
            out[k]["alg_bytes"] = alg
            out[k]["traffic_over_alg"] = (fb + wb) / alg
    path = os.environ.get("PMC_OUT") or os.path.join(ROOT, "profiles", "pmc_traffic.json")
    data = {}
    if os.path.exists(path):
        data = json.load(open(path))
    data.setdefault(key, {}).update(out)   # kernels of this key not in these passes keep their entries
    json.dump(data, open(path, "w"), indent=1, sort_keys=True)
    print(json.dumps({key: out}, indent=1))


if __name__ == "__main__":
    main()
