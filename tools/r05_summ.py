#!/usr/bin/env python3
"""Summarise a tools/r05_ab.sh output directory: stamps medians and bench lines."""
import json
import os
import statistics as st
import sys

d = sys.argv[1]
for f in sorted(os.listdir(d)):
    p = os.path.join(d, f)
    if f.endswith(".jsonl"):
        recs = [json.loads(l) for l in open(p) if l.startswith("{")][1:]
        if recs:
            keys = ("span_us", "first_row_us", "rows_phase1_us", "drain_us", "epilogue_us", "end_spread_us")
            print(f, {k: round(st.median(r[k] for r in recs), 2) for k in keys})
    elif f.endswith(".json"):
        try:
            j = json.loads(open(p).read().strip().splitlines()[-1])
        except Exception as e:
            print(f, "unreadable", e)
            continue
        k = j["config"]["kernel_avg_ms"]
        print(f, round(j["value"], 1), "it/s", round(j["ms_per_step"] * 1e3, 2), "us/it",
              {a: round(b * 1e3, 2) for a, b in k.items() if b})
