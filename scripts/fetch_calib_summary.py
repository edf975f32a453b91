#!/usr/bin/env python3
"""Pairs fetch_kernel dispatches (in launch order) with scripts/fetch_calib.py's plan and prints
FETCH_SIZE bytes per item next to the bytes, 64-B sectors and 128-B lines each item touches."""
import collections
import csv
import glob
import json
import sys

d, planf = sys.argv[1], sys.argv[2]
meta = json.load(open(planf))
rows = [r for r in csv.DictReader(open(glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)[0])) if "fetch_kernel" in r["Kernel_Name"]]
by = collections.OrderedDict()
for r in rows:
    by.setdefault(int(r["Dispatch_Id"]), 0.0)
    by[int(r["Dispatch_Id"])] += float(r["Counter_Value"])
vals = [by[k] for k in sorted(by)]
plan = meta["plan"] * meta["reps"]
n = meta["n"]
out = []
for (w, ph), v in zip(plan, vals):
    sectors = (ph + w - 1) // 64 - ph // 64 + 1
    lines = (ph + w - 1) // 128 - ph // 128 + 1
    per = v * 1024 / n
    out.append({"width": w, "phase": ph, "fetch_bytes_per_item": round(per, 1), "sectors_x64": sectors * 64,
                "lines_x128": lines * 128})
    print(f"width {w:4d} phase {ph:4d}: FETCH_SIZE {per:7.1f} B/item   touched: {w} B, "
          f"{sectors} sectors ({sectors * 64} B), {lines} lines ({lines * 128} B)")
json.dump(out, open(sys.argv[3], "w"), indent=1) if len(sys.argv) > 3 else None
