#!/usr/bin/env python3
"""Median per-dispatch counters of parse_kernel from a scripts/pmc.sh output directory."""
import collections
import csv
import statistics
import sys

d = sys.argv[1]
kern = sys.argv[2] if len(sys.argv) > 2 else "parse_kernel"
vals = {}
waves = None
for sub in ["sq1", "sq2", "fetch", "write"]:
    try:
        rows = list(csv.DictReader(open(f"{d}/{sub}/pmc_counter_collection.csv")))
    except FileNotFoundError:
        continue
    agg = collections.defaultdict(list)
    for r in rows:
        if kern in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in agg.items():
        vals[k] = statistics.median(v)
w = vals.get("SQ_WAVES", 16384)
for k, v in sorted(vals.items()):
    extra = ""
    if k.startswith("SQ_INSTS"):
        extra = f"  ({v / w:.1f} per wave)"
    if k in ("FETCH_SIZE",):
        extra = f"  (x2 gfx950 correction: {2 * v * 1024 / 1e6:.2f} MB)"
    if k in ("WRITE_SIZE",):
        extra = f"  ({v * 1024 / 1e6:.2f} MB)"
    print(f"{k:24s} {v:16.1f}{extra}")
if "SQ_WAVE_CYCLES" in vals:
    wc = vals["SQ_WAVE_CYCLES"]
    for k in ("SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY"):
        if k in vals:
            print(f"  {k}/WAVE_CYCLES = {vals[k] / wc:.2f}")
