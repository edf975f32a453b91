#!/usr/bin/env python3
"""Where the blocking pcap step's wall clock goes: `pkt_parse_pcap` (bench.py's `pcap` record, C4
capture of 2^20 records in HBM) called `--reps` times with the wall clock of each call printed; run it
under `rocprofv3 --kernel-trace` and give the trace to --trace afterwards: per call, the span from the
first kernel's start to the last kernel's end, the kernels' own time and the gaps between them, against
the call's wall clock.  One JSON line per mode."""
import argparse
import csv
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "packet-rs_amd"))


def run(a):
    import torch
    import pktgpu
    from pktgpu import gen, schema
    n = a.records
    buf, offs, lens = gen.gen_c4(n, seed=0x5EED0005)
    P = pktgpu.Parser(0)
    d_buf = torch.from_numpy(buf).cuda()
    d_offs = torch.empty(n, dtype=torch.uint64, device="cuda")
    d_lens = torch.empty(n, dtype=torch.uint32, device="cuda")
    out = P.alloc(n, schema.COLUMN_NAMES)
    s = torch.cuda.current_stream()
    for _ in range(3):
        c, _, _, _ = P.parse_pcap(d_buf, n, out=out, offsets=d_offs, lens=d_lens, stream=s)
        assert c == n
    torch.cuda.synchronize()
    time.sleep(0.01)
    ws = []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        P.parse_pcap(d_buf, n, out=out, offsets=d_offs, lens=d_lens, stream=s)
        ws.append(time.perf_counter() - t0)
        if a.gap:
            time.sleep(a.gap)  # separates the calls in the trace
    print(json.dumps({"what": "pkt_parse_pcap wall", "reps": a.reps, "median_us": round(float(np.median(ws)) * 1e6, 1),
                      "min_us": round(min(ws) * 1e6, 1)}), flush=True)


def trace(a):
    rows = []
    for r in csv.DictReader(open(a.trace)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    # calls: groups of kernels separated by > 500 us of idle
    calls, cur = [], []
    for r in rows:
        if cur and r[0] - cur[-1][1] > 500_000:
            calls.append(cur)
            cur = []
        cur.append(r)
    if cur:
        calls.append(cur)
    calls = [c for c in calls if len(c) >= 4][-a.reps:]
    span = [(c[-1][1] - c[0][0]) / 1e3 for c in calls]
    busy = [sum(e - s for s, e, _ in c) / 1e3 for c in calls]
    gaps = [[(c[i + 1][0] - c[i][1]) / 1e3 for i in range(len(c) - 1)] for c in calls]
    names = [k.split("(")[0].split("::")[-1][:40] for _, _, k in calls[-1]]
    print(json.dumps({"what": "pkt_parse_pcap kernels", "calls": len(calls), "kernels": names,
                      "span_us_median": round(float(np.median(span)), 2), "busy_us_median": round(float(np.median(busy)), 2),
                      "gaps_us_median": [round(float(np.median([g[i] for g in gaps])), 2) for i in range(len(gaps[0]))],
                      "kernel_us_median": [round(float(np.median([(c[i][1] - c[i][0]) / 1e3 for c in calls])), 2)
                                           for i in range(len(calls[0]))]}))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=1 << 20)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--gap", type=float, default=0.002, help="seconds between calls (0: back to back)")
    ap.add_argument("--trace", default=None, help="a rocprofv3 kernel_trace.csv of a run of this script")
    a = ap.parse_args()
    trace(a) if a.trace else run(a)
