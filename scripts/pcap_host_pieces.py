#!/usr/bin/env python3
"""pkt_parse_pcap_host (capture in pinned host memory -> all columns in pinned host memory) by piece
size (pkt_ctx_set_host_piece), next to the link's rates alone: the file's H2D copy (one pinned
hipMemcpy through torch) and the columns' D2H copy of the same bytes.  One JSON line per row."""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "packet-rs_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=1 << 20)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--pieces", default="0,4194304,8388608,33554432,one")
    a = ap.parse_args()
    import torch
    import pktgpu
    from pktgpu import gen, schema
    buf, offs, lens = gen.gen_c4(a.records, seed=0x5EED0006)
    n = a.records
    P = pktgpu.Parser(0)
    hb = P.host_empty((buf.size,), np.uint8)
    hb[:] = buf
    cols = list(schema.COLUMN_NAMES)
    out = {c: P.host_empty(schema.column_shape(c, n), schema.column_dtype(c)) for c in cols}
    m, _, _ = P.parse_pcap_host(hb, n, out=out, index=False)
    assert m == n
    written = schema.bytes_per_packet(cols, n_slots=0) * n + 3 * int(out["n_hdrs"].astype(np.int64).sum())
    # the link alone: the file in, the columns' bytes out (torch pinned buffers, one copy each)
    th = torch.empty(buf.size, dtype=torch.uint8, pin_memory=True)
    td = torch.empty(buf.size, dtype=torch.uint8, device="cuda")
    tw = torch.empty(written, dtype=torch.uint8, device="cuda")
    tho = torch.empty(written, dtype=torch.uint8, pin_memory=True)
    s = torch.cuda.Stream()
    t_in, t_out, t_both = [], [], []
    s2 = torch.cuda.Stream()
    for _ in range(a.reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.cuda.stream(s):
            td.copy_(th, non_blocking=True)
        s.synchronize()
        t_in.append(time.perf_counter() - t0)
        t0 = time.perf_counter()
        with torch.cuda.stream(s):
            tho.copy_(tw, non_blocking=True)
        s.synchronize()
        t_out.append(time.perf_counter() - t0)
        t0 = time.perf_counter()
        with torch.cuda.stream(s):
            td.copy_(th, non_blocking=True)
        with torch.cuda.stream(s2):
            tho.copy_(tw, non_blocking=True)
        s.synchronize()
        s2.synchronize()
        t_both.append(time.perf_counter() - t0)
    ti, to, tb = (float(np.median(x)) for x in (t_in, t_out, t_both))
    print(json.dumps({"what": "link", "file_bytes": int(buf.size), "column_bytes": int(written),
                      "h2d_ms": round(ti * 1e3, 3), "h2d_GBps": round(buf.size / ti / 1e9, 2),
                      "d2h_ms": round(to * 1e3, 3), "d2h_GBps": round(written / to / 1e9, 2),
                      "both_at_once_ms": round(tb * 1e3, 3)}), flush=True)
    for pc in a.pieces.split(","):
        piece = buf.size + 1 if pc == "one" else int(pc)
        P.set_host_piece(piece)
        ts = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            m, _, _ = P.parse_pcap_host(hb, n, out=out, index=False)
            ts.append(time.perf_counter() - t0)
            assert m == n
        t = float(np.median(ts))
        print(json.dumps({"what": "pkt_parse_pcap_host", "piece": pc, "records": n, "ms": round(t * 1e3, 3),
                          "Grecords_s": round(n / t / 1e9, 4), "in_GBps": round(buf.size / t / 1e9, 2),
                          "out_GBps": round(written / t / 1e9, 2)}), flush=True)
    P.set_host_piece(0)
    P.close()


if __name__ == "__main__":
    main()
