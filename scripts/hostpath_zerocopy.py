#!/usr/bin/env python3
"""Host path without copies: the parse kernel reads the pinned host slab and writes the pinned host
columns directly over PCIe (pkt_host_alloc memory is mapped into the device address space).
Wave spans (staging 2) read each wave's packets as 1-KiB contiguous pieces; per-lane windows
(staging 1) read 16-byte pieces.  Checked against the oracle, then timed.

  python scripts/hostpath_zerocopy.py [--packets N]
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "packet-rs_amd"), os.path.join(REPO, "oracle")]
import torch  # noqa: E402
import pktgpu  # noqa: E402
from pktgpu import gen, schema  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--packets", type=int, default=1 << 20)
ap.add_argument("--reps", type=int, default=5)
args = ap.parse_args()
n = args.packets
P = pktgpu.Parser(0)
L = P._L
src = gen.gen_c2(n).reshape(-1)
slab = P.host_empty(src.shape, np.uint8)
slab[:] = src
cols = pktgpu.resolve_columns(["chain", "ether", "ipv4", "udp"])
out = {c: P.host_empty(schema.column_shape(c, n), schema.column_dtype(c)) for c in cols}
b = P._lib.PktBatch()
b.slab, b.slab_len, b.stride, b.n = slab.ctypes.data, slab.size, 64, n
o = P._lib.PktOut()
for c, a in out.items():
    setattr(o, c, a.ctypes.data)
stream = torch.cuda.current_stream()
for staging in (2, 1):
    P.set_staging(staging)
    for a in out.values():
        a[...] = 0
    P._check(L.pkt_parse_batch(P._ctx, ctypes.byref(b), 0, ctypes.byref(o), ctypes.c_void_p(stream.cuda_stream)), "parse")
    torch.cuda.synchronize()
    if staging == 2:
        import oracle
        ref = oracle.parse_batch(src, n, stride=64, columns=cols, nthreads=16)
        for c in cols:
            g, r = out[c], ref[c]
            if c in ("hdr_type", "hdr_off"):
                g, r = g[:3], r[:3]
            assert np.array_equal(g, r), c
    ts = []
    for _ in range(args.reps):
        t0 = time.perf_counter()
        P._check(L.pkt_parse_batch(P._ctx, ctypes.byref(b), 0, ctypes.byref(o), ctypes.c_void_p(stream.cuda_stream)), "parse")
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    t = float(np.median(ts))
    ob = sum(schema.bytes_per_packet([c], n_slots=3) for c in cols) * n
    print(json.dumps({"path": "zero-copy (kernel reads/writes pinned host memory)", "staging": staging,
                      "packets": n, "ms_per_batch": round(t * 1e3, 3), "gpkt_s": round(n / t / 1e9, 4),
                      "in_GB_s": round(slab.nbytes / t / 1e9, 2), "out_GB_s": round(ob / t / 1e9, 2),
                      "checked_vs_oracle": staging == 2}), flush=True)
P.set_staging(0)
