#!/usr/bin/env python3
"""Host-memory path through the library's own pipeline (pkt_parse_host): a pinned host batch in,
pinned host columns out, chunk-pipelined over the ctx's three HIP streams.  Reports the
PCIe-inclusive packet rate next to the bytes each direction moved.

  python scripts/hostpath_native.py [--config c2|c4] [--packets N] [--chunks 65536,131072,...]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "packet-rs_amd"))
import torch  # noqa: E402,F401  (HIP runtime first)
import pktgpu  # noqa: E402
from pktgpu import gen, schema  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c2")
ap.add_argument("--packets", type=int, default=1 << 20)
ap.add_argument("--chunks", default="65536,131072,262144,524288")
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--columns", default=None)
ap.add_argument("--staging", type=int, default=0,
                help="pkt_ctx_set_staging: 0 = pinned columns through the export pipeline, 2 = zero copy")
ap.add_argument("--pageable", action="store_true",
                help="plain numpy buffers (staged chunk pipeline) instead of pinned (zero copy)")
args = ap.parse_args()

P = pktgpu.Parser(0)
P.set_staging(args.staging)
n = args.packets
if args.config == "c2":
    src, stride, offs, lens = gen.gen_c2(n).reshape(-1), 64, None, None
    cols = pktgpu.resolve_columns((args.columns or "chain,ether,ipv4,udp").split(","))
else:
    src, offs, lens = gen.gen_c4(n)
    stride = None
    cols = pktgpu.resolve_columns("all" if (args.columns or "all") == "all" else args.columns.split(","))
alloc = (lambda shp, dt: np.empty(shp, dt)) if args.pageable else P.host_empty
slab = alloc(src.shape, np.uint8)
slab[:] = src
if offs is not None:
    h_offs = alloc(offs.shape, np.uint64)
    h_offs[:] = offs
    h_lens = alloc(lens.shape, np.uint32)
    h_lens[:] = lens
else:
    h_offs = h_lens = None
out = {c: alloc(schema.column_shape(c, n), schema.column_dtype(c)) for c in cols}
for a in out.values():
    a[...] = 0
out_bytes = sum(a.nbytes for a in out.values())
in_bytes = slab.nbytes + (h_offs.nbytes + h_lens.nbytes if h_offs is not None else 0)
for ch in [int(x) for x in args.chunks.split(",")]:
    P.parse_host(slab, stride=stride, n=n, offsets=h_offs, lens=h_lens, out=out, chunk=ch)  # warm
    ts = []
    for _ in range(args.reps):
        t0 = time.perf_counter()
        P.parse_host(slab, stride=stride, n=n, offsets=h_offs, lens=h_lens, out=out, chunk=ch)
        ts.append(time.perf_counter() - t0)
    t = float(np.median(ts))
    print(json.dumps({"path": "pkt_parse_host " + ("(pageable: chunked copies on 3 streams)" if args.pageable else
                                                  "(pinned: zero copy)" if args.staging == 2 else
                                                  "(pinned: DMA in, column export kernel out)"), "config": args.config,
                      "packets": n, "chunk": ch, "ms_per_batch": round(t * 1e3, 3),
                      "gpkt_s": round(n / t / 1e9, 4), "in_GB": round(in_bytes / 1e9, 4),
                      "out_GB": round(out_bytes / 1e9, 4), "in_GB_s": round(in_bytes / t / 1e9, 2),
                      "out_GB_s": round(out_bytes / t / 1e9, 2), "columns": len(cols)}), flush=True)
