#!/usr/bin/env python3
"""Host-memory path: pinned host slab -> H2D -> parse -> D2H of the tuple into pinned host
memory, chunk-pipelined over 3 HIP streams (copy-in of chunk k+1 and copy-out of chunk k-1
overlap the parse of chunk k).  Reports PCIe-inclusive Gpkt/s next to the device-resident rate.

  python scripts/hostpath.py [--config c2] [--packets 1048576] [--chunks 8] [--reps 10]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "packet-rs_amd"))
import pktgpu  # noqa: E402
from pktgpu import gen, schema  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c2")
ap.add_argument("--packets", type=int, default=1 << 20)
ap.add_argument("--chunks", type=int, default=8)
ap.add_argument("--streams", type=int, default=3)
ap.add_argument("--reps", type=int, default=10)
ap.add_argument("--columns", default="chain,ether,ipv4,udp")
args = ap.parse_args()

dev = torch.device("cuda", 0)
P = pktgpu.Parser(0)
n = args.packets
stride = 64 if args.config == "c2" else 128
slab = (gen.gen_c2(n) if args.config == "c2" else gen.gen_c3(n)).reshape(-1)
cols = pktgpu.resolve_columns(args.columns.split(","))
h_slab = torch.from_numpy(slab).pin_memory()
assert n % args.chunks == 0, "packets must divide into equal chunks"
cn = n // args.chunks


def packed(nn, device, pin=False):
    sizes, tot = [], 0
    for c in cols:
        shp = schema.column_shape(c, nn)
        nb = int(np.prod(shp)) * schema.column_dtype(c).itemsize
        sizes.append((c, shp, nb, tot))
        tot += (nb + 255) // 256 * 256
    buf = torch.empty(tot, dtype=torch.uint8, device=device, pin_memory=pin)
    return buf, {c: buf[o:o + nb].view(pktgpu._tdtype(schema.column_dtype(c))).view(shp)
                 for c, shp, nb, o in sizes}


streams = [torch.cuda.Stream(dev) for _ in range(args.streams)]
d_slab = [torch.empty(cn * stride, dtype=torch.uint8, device=dev) for _ in streams]
d_out = [packed(cn, dev) for _ in streams]
h_out = [packed(cn, "cpu", pin=True) for _ in range(args.chunks)]


def run_once():
    for k in range(args.chunks):
        s = streams[k % len(streams)]
        lo, hi = k * cn, min(n, (k + 1) * cn)
        nn = hi - lo
        with torch.cuda.stream(s):
            ds = d_slab[k % len(streams)][:nn * stride]
            ds.copy_(h_slab[lo * stride:hi * stride], non_blocking=True)
            buf, views = d_out[k % len(streams)]
            P.parse(ds, stride=stride, n=nn, columns=cols, out=views, stream=s)
            h_out[k][0].copy_(buf, non_blocking=True)
    torch.cuda.synchronize()


run_once()
ts = []
for _ in range(args.reps):
    t0 = time.perf_counter()
    run_once()
    ts.append(time.perf_counter() - t0)
t = float(np.median(ts))
in_b = n * stride
out_b = sum(h[0].numel() for h in h_out)
res = {"path": "host memory: pinned H2D + parse + D2H, chunk-pipelined",
       "config": args.config, "packets": n, "chunks": args.chunks, "streams": args.streams,
       "ms_per_batch": round(t * 1e3, 4), "gpkt_s": round(n / t / 1e9, 4),
       "h2d_GB_s": round(in_b / t / 1e9, 2), "d2h_GB_s": round(out_b / t / 1e9, 2),
       "columns": args.columns}
print(json.dumps(res))
