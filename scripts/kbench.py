#!/usr/bin/env python3
"""Kernel A/B micro-benchmark (one process, interleaved rounds): parse_kernel over a >= 1 GiB
slab ring for several column sets / windows, next to a plain device copy of the same bytes.
Prints one line per variant: median kernel us, Gpkt/s, algorithmic GB/s."""
import argparse
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "packet-rs_amd"))
import pktgpu  # noqa: E402
from pktgpu import gen, schema  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c2")
ap.add_argument("--n", type=int, default=1 << 20)
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--iters", type=int, default=32)
ap.add_argument("--variants", default="status;chain;chain,ether,ipv4,udp;all")
ap.add_argument("--windows", default="0")
ap.add_argument("--streams", default="1")
ap.add_argument("--staging", type=int, default=0, help="pkt_ctx_set_staging mode")
args = ap.parse_args()

dev = torch.device("cuda", 0)
P = pktgpu.Parser(0)
P.set_staging(args.staging)
n = args.n
if args.config == "c2":
    slab_np, stride, offs, lens = gen.gen_c2(n).reshape(-1), 64, None, None
elif args.config == "c3":
    slab_np, stride, offs, lens = gen.gen_c3(n).reshape(-1), 128, None, None
else:
    slab_np, offs, lens = gen.gen_c4(n)
    stride = None
ring = max(2, int(np.ceil((1 << 30) / slab_np.size)))
base = torch.from_numpy(slab_np).to(dev)
slabs = [base] + [base.clone() for _ in range(ring - 1)]
d_offs = torch.from_numpy(offs).to(dev) if offs is not None else None
d_lens = torch.from_numpy(lens).to(dev) if lens is not None else None

stream = torch.cuda.current_stream()
variants = []
for w in [int(x) for x in args.windows.split(",")]:
    for v in args.variants.split(";"):
        cols = pktgpu.resolve_columns("all" if v == "all" else v.split(","))
        outs = [P.alloc(n, cols) for _ in range(ring)]
        bs = [P._batch(slabs[r], n, stride, d_offs, d_lens) for r in range(ring)]
        os_ = [P.out_struct(o) for o in outs]
        variants.append((f"w={w} cols={v}", w, bs, os_, cols, outs))

copy_dst = [torch.empty_like(base) for _ in range(ring)]
# warm every variant (code-object load, first touch of its output ring, clocks)
for name, w, bs, os_, cols, outs in variants:
    P.set_window(w)
    for k in range(2 * ring):
        P.launch(bs[k % ring], 0, os_[k % ring], stream)
torch.cuda.synchronize()
res = {name: [] for name, *_ in variants}
res["torch_copy"] = []
for rnd in range(args.rounds):
    for name, w, bs, os_, cols, outs in variants:
        P.set_window(w)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(args.iters)]
        for k in range(args.iters):
            ev[k][0].record(stream)
            P.launch(bs[k % ring], 0, os_[k % ring], stream)
            ev[k][1].record(stream)
        torch.cuda.synchronize()
        res[name] += [a.elapsed_time(b) * 1e3 for a, b in ev[2:]]
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.iters)]
    for k in range(args.iters):
        ev[k][0].record(stream)
        copy_dst[k % ring].copy_(slabs[(k + 3) % ring])
        ev[k][1].record(stream)
    torch.cuda.synchronize()
    res["torch_copy"] += [a.elapsed_time(b) * 1e3 for a, b in ev[2:]]
P.set_window(0)

# whole-loop wall time with launches spread over S streams (consecutive steps overlap)
import time
for S in [int(x) for x in args.streams.split(",")]:
    streams = [torch.cuda.Stream() for _ in range(S)]
    for k in range(64):  # first use of a new stream is slow: warm them
        P.launch(variants[0][2][k % ring], 0, variants[0][3][k % ring], streams[k % S])
    torch.cuda.synchronize()
    for name, w, bs, os_, cols, outs in variants:
        P.set_window(w)
        ts = []
        for rnd in range(args.rounds):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for k in range(args.iters * 4):
                P.launch(bs[k % ring], 0, os_[k % ring], streams[k % S])
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) / (args.iters * 4) * 1e6)
        us = float(np.median(ts))
        print(f"[{S} streams] {name:40s} {us:8.2f} us/step  {n / us / 1e3:7.2f} Gpkt/s")
P.set_window(0)

span = 64
for name, w, bs, os_, cols, outs in variants:
    us = float(np.median(res[name]))
    nh = int(outs[0]["n_hdrs"].max().item()) if "n_hdrs" in outs[0] else 3
    wb = schema.bytes_per_packet(cols, n_slots=max(nh, 1))
    tot = (span + wb) * n
    print(f"{name:50s} {us:8.2f} us  {n / us / 1e3:7.2f} Gpkt/s  {tot / us / 1e3:8.1f} GB/s "
          f"(read {span} + write {wb} B/pkt)  min {min(res[name]):.2f}")
us = float(np.median(res["torch_copy"]))
print(f"{'torch copy (read+write slab)':50s} {us:8.2f} us  {2 * slab_np.size / us / 1e3:8.1f} GB/s")
