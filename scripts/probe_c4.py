#!/usr/bin/env python3
"""C4 window-load probe: time of the per-record window loads alone (no walk), for window placements
(16-byte-aligned start + 5 chunks = the parse kernel's, sector- and line-aligned starts, wider
windows), next to the parse kernel's status-only launch and a read of the whole file."""
import ctypes
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "packet-rs_amd"))
import pktgpu  # noqa: E402
from pktgpu import gen  # noqa: E402

L = ctypes.CDLL(os.path.join(REPO, "packet-rs_amd", "lib", "libpktprobe.so"))
L.pkt_probe_c4load.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                               ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]
n = 1 << 20
buf, offs, lens = gen.gen_c4(n)
ring = 6
slabs = [torch.from_numpy(buf).cuda() for _ in range(ring)]
d_offs = torch.from_numpy(offs).cuda()
d_lens = torch.from_numpy(lens).cuda()
out = torch.empty(n, dtype=torch.uint8, device="cuda")
s = torch.cuda.current_stream()


def timeit(fn, iters=20):
    for k in range(3):
        fn(k)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for k in range(iters):
        fn(k)
    b.record(s)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3


for nch, al in ((5, 4), (8, 4), (4, 6), (8, 6), (8, 7), (10, 4), (2, 4)):
    us = timeit(lambda k: L.pkt_probe_c4load(slabs[k % ring].data_ptr(), buf.size, d_offs.data_ptr(), n, nch, al,
                                             out.data_ptr(), ctypes.c_void_p(s.cuda_stream)))
    print(f"load {nch:2d} chunks from off & ~{(1 << al) - 1:3d}: {us:7.2f} us")
P = pktgpu.Parser(0)
for cols in (["status"], ["chain"]):
    outs = P.alloc(n, cols)
    us = timeit(lambda k: P.parse(slabs[k % ring], offsets=d_offs, lens=d_lens, columns=cols, out=outs))
    print(f"parse {cols}: {us:7.2f} us")
dst = torch.empty(buf.size // 4, dtype=torch.int32, device="cuda")
us = timeit(lambda k: dst.copy_(slabs[k % ring].view(torch.int32)[: buf.size // 4]) if False else slabs[k % ring].view(torch.uint8).sum(dtype=torch.int32))
print(f"torch sum of the file (read once): {us:7.2f} us  ({buf.size / 1e6:.0f} MB)")
