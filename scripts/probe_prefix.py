#!/usr/bin/env python3
"""Does reading 64 B of each 128-B slot cost 64 or 128 B of HBM time?  (fetch granularity)"""
import ctypes, os, subprocess
import numpy as np, torch
HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "build", "libprobe.so")
L = ctypes.CDLL(SO)
L.probe_prefix.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]
n = 1 << 20
st = torch.cuda.current_stream()
for stride, rd in ((64, 64), (128, 64), (128, 128 // 2 * 2 if False else 64), (256, 64), (128, 32), (64, 32)):
    ring = max(2, (1 << 30) // (n * stride))
    slabs = [torch.randint(0, 255, (n * stride,), dtype=torch.uint8, device="cuda") for _ in range(ring)]
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    ts = []
    for rnd in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for k in range(32):
            L.probe_prefix(slabs[k % ring].data_ptr(), n, stride, rd, out.data_ptr(), ctypes.c_void_p(st.cuda_stream))
        e1.record(st)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / 32 * 1e3)
    us = min(ts)
    print(f"stride {stride:4d} read {rd:3d} B/slot: {us:7.2f} us  -> {n * rd / us / 1e3:7.1f} GB/s useful, {n * max(rd, 128 if stride >= 128 else stride) / us / 1e3:7.1f} GB/s if whole 128-B lines")
    del slabs
