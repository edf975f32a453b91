#!/usr/bin/env python3
"""Store-shape probes (scripts/probe_store.hip) over a >= 1 GiB ring of 64-byte-packet slabs:
isolated launch time (R back-to-back launches between one event pair, as bench.py's roofline
phase) for K = 1, 2, 4 packets per lane and the ideal 1-KiB-per-instruction store shape."""
import ctypes
import os
import subprocess
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "build", "libprobe_store.so")
if not os.path.exists(SO):
    os.makedirs(os.path.dirname(SO), exist_ok=True)
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", SO,
                    os.path.join(HERE, "probe_store.hip")], check=True)
L = ctypes.CDLL(SO)
L.probe_store.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
ring = max(2, (1 << 30) // (n * 64))
slabs = [torch.randint(0, 255, (n * 64,), dtype=torch.uint8, device="cuda") for _ in range(ring)]
sizes = [1] * 11 + [2] * 15 + [4] * 3 + [8] * 2
ideal = [16] * 4 + [8] + [1] * 26
sets = {}
for nm, sz in (("tuple", sizes), ("ideal", ideal)):
    sets[nm] = []
    for r in range(ring):
        cols = [torch.empty(n * s_, dtype=torch.uint8, device="cuda") for s_ in sz]
        sets[nm].append((cols, (ctypes.c_void_p * 31)(*[c.data_ptr() for c in cols])))
st = torch.cuda.current_stream()
variants = [("K=1 (per-lane narrow stores)", 0, "tuple", 133), ("K=2", 1, "tuple", 133),
            ("K=4", 2, "tuple", 133), ("ideal 72 B (uint4 columns)", 3, "ideal", 136),
            ("2 packets/lane, K=1 stores", 4, "tuple", 133), ("4 packets/lane, K=1 stores", 5, "tuple", 133)]
R = 50
res = {v[0]: [] for v in variants}
for k in range(2 * ring):
    for nm, w, cs, _ in variants:
        L.probe_store(w, slabs[k % ring].data_ptr(), n, sets[cs][k % ring][1], ctypes.c_void_p(st.cuda_stream))
torch.cuda.synchronize()
for rnd in range(5):
    for nm, w, cs, _ in variants:
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        for k in range(R):
            assert L.probe_store(w, slabs[k % ring].data_ptr(), n, sets[cs][k % ring][1],
                                 ctypes.c_void_p(st.cuda_stream)) == 0
        b.record(st)
        torch.cuda.synchronize()
        res[nm].append(a.elapsed_time(b) * 1e3 / R)
for nm, w, cs, bpp in variants:
    us = float(np.median(res[nm]))
    print(f"{nm:32s} {us:8.2f} us/launch  {n * bpp / us / 1e3:8.1f} GB/s ({bpp} B/pkt)", flush=True)

# pipelined: launches round-robin on 2 streams (as bench.py's timed region), device time per launch
streams = [torch.cuda.Stream() for _ in range(2)]
for nm, w, cs, bpp in variants[:1] + variants[4:]:
    ts = []
    for rnd in range(5):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s0 = streams[0]
        a.record(s0)
        streams[1].wait_stream(s0)
        for k in range(200):
            s_ = streams[k % 2]
            L.probe_store(w, slabs[k % ring].data_ptr(), n, sets[cs][k % ring][1], ctypes.c_void_p(s_.cuda_stream))
        s0.wait_stream(streams[1])
        b.record(s0)
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3 / 200)
    us = float(np.median(ts))
    print(f"pipelined 2 streams {nm:22s} {us:8.2f} us/launch  {n * bpp / us / 1e3:8.1f} GB/s", flush=True)
