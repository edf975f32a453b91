#!/usr/bin/env python3
"""Run the read-path probes of scripts/probe.hip over a >= 1 GiB ring of 64-byte-packet slabs."""
import ctypes
import os
import subprocess
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "build", "libprobe.so")
if not os.path.exists(SO):
    os.makedirs(os.path.dirname(SO), exist_ok=True)
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", SO,
                    os.path.join(HERE, "probe.hip")], check=True)
L = ctypes.CDLL(SO)
L.probe_launch.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_int,
                           ctypes.c_void_p]
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
ring = max(2, (1 << 30) // (n * 64))
slabs = [torch.randint(0, 255, (n * 64,), dtype=torch.uint8, device="cuda") for _ in range(ring)]
outs = [torch.empty(n, dtype=torch.int32, device="cuda") for _ in range(ring)]
names = ["dma_gather", "dma_contig", "reg_strided", "reg_contig"] + [f"dma_persist g={g}" for g in (256, 512, 1024, 2048)]
grids = [0, 0, 0, 0, 256, 512, 1024, 2048]
which = [0, 1, 2, 3, 4, 4, 4, 4]
res = {k: [] for k in names}
st = torch.cuda.current_stream()
for rnd in range(5):
    for nm, w, g in zip(names, which, grids):
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(24)]
        for k in range(24):
            ev[k][0].record(st)
            assert L.probe_launch(w, slabs[k % ring].data_ptr(), n, outs[k % ring].data_ptr(), g, ctypes.c_void_p(st.cuda_stream)) == 0
            ev[k][1].record(st)
        torch.cuda.synchronize()
        res[nm] += [a.elapsed_time(b) * 1e3 for a, b in ev[2:]]
L.probe_write.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]
sizes = [1] * 11 + [2] * 15 + [4] * 3 + [8] * 2
colsets = []
for r in range(ring):
    cols = [torch.empty(n * s_, dtype=torch.uint8, device="cuda") for s_ in sizes]
    arr = (ctypes.c_void_p * 31)(*[c.data_ptr() for c in cols])
    colsets.append((cols, arr))
for nm in ("write_lane", "write_lds"):
    res[nm] = []
for rnd in range(5):
    for w, nm in enumerate(("write_lane", "write_lds")):
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(24)]
        for k in range(24):
            ev[k][0].record(st)
            assert L.probe_write(w, slabs[k % ring].data_ptr(), n, colsets[k % ring][1], ctypes.c_void_p(st.cuda_stream)) == 0
            ev[k][1].record(st)
        torch.cuda.synchronize()
        res[nm] += [a.elapsed_time(b) * 1e3 for a, b in ev[2:]]
for nm in ("write_lane", "write_lds"):
    us = float(np.median(res[nm]))
    print(f"{nm:22s} {us:8.2f} us  read+write {(n * 133) / us / 1e3:8.1f} GB/s")
for nm in names:
    us = float(np.median(res[nm]))
    print(f"{nm:22s} {us:8.2f} us  read {n * 64 / us / 1e3:8.1f} GB/s  total {(n * 68) / us / 1e3:8.1f} GB/s")
