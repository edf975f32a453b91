#!/usr/bin/env python3
"""FETCH_SIZE calibration for scattered per-lane reads (run under rocprofv3 --pmc FETCH_SIZE):
one launch per (width, phase) of pkt_probe_fetch over 2^20 items at a 256-B stride (every item on
its own lines, 256 MiB buffer, fresh lines per launch), then a coalesced torch copy for the
guide's x2 reference.  The launches run in a fixed order; scripts/fetch_calib_summary.py pairs
them with their counters."""
import ctypes
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
L = ctypes.CDLL(os.path.join(REPO, "packet-rs_amd", "lib", "libpktprobe.so"))
L.pkt_probe_fetch.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                              ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]
n, stride = 1 << 20, 256
bufs = [torch.randint(0, 255, (n * stride + 256,), dtype=torch.uint8, device="cuda") for _ in range(4)]
out = torch.empty(n, dtype=torch.int32, device="cuda")
s = torch.cuda.current_stream().cuda_stream
plan = [(w, ph) for w in (16, 32, 64, 80, 128) for ph in (0, 48, 112)]
k = 0
for rep in range(2):
    for w, ph in plan:
        assert L.pkt_probe_fetch(bufs[k % 4].data_ptr(), bufs[k % 4].numel(), n, stride, ph, w, out.data_ptr(), s) == 0
        k += 1
torch.cuda.synchronize()
json.dump({"n": n, "stride": stride, "plan": plan, "reps": 2}, open(sys.argv[1], "w"))
