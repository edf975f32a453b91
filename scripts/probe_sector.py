#!/usr/bin/env python3
"""Driver of scripts/probe_sector.hip (measurement only): C3's read shape — 2^20 slots of 128 B, the
first `width` bytes of each read by one lane — with plain, nt, sc0 sc1 and nt sc0 sc1 loads.  Prints
the median time per launch of each (HIP events; the asm forms wait after each load, so only their
request counters are comparable); run it under rocprofv3 --pmc TCC_EA0_RDREQ_64B_sum
TCC_EA0_RDREQ_128B_sum for the memory-side request sizes of each kernel instantiation."""
import ctypes
import json
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
L = ctypes.CDLL(os.path.join(HERE, "_probe_sector.so"))
L.probe_sector.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                           ctypes.c_void_p, ctypes.c_void_p]
n, stride = 1 << 20, 128
width = int(sys.argv[1]) if len(sys.argv) > 1 else 64
bufs = [torch.randint(0, 255, (n * stride,), dtype=torch.uint8, device="cuda") for _ in range(4)]
out = torch.empty(n, dtype=torch.int32, device="cuda")
s = torch.cuda.current_stream().cuda_stream
res = {}
for kind in (0, 1, 2, 3):
    ts = []
    for r in range(12):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        assert L.probe_sector(kind, bufs[r % 4].data_ptr(), n, stride, width, out.data_ptr(), s) == 0
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    ts.sort()
    res[["plain", "nt", "sc0sc1", "nt_sc0sc1"][kind]] = round(ts[len(ts) // 2], 2)
print(json.dumps({"what": "probe_sector", "slots": n, "stride": stride, "width": width, "us_per_launch": res}))
