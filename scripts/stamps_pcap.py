#!/usr/bin/env python3
"""Where a pcap_guess_kernel wave spends its time (diagnostic stamps build, PKTGPU_LIB=.../stamps.so):
one pkt_pcap_index_device call on a 2^20-record C4 capture; segments per wave: stage the block's
4 regions, find the region's entry (candidate scan), walk its records, store.  SHARES, not lengths."""
import ctypes
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "packet-rs_amd"))
import pktgpu  # noqa: E402
from pktgpu import gen  # noqa: E402

assert "stamps" in os.environ.get("PKTGPU_LIB", "")
n = 1 << 20
buf, offs, lens = gen.gen_c4(n, seed=0x5EED0004)
P = pktgpu.Parser(0)
d = torch.from_numpy(buf).cuda()
K = (buf.size + 4095) // 4096
st = torch.zeros(K * 8, dtype=torch.uint64, device="cuda")
L = ctypes.CDLL(os.environ["PKTGPU_LIB"])
L.pkt_debug_pcap_stamps.argtypes = [ctypes.c_void_p]
for _ in range(3):
    P.pcap_index(d, cap=n)
torch.cuda.synchronize()
assert L.pkt_debug_pcap_stamps(ctypes.c_void_p(st.data_ptr())) == 0
o, l_, cnt = P.pcap_index(d, cap=n)
torch.cuda.synchronize()
L.pkt_debug_pcap_stamps(ctypes.c_void_p(0))
assert cnt == n and np.array_equal(o.cpu().numpy(), offs)
x = st.cpu().numpy().view(np.int64).reshape(K, 8)
x = x[x[:, 0] != 0].copy()
# s_memtime counts per XCD: rebase each XCD's stamps on its own first wave start
for xc in np.unique(x[:, 6]):
    m = x[:, 6] == xc
    x[m, :5] -= x[m, 0].min()
span = (x[:, 4] - x[:, 0].min()).max()
segs = {"stage (16 KiB per block)": x[:, 1] - x[:, 0], "entry scan": x[:, 2] - x[:, 1], "walk": x[:, 3] - x[:, 2],
        "store + drain": x[:, 4] - x[:, 3], "wave total": x[:, 4] - x[:, 0]}
tot = segs["wave total"].sum()
print(f"pcap_guess_kernel: {len(x)} waves, stamp span {span} cycles")
for k, v in segs.items():
    print(f"  {k:28s} median {np.median(v):9.0f} cyc  p90 {np.percentile(v, 90):9.0f}  share {v.sum() / tot:6.1%}")
t0 = x[:, 0] - x[:, 0].min()
end = x[:, 4] - x[:, 0].min()
grid = np.linspace(0, span, 25)
print("  waves alive:", " ".join(str(int(((t0 <= g) & (end > g)).sum())) for g in grid))
