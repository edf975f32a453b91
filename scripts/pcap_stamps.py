#!/usr/bin/env python3
"""Where a pcap guess wave spends its time (diagnostic build, -DPKTGPU_STAMPS=1: run with
PKTGPU_LIB=packet-rs_amd/lib/variants/stamps.so).  One blocking pkt_pcap_index_device call over the
C4 capture with per-wave s_memrealtime stamps: staged, candidate scan done, walk barrier, stores
drained.  Prints the segment medians/shares, the wave-start spread and the candidate distances."""
import ctypes
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "packet-rs_amd"))
import pktgpu  # noqa: E402
from pktgpu import gen  # noqa: E402

assert "stamps" in os.environ.get("PKTGPU_LIB", ""), "run with PKTGPU_LIB=.../variants/stamps.so"
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
buf, offs, lens = gen.gen_c4(n, seed=0x5EED0004)
P = pktgpu.Parser(0)
d = torch.from_numpy(buf).cuda()
o = torch.empty(n, dtype=torch.uint64, device="cuda")
l = torch.empty(n, dtype=torch.uint32, device="cuda")
cnt = ctypes.c_uint64()
s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
L = P._L


def call():
    rc = L.pkt_pcap_index_device(P._ctx, d.data_ptr(), d.numel(), o.data_ptr(), l.data_ptr(), n,
                                 ctypes.byref(cnt), s)
    assert rc == 0, rc


for _ in range(3):
    call()
K = (buf.size + 4095) // 4096
NB = (K + 255) // 256
st = torch.zeros(K * 8 + NB * 16, dtype=torch.uint64, device="cuda")
D = ctypes.CDLL(os.environ["PKTGPU_LIB"])
D.pkt_debug_pcap_stamps.argtypes = [ctypes.c_void_p]
assert D.pkt_debug_pcap_stamps(ctypes.c_void_p(st.data_ptr())) == 0
torch.cuda.synchronize()
call()
torch.cuda.synchronize()
D.pkt_debug_pcap_stamps(ctypes.c_void_p(0))
assert cnt.value == n and np.array_equal(o.cpu().numpy(), offs)
xa = st.cpu().numpy().view(np.int64)
y = xa[K * 8:].reshape(NB, 16).copy()
x = xa[:K * 8].reshape(K, 8)
# wrong guesses: regions whose guessed entry is not the first record start at or past the region base
st_ = offs.astype(np.int64) - 16
bases = np.arange(K, dtype=np.int64) * 4096
i_ = np.searchsorted(st_, bases)
true_ = np.where((i_ < len(st_)) & (st_[np.minimum(i_, len(st_) - 1)] < bases + 4096),
                 st_[np.minimum(i_, len(st_) - 1)] - bases, 4096)
bad_ = np.nonzero((x[:, 0] != 0) & (x[:, 6] != true_))[0]
print(f"wrong guesses: {len(bad_)}" + "".join(f"\n  region {k} (k % 4 = {k % 4}): guess {x[k, 6]} true {true_[k]}"
                                                for k in bad_[:16]))
x = x[x[:, 0] != 0].copy()
t00 = x[:, 0].min()
x[:, :5] -= t00  # one device-wide constant clock
span = x[:, 4].max()
# s_memrealtime: the 100 MHz constant clock -> us
f = 100.0
print(f"{len(x)} waves (regions), stamp span {span / f:.1f} us at 100 MHz")
segs = {"stage (start -> barrier)": x[:, 1] - x[:, 0], "candidate scan": x[:, 2] - x[:, 1],
        "barrier + lane walks": x[:, 3] - x[:, 2], "stores drained": x[:, 4] - x[:, 3],
        "wave total": x[:, 4] - x[:, 0]}
tot = segs["wave total"].sum()
for k, v in segs.items():
    print(f"  {k:28s} median {np.median(v) / f:7.2f} us  p90 {np.percentile(v, 90) / f:7.2f} us  share {v.sum() / tot:6.1%}")
h, _ = np.histogram(x[:, 0] / f, bins=12, range=(0, span / f))
print("  wave starts per bin:", " ".join(str(int(c)) for c in h))
dist = x[:, 6]
print(f"  entry - base: median {np.median(dist):.0f} B, p90 {np.percentile(dist, 90):.0f}, max {dist.max()}; "
      f"records per region median {np.median(x[:, 7]):.0f}")
steps = dist // 64 + 1
for q in (1, 2, 3, 4, 5):
    print(f"    candidate steps == {q}: {(steps == q).mean():6.1%}")
print(f"    candidate steps > 5: {(steps > 5).mean():6.1%}")

# scan blocks (one row per block: start, states loaded, local fixes done, look-back done, end)
y = y[y[:, 0] != 0]
y[:, :5] -= t00
y[:, 7] -= t00
y[:, 8:10] -= t00
print(f"scan: {len(y)} blocks; first start {y[:, 0].min() / f:.1f} us after the first guess wave, "
      f"last end {y[:, 4].max() / f:.1f} us")
ss = {"states loaded": y[:, 1] - y[:, 0], "first block composition": y[:, 7] - y[:, 1],
      "  its wave scans": y[:, 8] - y[:, 1], "  its first barrier": y[:, 9] - y[:, 8],
      "local fixes": y[:, 2] - y[:, 1], "look-back": y[:, 3] - y[:, 2],
      "exact state + prefixes": y[:, 4] - y[:, 3], "block total": y[:, 4] - y[:, 0]}
for k, v in ss.items():
    print(f"  {k:28s} median {np.median(v) / f:7.2f} us  p90 {np.percentile(v, 90) / f:7.2f} us  max {v.max() / f:7.2f} us")
print(f"  blocks with fixes: {(y[:, 5] > 0).sum()} (regions re-walked {y[:, 5].sum()}); look-back retries "
      f"median {np.median(y[:, 6] & 0xFFFF):.0f} max {(y[:, 6] & 0xFFFF).max()}; first-seam waits max {(y[:, 6] >> 16).max()}")
print("  scan blocks with fixes:", " ".join(str(int(b)) for b in np.nonzero(y[:, 5] > 0)[0][:16]))
o_ = np.argsort(y[:, 0])
print("  look-back done (us) by start:", " ".join(f"{v / f:.1f}" for v in y[o_, 3][:: max(1, len(y) // 16)]))
