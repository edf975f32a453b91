#!/usr/bin/env python3
"""Where a parse wave spends its time (diagnostic build, -DPKTGPU_STAMPS=1: run with
PKTGPU_LIB=packet-rs_amd/lib/variants/stamps.so).  One isolated launch of the config's parse with
per-wave s_memtime stamps: windows loaded, walk done, emit issued, stores drained.  Prints the
segment shares and the spread of wave start times (how many 'rounds' of waves the launch runs).
Read the SHARES: the stamps' waits forbid overlaps the real kernel has (cdna_hip_programming.md §7)."""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "packet-rs_amd"))
import pktgpu  # noqa: E402
from pktgpu import gen  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c4")
ap.add_argument("--columns", default="all")
ap.add_argument("--window", type=int, default=0)
ap.add_argument("--staging", type=int, default=0)
ap.add_argument("--n", type=int, default=1 << 20)
a = ap.parse_args()
assert "stamps" in os.environ.get("PKTGPU_LIB", ""), "run with PKTGPU_LIB=.../variants/stamps.so"
P = pktgpu.Parser(0)
P.set_window(a.window)
P.set_staging(a.staging)
n = a.n
if a.config == "c2":
    slab_np, stride, offs, lens = gen.gen_c2(n).reshape(-1), 64, None, None
elif a.config == "c3":
    slab_np, stride, offs, lens = gen.gen_c3(n).reshape(-1), 128, None, None
else:
    slab_np, offs, lens = gen.gen_c4(n)
    stride = None
ring = max(2, int(np.ceil((1 << 30) / slab_np.size)))
base = torch.from_numpy(slab_np).cuda()
slabs = [base] + [base.clone() for _ in range(ring - 1)]
d_offs = torch.from_numpy(offs).cuda() if offs is not None else None
d_lens = torch.from_numpy(lens).cuda() if lens is not None else None
cols = pktgpu.resolve_columns("all" if a.columns == "all" else a.columns.split(","))
outs = [P.alloc(n, cols) for _ in range(ring)]
bs = [P._batch(slabs[r], n, stride, d_offs, d_lens) for r in range(ring)]
os_ = [P.out_struct(o) for o in outs]
s = torch.cuda.current_stream()
for k in range(3 * ring):
    P.launch(bs[k % ring], 0, os_[k % ring], s)
torch.cuda.synchronize()
nw = (n + 255) // 256 * 4
st = torch.zeros(nw * 8, dtype=torch.uint64, device="cuda")
L = ctypes.CDLL(os.environ["PKTGPU_LIB"])
L.pkt_debug_stamps.argtypes = [ctypes.c_void_p]
assert L.pkt_debug_stamps(ctypes.c_void_p(st.data_ptr())) == 0
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(s)
P.launch(bs[1], 0, os_[1], s)
e1.record(s)
torch.cuda.synchronize()
L.pkt_debug_stamps(ctypes.c_void_p(0))
us = e0.elapsed_time(e1) * 1e3
x = st.cpu().numpy().view(np.int64).reshape(nw, 8)
x = x[x[:, 0] != 0].copy()
# s_memtime counts per XCD: rebase each XCD's stamps on its own first wave start
for xc in np.unique(x[:, 6]):
    m = x[:, 6] == xc
    x[m, :5] -= x[m, 0].min()
t0 = x[:, 0] - x[:, 0].min()
span = (x[:, 4] - x[:, 0].min()).max()
cyc_per_us = span / us
print(f"{a.config} cols={a.columns} window={a.window}: {len(x)} waves, launch {us:.1f} us (events), "
      f"stamp span {span} cycles -> {cyc_per_us:.0f} cycles/us")
segs = {"load (start -> windows in LDS)": x[:, 1] - x[:, 0], "walk": x[:, 2] - x[:, 1],
        "emit issue": x[:, 3] - x[:, 2], "store drain": x[:, 4] - x[:, 3], "wave total": x[:, 4] - x[:, 0]}
tot = segs["wave total"].sum()
for k, v in segs.items():
    print(f"  {k:32s} median {np.median(v) / cyc_per_us:7.2f} us  p90 {np.percentile(v, 90) / cyc_per_us:7.2f} us"
          f"  share {v.sum() / tot:6.1%}")
st_us = t0 / cyc_per_us
h, edges = np.histogram(st_us, bins=12, range=(0, us))
print("  wave starts per %.1f-us bin:" % (us / 12), " ".join(str(int(c)) for c in h))
end_us = (x[:, 4] - x[:, 0].min()) / cyc_per_us
h, _ = np.histogram(end_us, bins=12, range=(0, us))
print("  wave ends   per %.1f-us bin:" % (us / 12), " ".join(str(int(c)) for c in h))
# concurrency: waves alive at each time
grid = np.linspace(0, us, 25)
alive = [int(((st_us <= g) & (end_us > g)).sum()) for g in grid]
print("  waves alive:", " ".join(str(v) for v in alive))
