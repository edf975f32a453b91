#!/usr/bin/env python3
"""The HBM read floor of the indexed (C4) parse, computed from the capture itself (CPU only):
128-B lines the per-record windows cover, the same counted per cooperative-load instruction (each
wave instruction fetches its own lines: scripts/fetch_calib.py), and the lines the walk reads past
the window (up to each record's payload offset, from the oracle).  Compare with PMC FETCH_SIZE x2."""
import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "packet-rs_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
from pktgpu import gen  # noqa: E402


def cover(s, e, g):
    d = np.zeros(int(e.max()) + 3, np.int64)
    np.add.at(d, s, 1)
    np.add.at(d, e + 1, -1)
    return int((np.cumsum(d) > 0).sum()) * g


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--chunks", default="6,7")
    a = ap.parse_args()
    import oracle  # test infrastructure: the walk's depth per record
    buf, offs, lens = gen.gen_c4(a.n, seed=0)
    o = offs.astype(np.int64)
    L = lens.astype(np.int64)
    r = oracle.parse_batch(buf, a.n, offsets=offs, lens=lens, columns=["status", "n_hdrs", "payload_off"], nthreads=8)
    po = r["payload_off"].astype(np.int64)
    al = o & ~15
    print(f"file {buf.size / 1e6:.1f} MB, index {a.n * 12 / 1e6:.1f} MB")
    for nch in [int(x) for x in a.chunks.split(",")]:
        W = 16 * nch
        win = cover(al // 128, (al + W - 1) // 128, 128)
        walk = cover(al // 128, (np.maximum(al + W, o + po) - 1) // 128, 128)
        # per wave instruction: pairs 64k..64k+63 of the wave's 64*nch (record, chunk) pairs,
        # chunks past the record's end skipped (the lockstep loader's rule)
        nw = a.n // 64
        pid = np.arange(64 * nch)
        rr, cc, kk = pid // nch, pid % nch, pid // 64
        oo = o[: nw * 64].reshape(nw, 64)[:, rr]
        ll = L[: nw * 64].reshape(nw, 64)[:, rr]
        line = np.where(16 * cc[None, :] < (oo & 15) + ll, ((oo & ~15) + 16 * cc[None, :]) // 128, -1)
        per_ins = 0
        for k in range(nch):
            sl = np.sort(line[:, kk == k], axis=1)
            per_ins += int(((sl[:, 1:] != sl[:, :-1]) & (sl[:, 1:] >= 0)).sum() + (sl[:, 0] >= 0).sum())
        print(f"{nch} chunks ({W} B): window lines {win / 1e6:.1f} MB, per instruction {per_ins * 128 / 1e6:.1f} MB, "
              f"window + walk depth {walk / 1e6:.1f} MB")


if __name__ == "__main__":
    main()
