#!/usr/bin/env python3
"""pkt_pcap_stream_* (a capture that arrives as it is produced: north_star's NIC ring / growing file) by
push size: a C4 capture in pinned host memory pushed in pieces of `push` bytes (each push returns once
its bytes have landed on the device, so the caller can reuse its ring slot), a step per `step_bytes` of
new bytes (0 = the 4 MiB default), finish; wall clock from the first push to finish's return, median
of reps.  Columns on the device (`dev`) or in pinned host memory (`pinned`: each step's columns
exported over the link).  One JSON line per row; the record count is checked against the generator's."""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "packet-rs_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=1 << 20)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--pushes", default="65536,1048576,16777216")
    ap.add_argument("--step-bytes", type=int, default=0)
    a = ap.parse_args()
    import torch  # noqa: F401  (the device columns are torch tensors)
    import pktgpu
    from pktgpu import gen
    from pktgpu.stream import PcapStream
    buf, offs, lens = gen.gen_c4(a.records, seed=0x5EED0007)
    n = a.records
    P = pktgpu.Parser(0)
    hb = P.host_empty((buf.size,), np.uint8)
    hb[:] = buf
    for out in ("dev", "pinned"):
        st = PcapStream(0, max_bytes=buf.size + 64, cap=n, columns="all", out=None if out == "dev" else "pinned",
                        step_bytes=a.step_bytes)
        st.close()  # the buffers are allocated; each rep opens its own stream (a fresh capture)
        for push in (int(x) for x in a.pushes.split(",")):
            ts = []
            for _ in range(a.reps):
                st = PcapStream(0, max_bytes=buf.size + 64, cap=n, columns="all",
                                out=None if out == "dev" else "pinned", step_bytes=a.step_bytes)
                try:
                    t0 = time.perf_counter()
                    for p0 in range(0, buf.size, push):
                        st.push(hb[p0:p0 + push])
                    c, _ = st.finish(index=False)
                    ts.append(time.perf_counter() - t0)
                    assert c == n, (c, n)
                finally:
                    st.close()
            t = float(np.median(ts))
            print(json.dumps({"what": "pkt_pcap_stream", "columns": out, "push_bytes": push,
                              "step_bytes": a.step_bytes or (4 << 20), "records": n, "file_bytes": int(buf.size),
                              "ms": round(t * 1e3, 3), "Grecords_s": round(n / t / 1e9, 4),
                              "in_GBps": round(buf.size / t / 1e9, 2)}), flush=True)
    P.close()


if __name__ == "__main__":
    main()
