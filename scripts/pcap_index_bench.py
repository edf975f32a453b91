"""Device pcap indexer (pkt_pcap_index_device) vs the host indexer (pkt_pcap_index) on a C4-style
capture of N records: wall time per call (the device call is blocking: guess + repair rounds +
scan + emit, including its host round trips), records/s and file GB/s.  One JSON line."""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "packet-rs_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=1 << 20)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--no-check", action="store_true", help="timing experiments on broken variants")
    a = ap.parse_args()
    import torch
    import pktgpu
    from pktgpu import gen, _lib
    buf, offs, lens = gen.gen_c4(a.records, seed=0x5EED0004)
    P = pktgpu.Parser(0)
    d = torch.from_numpy(buf).cuda()
    o = torch.empty(a.records, dtype=torch.uint64, device="cuda")
    l = torch.empty(a.records, dtype=torch.uint32, device="cuda")
    n = ctypes.c_uint64()
    L = P._L
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

    def dev_call():
        rc = L.pkt_pcap_index_device(P._ctx, d.data_ptr(), d.numel(), o.data_ptr(), l.data_ptr(), a.records,
                                     ctypes.byref(n), s)
        assert rc == 0 or a.no_check, rc

    for _ in range(3):
        dev_call()
    torch.cuda.synchronize()
    if not a.no_check:
        assert n.value == a.records
        assert np.array_equal(o.cpu().numpy(), offs) and np.array_equal(l.cpu().numpy(), lens)
    t = []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        dev_call()
        t.append(time.perf_counter() - t0)
    dev_s = float(np.median(t))
    ho = np.empty(a.records, np.uint64)
    hl = np.empty(a.records, np.uint32)
    th = []
    for _ in range(5):
        t0 = time.perf_counter()
        rc = L.pkt_pcap_index(buf.ctypes.data, buf.size, ho.ctypes.data, hl.ctypes.data, a.records, ctypes.byref(n))
        th.append(time.perf_counter() - t0)
        assert rc == 0
    host_s = float(np.median(th))
    print(json.dumps({"what": "pcap_index", "records": a.records, "file_bytes": int(buf.size),
                      "device_us": round(dev_s * 1e6, 1), "device_min_us": round(min(t) * 1e6, 1),
                      "device_mrec_s": round(a.records / dev_s / 1e6, 1),
                      "device_file_GBps": round(buf.size / dev_s / 1e9, 1),
                      "host_us": round(host_s * 1e6, 1), "host_mrec_s": round(a.records / host_s / 1e6, 1),
                      "speedup": round(host_s / dev_s, 2)}))


if __name__ == "__main__":
    main()
