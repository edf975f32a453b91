import sys, time, os
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "packet-rs_amd"))
import numpy as np, pktgpu
from pktgpu import gen, schema
n = 1 << 20
buf, offs, lens = gen.gen_c4(n, seed=0x5EED0006)
P = pktgpu.Parser(0)
hb = P.host_empty((buf.size,), np.uint8); hb[:] = buf
out = {c: P.host_empty(schema.column_shape(c, n), schema.column_dtype(c)) for c in schema.COLUMN_NAMES}
for piece in (1 << 20, 4 << 20, 16 << 20):
    P.set_host_piece(piece)
    for rep in range(3):
        t0 = time.perf_counter(); P.parse_pcap_host_async(hb, n, out); t1 = time.perf_counter()
        m = P.pcap_host_result(); t2 = time.perf_counter()
        print(piece, rep, "queue ms %.3f total ms %.3f" % ((t1-t0)*1e3, (t2-t0)*1e3), m == n, flush=True)
