"""world_size-2 gloo tests (CPU) of the multi-GPU path: contiguous sharding (even, uneven and
pcap-indexed), per-rank parse, and the tuple gather reassembled in global order must equal the
single-process parse of the whole batch.  The per-rank compute here is the oracle (no GPU);
on GPUs the same code runs with pktgpu.Parser and the nccl (RCCL) backend."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, case, q):
    sys.path[:0] = [os.path.join(REPO, "packet-rs_amd"), os.path.join(REPO, "oracle")]
    import torch.distributed as dist
    import oracle
    from pktgpu import dist as pd, gen, resolve_columns
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cols = resolve_columns("all")
        if case in ("even", "uneven"):
            n = 4096 if case == "even" else 4099
            slab = gen.gen_c3(n, seed=21)
            flat = slab.reshape(-1)
            view, nl, _, lo = pd.shard_fixed(flat, n, 128, world, rank)
            res = oracle.parse_batch(view, nl, stride=128, columns=cols)
        else:
            buf, offs, lens = gen.gen_c4(3001, seed=22)
            o, l, lo = pd.shard_indexed(offs, lens, world, rank)
            res = oracle.parse_batch(buf, len(o), offsets=o, lens=l, columns=cols)
            nl = len(o)
        merged = pd.gather_columns(res, cols, nl, dst=0)
        if rank == 0:
            if case in ("even", "uneven"):
                whole = oracle.parse_batch(slab, n, stride=128, columns=cols)
            else:
                whole = oracle.parse_batch(buf, len(offs), offsets=offs, lens=lens, columns=cols)
            bad = []
            nh = whole["n_hdrs"].astype(int)
            for c in cols:
                if c in ("hdr_type", "hdr_off"):
                    m = np.arange(16)[:, None] < nh[None, :]
                    ok = np.array_equal(merged[c][m], whole[c][m])
                else:
                    ok = np.array_equal(merged[c], whole[c])
                if not ok:
                    bad.append(c)
            q.put(bad)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("case", ["even", "uneven", "pcap"])
def test_sharded_parse_and_gather_world2(case):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, case, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert q.get(timeout=10) == []


def test_shard_range_partition():
    sys.path.insert(0, os.path.join(REPO, "packet-rs_amd"))
    from pktgpu import dist as pd
    for n in (0, 1, 7, 64, 1 << 20, (1 << 24) + 3):
        for w in (1, 2, 3, 8):
            rs = [pd.shard_range(n, w, r) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(rs[i][1] == rs[i + 1][0] for i in range(w - 1))
            sz = [b - a for a, b in rs]
            assert max(sz) - min(sz) <= 1
