"""world_size-2 gloo tests of the multi-GPU path: contiguous sharding (even, uneven and
pcap-indexed), per-rank parse, and the tuple gather reassembled in global order must equal the
single-process parse of the whole batch.  CPU variant: the per-rank compute is the oracle (no
GPU here).  GPU variant (-m gpu): each rank parses its shard with the HIP path (pktgpu.Parser;
both ranks share the box's one device) and the gathered tuples are checked against the oracle."""
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


def _worker(rank, world, port, case, q, use_gpu=False):
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
            if use_gpu:
                res = _gpu_parse(np.ascontiguousarray(view), nl, 128, None, None, cols)
            else:
                res = oracle.parse_batch(view, nl, stride=128, columns=cols)
        else:
            buf, offs, lens = gen.gen_c4(3001, seed=22)
            o, l, lo = pd.shard_indexed(offs, lens, world, rank)
            if use_gpu:
                res = _gpu_parse(buf, len(o), None, o, l, cols)
            else:
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


def _gpu_parse(slab, n, stride, offs, lens, cols):
    """This rank's shard through the HIP path; columns come back as CPU tensors (gloo)."""
    import torch
    import pktgpu
    P = pktgpu.Parser(0)
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    res = P.parse(d(np.frombuffer(slab, np.uint8) if isinstance(slab, bytes) else slab.reshape(-1)),
                  stride=stride, n=n, offsets=d(offs.astype(np.uint64)) if offs is not None else None,
                  lens=d(lens.astype(np.uint32)) if lens is not None else None, columns=cols)
    torch.cuda.synchronize()
    return {k: v.cpu() for k, v in res.items()}


def _run(case, use_gpu):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, case, q, use_gpu)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert q.get(timeout=10) == []


@pytest.mark.parametrize("case", ["even", "uneven", "pcap"])
def test_sharded_parse_and_gather_world2(case):
    _run(case, use_gpu=False)


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["uneven", "pcap"])
def test_sharded_hip_parse_and_gather_world2(case):
    _run(case, use_gpu=True)


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
