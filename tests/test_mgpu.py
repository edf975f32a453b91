"""The multi-GPU entry of the C ABI (pkt_mgpu_*, pkt_out_packed, pkt_shard_range).

CPU tests: the packed layout and the shard split are host-only functions of the library; they
are checked against the Python schema and pktgpu.dist's split.  GPU tests: one process drives
the box's devices through pkt_mgpu (ncclCommInitAll + grouped ncclSend/ncclRecv; a 1-GPU box
gives ndev = 1, where the root's block is an RCCL send to itself) and the gathered tuples must
equal the oracle's over the whole batch — fast::parse is a pure function of each packet
(reference src/parser/fast.rs:5-12), so sharding must not change a single byte.
"""
import ctypes

import numpy as np
import pytest

import oracle
from pktgpu import _lib, dist, gen, schema


def _L():
    return _lib.load()


def test_packed_layout_matches_schema():
    L = _L()
    rng = np.random.default_rng(3)
    for trial in range(60):
        cols = [c for c in schema.COLUMN_NAMES if rng.random() < 0.5] or ["status"]
        n = int(rng.integers(0, 5000))
        mask = schema.column_mask(cols)
        o = _lib.PktOut()
        nb = ctypes.c_uint64()
        base = 1 << 20
        assert L.pkt_out_packed(mask, n, ctypes.c_void_p(base), ctypes.byref(o), ctypes.byref(nb)) == 0
        off, at = 0, {}
        slot = ("hdr_type", "hdr_off")  # the slot columns come last (ABI v4)
        for c in [c for c in schema.COLUMN_NAMES if c not in slot] + list(slot):
            p = getattr(o, c)
            if c not in cols:
                assert p is None, c
                continue
            assert p == base + off, (c, p - base, off)
            at[c] = off
            sz = int(np.prod(schema.column_shape(c, n))) * schema.column_dtype(c).itemsize
            off += (sz + 255) // 256 * 256
        assert nb.value == off
        assert L.pkt_out_mask(ctypes.byref(o)) == mask
        # the pieces that hold every column with `rows` slot rows
        rows = int(rng.integers(0, schema.MAX_HDRS + 1))
        po, pl, npc = (ctypes.c_uint64 * 2)(), (ctypes.c_uint64 * 2)(), ctypes.c_int()
        assert L.pkt_out_packed_pieces(mask, n, rows, po, pl, ctypes.byref(npc)) == 0
        covered = np.zeros(off, bool)
        for k in range(npc.value):
            covered[po[k]:po[k] + pl[k]] = True
        need = np.zeros(off, bool)
        for c in cols:
            sz = int(np.prod(schema.column_shape(c, n))) * schema.column_dtype(c).itemsize
            if c in slot:
                sz = rows * n * schema.column_dtype(c).itemsize
            need[at[c]:at[c] + sz] = True
        assert not (need & ~covered).any(), (cols, n, rows)
        moved = sum(pl[k] for k in range(npc.value))
        slack = 255 * (len(cols) + 1)
        assert moved <= need.sum() + slack, (moved, need.sum())
        assert npc.value == (2 if ("hdr_type" in cols and "hdr_off" in cols and rows and n) else 1)
    assert L.pkt_out_packed(1 << 49, 10, None, None, ctypes.byref(nb)) != 0
    po, pl, npc = (ctypes.c_uint64 * 2)(), (ctypes.c_uint64 * 2)(), ctypes.c_int()
    assert L.pkt_out_packed_pieces(1, 10, schema.MAX_HDRS + 1, po, pl, ctypes.byref(npc)) != 0


def test_packed_pieces_c2_bytes_per_packet():
    """a C2 shard's chain + Ether/IPv4/UDP tuples with their 3 used slot rows are
    69 B per packet (+ 256-B column alignment), not the 108 B of all 16 rows."""
    L = _L()
    n = 1 << 21
    cols = schema.columns_of(["chain", "ether", "ipv4", "udp"])
    po, pl, npc = (ctypes.c_uint64 * 2)(), (ctypes.c_uint64 * 2)(), ctypes.c_int()
    assert L.pkt_out_packed_pieces(schema.column_mask(cols), n, 3, po, pl, ctypes.byref(npc)) == 0
    moved = sum(pl[k] for k in range(npc.value))
    assert 69 * n <= moved <= 69 * n + 256 * len(cols), moved / n


def test_shard_range_matches_dist():
    L = _L()
    lo, hi = ctypes.c_uint64(), ctypes.c_uint64()
    for n in (0, 1, 7, 8, 9, 1 << 20, (1 << 24) + 3):
        for k in (1, 2, 3, 4, 7, 8):
            prev = 0
            for i in range(k):
                assert L.pkt_shard_range(n, k, i, ctypes.byref(lo), ctypes.byref(hi)) == 0
                assert (lo.value, hi.value) == dist.shard_range(n, k, i)
                assert lo.value == prev
                prev = hi.value
            assert prev == n
    assert L.pkt_shard_range(10, 0, 0, ctypes.byref(lo), ctypes.byref(hi)) != 0
    assert L.pkt_shard_range(10, 2, 2, ctypes.byref(lo), ctypes.byref(hi)) != 0


def _packed_offsets(L, mask, n):
    """{column: byte offset} of an n-packet packed buffer (pkt_out_packed) and its size."""
    o = _lib.PktOut()
    nb = ctypes.c_uint64()
    base = 1 << 40
    assert L.pkt_out_packed(mask, n, ctypes.c_void_p(base), ctypes.byref(o), ctypes.byref(nb)) == 0
    return {c: getattr(o, c) - base for c in schema.COLUMN_NAMES if getattr(o, c)}, nb.value


def _pack(L, cols, res, lo, hi):
    """Packets [lo, hi) of an oracle result as the shard's packed buffer (bytes)."""
    mask = schema.column_mask(cols)
    n = hi - lo
    off, nb = _packed_offsets(L, mask, n)
    buf = np.full(max(nb, 1), 0xEE, np.uint8)  # poison: bytes the plan must not rely on
    for c in cols:
        v = res[c][:, lo:hi] if c in ("hdr_type", "hdr_off") else res[c][lo:hi]
        b = np.ascontiguousarray(v).view(np.uint8).reshape(-1)
        buf[off[c]:off[c] + b.size] = b
    return buf


def _unpack(L, cols, buf, base, n):
    mask = schema.column_mask(cols)
    off, _ = _packed_offsets(L, mask, n)
    out = {}
    for c in cols:
        dt = schema.column_dtype(c)
        shp = schema.column_shape(c, n)
        nbytes = int(np.prod(shp)) * dt.itemsize
        out[c] = buf[base + off[c]:base + off[c] + nbytes].view(dt).reshape(shp)
    return out


@pytest.mark.parametrize("nd", [2, 3, 8])
@pytest.mark.parametrize("merge", [False, True])
@pytest.mark.parametrize("cfg", ["c2", "c4"])
def test_gather_plan_executed_on_host(nd, merge, cfg):
    """pkt_mgpu_parse_gather's message plan (pkt_gather_plan, the same function the
    device gather issues) executed with host memcpy over oracle-parsed packed shards of uneven size
    (an empty shard among them): the root buffer must hold exactly the whole batch's oracle output
    (merge = 1), or each shard's tuples at its 256-B aligned block (merge = 0) — sharding is legal
    because fast::parse is pure per packet (reference src/parser/fast.rs:5-12)."""
    from pktgpu import mgpu
    L = _L()
    rng = np.random.default_rng(nd * 7 + merge + (cfg == "c4"))
    cuts = sorted(int(x) for x in rng.integers(0, 4000, nd - 1))
    if nd >= 3:
        cuts[1] = cuts[0]  # an empty shard
    bounds = [0] + cuts + [4000 + nd]
    n = bounds[-1]
    if cfg == "c2":
        slab = gen.gen_c2(n, seed=nd)
        cols = schema.columns_of(["chain", "ether", "ipv4", "udp"])
        res = oracle.parse_batch(slab, n, stride=64, columns=cols, nthreads=8)
    else:
        buf, offs, lens = gen.gen_c4(n, seed=nd)
        cols = list(schema.COLUMN_NAMES)
        res = oracle.parse_batch(buf, n, offsets=offs, lens=lens, nthreads=8)
    ns = [bounds[i + 1] - bounds[i] for i in range(nd)]
    rows = [int(res["n_hdrs"][bounds[i]:bounds[i + 1]].max()) if ns[i] else 0 for i in range(nd)]
    shards = [_pack(L, cols, res, bounds[i], bounds[i + 1]) for i in range(nd)]
    plan, rb = mgpu.gather_plan(cols, ns, rows, merge)
    recv = np.full(rb, 0xCD, np.uint8)
    for shard, src, dst, nbytes in plan:
        assert ns[shard] and src + nbytes <= shards[shard].size and dst + nbytes <= rb
        recv[dst:dst + nbytes] = shards[shard][src:src + nbytes]
    if merge:
        _compare(_unpack(L, cols, recv, 0, n), res, f"{cfg} nd={nd} merged")
    else:
        o = 0
        for i in range(nd):
            if ns[i]:
                sub = {k: (v[:, bounds[i]:bounds[i + 1]] if k in ("hdr_type", "hdr_off") else v[bounds[i]:bounds[i + 1]])
                       for k, v in res.items()}
                _compare(_unpack(L, cols, recv, o, ns[i]), sub, f"{cfg} nd={nd} shard {i}")
            o += (_packed_offsets(L, schema.column_mask(cols), ns[i])[1] + 255) // 256 * 256
    # rows = None moves all 16 slot rows; the plan's receive size is independent of rows
    plan16, rb16 = mgpu.gather_plan(cols, ns, None, merge)
    assert rb16 == rb and sum(p[3] for p in plan16) >= sum(p[3] for p in plan)


def test_gather_plan_rejects_bad_arguments():
    L = _L()
    n = (ctypes.c_uint64 * 2)(5, 6)
    cnt, rb = ctypes.c_uint64(), ctypes.c_uint64()
    assert L.pkt_gather_plan(1 << 49, 2, n, None, 0, None, 0, ctypes.byref(cnt), ctypes.byref(rb)) != 0
    assert L.pkt_gather_plan(3, 0, n, None, 0, None, 0, ctypes.byref(cnt), ctypes.byref(rb)) != 0
    assert L.pkt_gather_plan(3, 2, n, None, 2, None, 0, ctypes.byref(cnt), ctypes.byref(rb)) != 0
    bad_rows = (ctypes.c_uint32 * 2)(3, 17)
    assert L.pkt_gather_plan(3, 2, n, bad_rows, 0, None, 0, ctypes.byref(cnt), ctypes.byref(rb)) != 0
    assert L.pkt_gather_plan(3, 2, n, None, 0, None, 5, ctypes.byref(cnt), ctypes.byref(rb)) != 0
    assert L.pkt_sizeof_gather_piece() == ctypes.sizeof(_lib.PktGatherPiece) == 32


def test_mgpu_create_rejects_bad_device_lists():
    L = _L()
    h = ctypes.c_void_p()
    assert L.pkt_mgpu_create(None, 1, ctypes.byref(h)) != 0
    arr = (ctypes.c_int * 1)(0)
    assert L.pkt_mgpu_create(arr, 0, ctypes.byref(h)) != 0
    arr2 = (ctypes.c_int * 2)(0, 0)
    assert L.pkt_mgpu_create(arr2, 2, ctypes.byref(h)) != 0  # duplicate device (or no device)
    assert not h.value


# ------------------------------------------------------------------------------------------ GPU
def _compare(g, o, label):
    for k, ov in o.items():
        gv = g[k].cpu().numpy() if hasattr(g[k], "cpu") else g[k]
        if k in ("hdr_type", "hdr_off"):
            valid = np.arange(schema.MAX_HDRS)[:, None] < o["n_hdrs"].astype(np.int64)[None, :]
            assert not (valid & (gv != ov)).any(), f"{label} {k}"
        else:
            assert np.array_equal(gv, ov), f"{label} {k}"


@pytest.fixture(scope="module")
def MP():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.fail("no GPU visible: -m gpu tests need an MI355X")
    from pktgpu.mgpu import MultiParser
    return MultiParser(list(range(torch.cuda.device_count())))


@pytest.mark.gpu
@pytest.mark.parametrize("merge", [False, True])
def test_mgpu_c2_parse_gather_vs_oracle(MP, merge):
    n = 100_003
    slab = gen.gen_c2(n, seed=77)
    cols = schema.columns_of(["chain", "ether", "ipv4", "udp"])
    shards = MP.shard_fixed(slab, n, 64)
    views, recv, _ = MP.parse_gather(shards, columns=cols, merge=merge)
    MP.synchronize()
    o = oracle.parse_batch(slab, n, stride=64, columns=cols, nthreads=8)
    if merge:
        _compare(views, o, "merged")
    else:
        assert len(views) == MP.ndev
        merged = {}
        for c in cols:
            parts = [v[c].cpu().numpy() for v in views if v]
            merged[c] = np.concatenate(parts, axis=1 if c in ("hdr_type", "hdr_off") else 0)
        _compare(merged, o, "per-shard")


@pytest.mark.gpu
def test_mgpu_c4_pcap_all_columns_vs_oracle(MP):
    n = 20_000
    buf, offs, lens = gen.gen_c4(n, seed=41)
    shards = MP.shard_indexed(buf, offs, lens)
    views, _, _ = MP.parse_gather(shards, columns="all", merge=True)
    MP.synchronize()
    o = oracle.parse_batch(buf, n, offsets=offs, lens=lens, nthreads=8)
    _compare(views, o, "c4 merged")


@pytest.mark.gpu
def test_mgpu_parse_only_and_entries(MP):
    """pkt_mgpu_parse alone (no gather) into the packed shard buffers, a non-default entry."""
    from pktgpu.mgpu import packed_views
    n = 4099
    rng = np.random.default_rng(5)
    slab = rng.integers(0, 256, n * 48, dtype=np.uint8)
    cols = schema.columns_of(["chain", "ipv4", "udp"])
    shards = MP.shard_fixed(slab, n, 48)
    bufs = MP.parse(shards, entry="parse_ipv4", columns=cols)
    MP.synchronize()
    o = oracle.parse_batch(slab, n, stride=48, entry="parse_ipv4", columns=cols, nthreads=8)
    lo = 0
    for (s, ni, *_), b in zip(shards, bufs):
        if not ni:
            continue
        v = packed_views(b, cols, ni)
        sub = {k: (val[:, lo:lo + ni] if k in ("hdr_type", "hdr_off") else val[lo:lo + ni]) for k, val in o.items()}
        _compare(v, sub, "parse_ipv4 shard")
        lo += ni
    assert lo == n


@pytest.mark.gpu
def test_mgpu_orders_after_torch_stream(MP):
    """a shard produced asynchronously on torch's stream (a Generator.run slab) goes
    straight into parse_gather, and the gathered columns are read back through torch (.cpu() on
    torch's current stream) with no explicit synchronisation in between."""
    import torch
    from pktgpu import Parser, pktgen
    P = Parser(MP.devices[0])
    n, stride = 1 << 16, 64
    g = pktgen.Generator(P, pktgen.udp_template(), [pktgen.Field("IPv4", "src", kind="random", base=11),
                                                    pktgen.Field("UDP", "dst", kind="inc", step=7)], csum=[0])
    cols = schema.columns_of(["chain", "ether", "ipv4", "udp"])
    for rep in range(3):
        torch.cuda.current_stream(MP.torch_devices[0]).synchronize()
        slab = g.run(n, stride, first=rep * n)            # queued on torch's stream, not waited for
        shards = [(slab, n, stride, None, None)]
        views, recv, _ = MP.parse_gather(shards, columns=cols, merge=True)
        got = {k: v.cpu().numpy() for k, v in views.items()}  # torch's stream waits for the gather
        ref = oracle.parse_batch(slab.cpu().numpy(), n, stride=stride, columns=cols, nthreads=8)
        _compare(got, ref, f"generator -> parse_gather rep {rep}")
    g.close()
    P.close()


@pytest.mark.gpu
def test_bench_mgpu_leg_at_one_device():
    """bench.py's measured path is the library's multi-device entry
    (pkt_mgpu_parse_steps + pkt_mgpu_parse_gather); run it at ndev = 1 with small sizes and check the
    line's shape and that the C5 gather moved only the used slot rows (69 B per C2 packet)."""
    import json
    import os
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", "1", "--steps", "6",
                        "--warmup", "2", "--no-cpu-baseline", "--no-extra", "--ring-gib", "0.25",
                        "--total-packets", str(1 << 21)], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 1 and line["value"] > 0 and line["scaling"] == "weak"
    assert "pkt_mgpu_parse_steps" in line["config"]["launch"]
    assert line["roofline"]["frac"] > 0
    g = line["c5"]["gather"]
    assert g["slot_rows_moved"] == 3
    assert 69 <= g["bytes_per_pkt_moved"] <= 70, g
    assert g["bytes_into_root"] > 0 and g["rccl_messages"] >= 2, g  # RCCL moved the root's own shard


@pytest.mark.gpu
@pytest.mark.parametrize("merge", [False, True])
@pytest.mark.parametrize("cfg", ["c2", "c4"])
def test_mgpu_parse_gather_rccl_root_self_send(MP, merge, cfg):
    """with pkt_mgpu_set_root_copy(0) the root's own pieces go through RCCL
    (ncclSend / ncclRecv to itself inside the group), so on a 1-GPU box the gather still executes
    RCCL transfers; the result must equal the oracle over the whole batch."""
    MP.set_root_copy(False)
    try:
        if cfg == "c2":
            n = 65_537
            slab = gen.gen_c2(n, seed=78)
            cols = schema.columns_of(["chain", "ether", "ipv4", "udp"])
            shards = MP.shard_fixed(slab, n, 64)
            o = oracle.parse_batch(slab, n, stride=64, columns=cols, nthreads=8)
        else:
            n = 30_011
            buf, offs, lens = gen.gen_c4(n, seed=79)
            cols = list(schema.COLUMN_NAMES)
            shards = MP.shard_indexed(buf, offs, lens)
            o = oracle.parse_batch(buf, n, offsets=offs, lens=lens, nthreads=8)
        for rep in range(2):
            views, recv, _ = MP.parse_gather(shards, columns=cols, merge=merge)
            MP.synchronize()
            if merge:
                _compare(views, o, f"{cfg} merged rccl-self rep {rep}")
            else:
                merged = {c: np.concatenate([v[c].cpu().numpy() for v in views if v],
                                            axis=1 if c in ("hdr_type", "hdr_off") else 0) for c in cols}
                _compare(merged, o, f"{cfg} per-shard rccl-self rep {rep}")
    finally:
        MP.set_root_copy(True)


@pytest.mark.gpu
@pytest.mark.parametrize("streams", [1, 4])
def test_mgpu_parse_steps_vs_oracle(MP, streams):
    """pkt_mgpu_parse_steps (the bench's timed entry) with several steps of distinct
    inputs and outputs, round-robin over 1 or 4 streams, one step with n = 0 and no output: after
    synchronize() every step's packed output equals the oracle's parse of its own input."""
    import torch
    from pktgpu.mgpu import packed_bytes, packed_views
    nd = MP.ndev
    cols = schema.columns_of(["chain", "ether", "ipv4", "udp"])
    steps, refs = [], []
    for k in range(7):
        per_dev, ref_dev = [], []
        for i, d in enumerate(MP.torch_devices):
            n = 0 if k == 3 else 4096 * (k + 1) + 17 * i
            slab = gen.gen_c2(max(n, 1), seed=1000 + 10 * k + i) if n else np.zeros(64, np.uint8)
            t = torch.from_numpy(slab.reshape(-1)).to(d)
            out = torch.full((max(1, packed_bytes(cols, n)),), 0xEE, dtype=torch.uint8, device=d)
            per_dev.append(((t, n, 64, None, None), out))
            ref_dev.append((slab, n))
        steps.append(per_dev)
        refs.append(ref_dev)
    plan = MP.steps_plan(steps)
    b, o, _ = plan
    for i in range(nd):
        o[3 * nd + i] = None  # the empty step has no output buffer
    torch.cuda.synchronize()
    MP.parse_steps(plan, "parse", cols, streams=streams)
    MP.synchronize()
    for k in range(7):
        for i in range(nd):
            slab, n = refs[k][i]
            if not n:
                continue
            got = {c: v.cpu().numpy() for c, v in packed_views(steps[k][i][1], cols, n).items()}
            _compare(got, oracle.parse_batch(slab, n, stride=64, columns=cols, nthreads=8), f"step {k} dev {i}")


@pytest.mark.gpu
@pytest.mark.parametrize("root_copy", [True, False])
def test_mgpu_parse_gather_fixed_rows_and_repack(MP, root_copy):
    """pkt_mgpu_set_gather_rows(k) queues parse + gather with no host wait (k slot rows
    per shard, >= every n_hdrs), and merge = 1 is the merge = 0 transfer into the root's staging area
    plus the repack kernel (root copy on: the root's own pieces repacked straight from its shard
    buffer; off: through RCCL and the staging area).  Odd batch sizes put the slot rows at offsets that
    are not 16-byte aligned (the repack's head / tail bytes).  Every mode == oracle."""
    n = 40_001
    buf, offs, lens = gen.gen_c4(n, seed=81)
    cols = list(schema.COLUMN_NAMES)
    shards = MP.shard_indexed(buf, offs, lens)
    o = oracle.parse_batch(buf, n, offsets=offs, lens=lens, nthreads=8)
    rows_needed = int(o["n_hdrs"].max())
    MP.set_root_copy(root_copy)
    try:
        for rows in (16, rows_needed, 0):
            MP.set_gather_rows(rows)
            for merge in (True, False):
                views, recv, _ = MP.parse_gather(shards, columns=cols, merge=merge)
                MP.synchronize()
                if merge:
                    _compare(views, o, f"rows {rows} merged root_copy={root_copy}")
                else:
                    merged = {c: np.concatenate([v[c].cpu().numpy() for v in views if v],
                                                axis=1 if c in ("hdr_type", "hdr_off") else 0) for c in cols}
                    _compare(merged, o, f"rows {rows} per-shard root_copy={root_copy}")
    finally:
        MP.set_gather_rows(0)
        MP.set_root_copy(True)
