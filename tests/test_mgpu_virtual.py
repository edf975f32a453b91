"""The N-shard code paths of pkt_mgpu on one GPU: pkt_mgpu_create_virtual.

A virtual handle lists device 0 several times (nd = 2, 3, 8 shards, each with its own ctx and
streams) and moves the gather's messages by device copies instead of RCCL, so on a one-GPU box it
runs what only an 8-GPU node would otherwise reach: pkt_mgpu_parse_steps' per-shard issuing threads,
shard offsets for N > 1, gather plans with pieces from several shards, the merged gather's staging
area and repack over several shards, and bench.py's ndev > 1 loops.  Shards are uneven with one
empty shard.  Every result must equal the oracle over the whole batch: fast::parse is a pure
function of each packet (reference src/parser/fast.rs:5-12), so sharding must not change a byte.
"""
import ctypes

import numpy as np
import pytest

import oracle
from pktgpu import _lib, gen, schema

SLOT = ("hdr_type", "hdr_off")


def _compare(g, o, label):
    for k, ov in o.items():
        gv = g[k].cpu().numpy() if hasattr(g[k], "cpu") else g[k]
        if k in SLOT:
            valid = np.arange(schema.MAX_HDRS)[:, None] < o["n_hdrs"].astype(np.int64)[None, :]
            assert not (valid & (gv != ov)).any(), f"{label} {k}"
        else:
            assert np.array_equal(gv, ov), f"{label} {k}"


def _uneven_bounds(n, nd, seed):
    """nd + 1 bounds from 0 to n: random cut points, shard 1 empty when nd >= 3 (shard 0 when nd = 2
    keeps a record so the root always has work in one case and none in another across tests)."""
    rng = np.random.default_rng(seed)
    cuts = sorted(int(x) for x in rng.integers(1, n, nd - 1))
    if nd >= 3:
        cuts[1] = cuts[0]
    return [0] + cuts + [n]


def test_create_virtual_rejects_bad_arguments():
    L = _lib.load()
    h = ctypes.c_void_p()
    assert L.pkt_mgpu_create_virtual(None, 2, ctypes.byref(h)) != 0
    arr = (ctypes.c_int * 1)(0)
    assert L.pkt_mgpu_create_virtual(arr, 0, ctypes.byref(h)) != 0
    bad = (ctypes.c_int * 2)(0, -1)
    assert L.pkt_mgpu_create_virtual(bad, 2, ctypes.byref(h)) != 0
    assert not h.value
    assert L.pkt_mgpu_is_virtual(None) == 0


_HANDLES = {}


def _mp(nd):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.fail("no GPU visible: -m gpu tests need an MI355X")
    from pktgpu.mgpu import MultiParser
    if nd not in _HANDLES:
        _HANDLES[nd] = MultiParser([0] * nd, virtual=True)
    mp = _HANDLES[nd]
    assert mp._L.pkt_mgpu_is_virtual(mp._mg) == 1 and mp._L.pkt_mgpu_ndev(mp._mg) == nd
    return mp


@pytest.fixture(scope="module", autouse=True)
def _close_handles():
    yield
    for mp in _HANDLES.values():
        mp.close()
    _HANDLES.clear()


@pytest.mark.gpu
@pytest.mark.parametrize("nd", [2, 3, 8])
@pytest.mark.parametrize("streams", [1, 4])
def test_virtual_parse_steps_vs_oracle(nd, streams):
    """pkt_mgpu_parse_steps at nd shards: one issuing host thread per shard, round-robin over 1 or 4
    streams per shard; per-shard sizes differ, one shard is empty in every step and one whole step is
    empty; each step's packed output == the oracle's parse of its own input."""
    import torch
    from pktgpu.mgpu import packed_bytes, packed_views
    MP = _mp(nd)
    cols = schema.columns_of(["chain", "ether", "ipv4", "udp"])
    steps, refs = [], []
    for k in range(5):
        per_dev, ref_dev = [], []
        for i, d in enumerate(MP.torch_devices):
            n = 0 if (k == 2 or i == (k % nd)) else 1500 * (k + 1) + 37 * i
            slab = gen.gen_c2(max(n, 1), seed=2000 + 16 * k + i) if n else np.zeros(64, np.uint8)
            t = torch.from_numpy(slab.reshape(-1)).to(d)
            out = torch.full((max(1, packed_bytes(cols, n)),), 0xEE, dtype=torch.uint8, device=d)
            per_dev.append(((t, n, 64, None, None), out))
            ref_dev.append((slab, n))
        steps.append(per_dev)
        refs.append(ref_dev)
    plan = MP.steps_plan(steps)
    _, o, _ = plan
    for i in range(nd):
        o[2 * nd + i] = None  # the empty step has no output buffers
    torch.cuda.synchronize()
    MP.parse_steps(plan, "parse", cols, streams=streams)
    MP.synchronize()
    for k in range(5):
        for i in range(nd):
            slab, n = refs[k][i]
            if not n:
                continue
            got = {c: v.cpu().numpy() for c, v in packed_views(steps[k][i][1], cols, n).items()}
            _compare(got, oracle.parse_batch(slab, n, stride=64, columns=cols, nthreads=8),
                     f"nd={nd} streams={streams} step {k} shard {i}")


@pytest.mark.gpu
@pytest.mark.parametrize("nd", [2, 3, 8])
@pytest.mark.parametrize("cfg", ["c2", "c4"])
def test_virtual_parse_gather_vs_oracle(nd, cfg):
    """pkt_mgpu_parse_gather at nd uneven shards (one empty): merge 0 and 1, slot rows measured
    (0) and fixed (the batch's bound, and 16), root copy on and off, root 0 and the last shard;
    every gathered byte the oracle defines equals the oracle over the whole batch."""
    MP = _mp(nd)
    if cfg == "c2":
        n = 30_011 + nd
        slab = gen.gen_c2(n, seed=300 + nd)
        cols = schema.columns_of(["chain", "ether", "ipv4", "udp"])
        bounds = _uneven_bounds(n, nd, nd)
        shards = MP.shard_fixed(slab, n, 64, bounds=bounds)
        o = oracle.parse_batch(slab, n, stride=64, columns=cols, nthreads=8)
    else:
        n = 12_007 + nd
        buf, offs, lens = gen.gen_c4(n, seed=400 + nd)
        cols = list(schema.COLUMN_NAMES)
        bounds = _uneven_bounds(n, nd, 10 + nd)
        shards = MP.shard_indexed(buf, offs, lens, bounds=bounds)
        o = oracle.parse_batch(buf, n, offsets=offs, lens=lens, nthreads=8)
    assert [s[1] for s in shards] == [b - a for a, b in zip(bounds, bounds[1:])]
    need = int(o["n_hdrs"].max())
    try:
        for root in (0, nd - 1):
            for root_copy in (True, False):
                MP.set_root_copy(root_copy)
                for rows in (0, need, 16):
                    MP.set_gather_rows(rows)
                    for merge in (False, True):
                        label = f"{cfg} nd={nd} root={root} root_copy={root_copy} rows={rows} merge={merge}"
                        views, recv, _ = MP.parse_gather(shards, columns=cols, root=root, merge=merge)
                        MP.synchronize()
                        assert recv.device == MP.torch_devices[root]
                        if merge:
                            _compare(views, o, label)
                        else:
                            assert len(views) == nd
                            for i, (a, b) in enumerate(zip(bounds, bounds[1:])):
                                if a == b:
                                    assert views[i] == {}, label
                                    continue
                                sub = {k: (v[:, a:b] if k in SLOT else v[a:b]) for k, v in o.items()}
                                _compare(views[i], sub, f"{label} shard {i}")
    finally:
        MP.set_gather_rows(0)
        MP.set_root_copy(True)


@pytest.mark.gpu
def test_virtual_fixed_rows_below_n_hdrs_is_reported():
    """with pkt_mgpu_set_gather_rows(k) below some packet's n_hdrs, the rows past k are not
    gathered; the next synchronize returns PKT_ERR_GATHER_ROWS instead of passing silently, and the
    handle works normally afterwards."""
    MP = _mp(3)
    n = 5003
    buf, offs, lens = gen.gen_c4(n, seed=91)
    cols = list(schema.COLUMN_NAMES)
    shards = MP.shard_indexed(buf, offs, lens)
    o = oracle.parse_batch(buf, n, offsets=offs, lens=lens, nthreads=8)
    need = int(o["n_hdrs"].max())
    assert need > 2
    MP.set_gather_rows(2)
    try:
        MP.parse_gather(shards, columns=cols, merge=True)
        with pytest.raises(RuntimeError, match="slot rows"):
            MP.synchronize()
        assert MP._L.pkt_mgpu_synchronize(MP._mg) == 0  # reported once
        MP.set_gather_rows(need)
        views, _, _ = MP.parse_gather(shards, columns=cols, merge=True)
        MP.synchronize()
        _compare(views, o, "rows = need after the reported shortfall")
    finally:
        MP.set_gather_rows(0)


@pytest.mark.gpu
def test_bench_virtual_eight_shards_smoke():
    """bench.py --gpus 8 --virtual: the bench's ndev > 1 loops (run_mgpu's per-shard inputs and rings,
    pkt_mgpu_parse_steps with 8 issuing threads, run_c5_mgpu's 8 shards and every gather form) to
    completion on one GPU; the line is labelled a smoke, not a measurement or a scaling point."""
    import json
    import os
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", "8", "--virtual", "--steps", "4",
                        "--warmup", "1", "--no-cpu-baseline", "--ring-gib", "0.0625",
                        "--total-packets", str((1 << 21) + 5)], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["metric"].startswith("VIRTUAL SMOKE") and line["n_gpus"] == 1 and line["virtual_shards"] == 8
    assert line["scaling"] is None and line["value"] > 0
    c5 = line["c5"]
    assert len(c5["packets_per_gpu"]) == 8 and sum(c5["packets_per_gpu"]) == (1 << 21) + 5
    g = c5["gather"]
    assert g["slot_rows_moved"] == 3 and 69 <= g["bytes_per_pkt_moved"] <= 70, g
    assert g["bytes_from_other_devices"] > 0 and g["rccl_messages"] >= 16, g
