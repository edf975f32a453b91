"""pkt_view (include/pktgpu.h): the PacketSlice of one packet from host chain columns — what the Rust
adapter in INTEGRATION.md builds the reference's own PacketSlice from (lib.rs:136-140,
packet.rs:714-731).  CPU tests: the columns come from the oracle (C restatement of fast.rs) and the
view is checked against the golden ref22 chains (tests/golden/ref22_expected.json) and against the
independent forward walk of tests/pyref.py; the GPU variant takes the columns from the HIP parse."""
import ctypes
import json
import os

import numpy as np
import pytest

import oracle
import pyref
import pktgpu
from pktgpu import _lib, gen, schema

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _check_against_pyref(res, pkts, label):
    for i, p in enumerate(pkts):
        st, hl, po, pl = pktgpu.view(res, i)
        rst, rh, rpo, rpl = pyref.parse(p)
        assert schema.STATUS_NAMES[st] == rst, (label, i)
        if rst == "OK":
            assert [(schema.HDR_NAMES[t], o) for t, o in hl] == [tuple(x) for x in rh], (label, i)
            assert (po, pl) == (rpo, rpl), (label, i)
        else:
            assert hl == [] and po == 0 and pl == 0, (label, i)


def test_view_ref22_golden():
    pc = open(os.path.join(GOLD, "ref22.pcap"), "rb").read()
    offs, lens = pktgpu.pcap_index(pc)
    res = oracle.parse_batch(np.frombuffer(pc, np.uint8), len(offs), offsets=offs, lens=lens)
    exp = json.load(open(os.path.join(GOLD, "ref22_expected.json")))
    assert len(exp) == len(offs) == 22
    for i, e in enumerate(exp):
        st, hl, po, pl = pktgpu.view(res, i)
        assert schema.STATUS_NAMES[st] == e["status"]
        assert [[schema.HDR_NAMES[t], o] for t, o in hl] == e["hdrs"], e["name"]
        assert (po, pl) == (e["payload_off"], e["payload_len"]), e["name"]
        sl = pktgpu.packet_slice(res, i, pc[offs[i]:offs[i] + lens[i]])  # built through pkt_view
        assert sl.to_vec() == pc[offs[i]:offs[i] + lens[i]] or e["name"].startswith("gre")


def test_view_c4_and_truncations_vs_pyref():
    buf, offs, lens = gen.gen_c4(3000, seed=8)
    res = oracle.parse_batch(buf, len(offs), offsets=offs, lens=lens)
    _check_against_pyref(res, [bytes(buf[o:o + l]) for o, l in zip(offs, lens)], "c4")
    tm = [p.to_vec() for p in gen.reference_22_packets()]
    pk = [t[:k] for t in tm for k in range(0, len(t), 7)]
    b = b"".join(pk)
    ln = np.array([len(x) for x in pk], np.uint32)
    of = np.concatenate([[0], np.cumsum(ln)[:-1]]).astype(np.uint64)
    res = oracle.parse_batch(np.frombuffer(b + bytes(16), np.uint8), len(pk), offsets=of, lens=ln)
    _check_against_pyref(res, pk, "truncations")


def test_view_rejects_bad_arguments():
    L = _lib.load()
    res = oracle.parse_batch(gen.gen_c2(4, seed=1), 4, stride=64)
    cols = {c: np.ascontiguousarray(res[c]) for c in ("status", "n_hdrs", "hdr_type", "hdr_off",
                                                       "payload_off", "payload_len")}
    o = _lib.PktOut()
    for c, a in cols.items():
        setattr(o, c, a.ctypes.data)
    ty, of = (ctypes.c_uint8 * 16)(), (ctypes.c_uint16 * 16)()
    nh, po, pl = ctypes.c_uint32(), ctypes.c_uint16(), ctypes.c_uint16()
    args = (ty, of, ctypes.byref(nh), ctypes.byref(po), ctypes.byref(pl))
    assert L.pkt_view(ctypes.byref(o), 4, 3, *args) == 0 and nh.value == 3
    assert L.pkt_view(ctypes.byref(o), 4, 4, *args) < 0          # i >= n
    assert L.pkt_view(None, 4, 0, *args) < 0
    o.hdr_off = None
    assert L.pkt_view(ctypes.byref(o), 4, 0, *args) < 0          # a chain column missing


@pytest.mark.gpu
def test_view_of_gpu_columns_vs_pyref():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.fail("no GPU visible")
    P = pktgpu.Parser(0)
    try:
        buf, offs, lens = gen.gen_c4(1 << 16, seed=9)
        g = P.parse(torch.from_numpy(buf).cuda(), offsets=torch.from_numpy(offs).cuda(),
                    lens=torch.from_numpy(lens).cuda(), columns=["chain"])
        host = {k: v.cpu().numpy() for k, v in g.items()}
        idx = np.random.default_rng(3).choice(len(offs), 3000, replace=False)
        sub = {k: (v[:, idx] if k in ("hdr_type", "hdr_off") else v[idx]) for k, v in host.items()}
        _check_against_pyref(sub, [bytes(buf[offs[i]:offs[i] + lens[i]]) for i in idx], "gpu c4")
    finally:
        P.close()


@pytest.mark.gpu
def test_view_of_gpu_columns_vs_oracle_columns():
    """pkt_view over the HIP parse's chain columns equals pkt_view over the oracle's (the C
    restatement of fast.rs pinned by the reference's own fixtures) for every packet of a C4 batch with
    truncated records: the view the Rust adapter builds PacketSlice from is anchored on the oracle, not
    only on the independent walk of tests/pyref.py."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.fail("no GPU visible")
    P = pktgpu.Parser(0)
    try:
        n = 1 << 15
        buf, offs, lens = gen.gen_c4(n, seed=12)
        rng = np.random.default_rng(12)
        cut = rng.random(n) < 0.05
        lens = np.where(cut, (lens * rng.random(n)).astype(np.uint32), lens).astype(np.uint32)
        g = P.parse(torch.from_numpy(buf).cuda(), offsets=torch.from_numpy(offs).cuda(),
                    lens=torch.from_numpy(lens).cuda(), columns=["chain"])
        host = {k: v.cpu().numpy() for k, v in g.items()}
        ref = oracle.parse_batch(buf, n, offsets=offs, lens=lens, columns=list(host), nthreads=8)
        for i in range(n):
            assert pktgpu.view(host, i) == pktgpu.view(ref, i), i
    finally:
        P.close()
