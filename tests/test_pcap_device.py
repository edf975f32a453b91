"""Device pcap indexer (pkt_pcap_index_device, §8(f) row 1) against the host indexer restated in
gen.pcap_index_py (pinned by the golden ref22.pcap, test_abi/test_oracle): identical records,
counts, cap behaviour and errors — on the golden capture, C4 replays, and captures built to
defeat the speculative guess (fake record chains inside payloads, zero payloads, records larger
than a 4 KiB region, zero-length records) so the exact fix-up rounds are what makes it right.
Ends with the whole device path: file in HBM -> device index -> indexed parse == oracle."""
import os
import struct

import numpy as np
import pytest

import oracle
from pktgpu import gen, schema

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def P():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.fail("no GPU visible")
    import pktgpu
    return pktgpu.Parser(0)


def dev(buf):
    import torch
    return torch.from_numpy(np.frombuffer(bytes(buf), np.uint8).copy()).cuda()


def check_index(P, buf, label):
    o_ref, l_ref = gen.pcap_index_py(bytes(buf))
    offs, lens, n = P.pcap_index(dev(buf))
    assert n == len(o_ref), (label, n, len(o_ref))
    assert np.array_equal(offs.cpu().numpy(), o_ref), label
    assert np.array_equal(lens.cpu().numpy(), l_ref), label


def records(payloads, ts=None, snap_trunc=None):
    out = bytearray(gen.PCAP_GLOBAL_HEADER)
    for i, p in enumerate(payloads):
        sec, usec = (ts[i] if ts else (0, 0))
        orig = len(p) + (snap_trunc[i] if snap_trunc else 0)
        out += struct.pack("<IIII", sec, usec, len(p), orig) + bytes(p)
    return bytes(out)


def test_ref22_golden(P):
    check_index(P, open(os.path.join(GOLD, "ref22.pcap"), "rb").read(), "ref22")


@pytest.mark.parametrize("n", [1, 19, 20000, 300000, 1 << 20])
def test_c4_replay(P, n):
    buf, offs, lens = gen.gen_c4(n, seed=100 + n)
    o, l, m = P.pcap_index(dev(buf))
    assert m == n
    assert np.array_equal(o.cpu().numpy(), offs) and np.array_equal(l.cpu().numpy(), lens)


def test_header_only_and_tails(P):
    check_index(P, gen.PCAP_GLOBAL_HEADER, "empty capture")
    base = records([b"\x01" * 60, b"\x02" * 70])
    for extra in range(0, 16):  # a trailing partial record header is ignored
        check_index(P, base + b"\x07" * extra, f"tail {extra}")


def test_errors_match_host(P):
    import pktgpu
    good = records([b"\x01" * 60, b"\x02" * 70, b"\x03" * 80])
    for bad in (good[:-3], b"\x00" * 40, b"\xd4\xc3\xb2", good[:24 + 16 + 60 + 16 + 5]):
        with pytest.raises(ValueError):
            pktgpu.pcap_index(bad)
        with pytest.raises(RuntimeError):
            P.pcap_index(dev(bad))


def test_cap_smaller_than_count(P):
    import torch
    buf, offs, lens = gen.gen_c4(5000, seed=7)
    o, l, n = P.pcap_index(dev(buf), cap=1234)
    assert n == 5000 and o.numel() == 1234
    assert np.array_equal(o.cpu().numpy(), offs[:1234]) and np.array_equal(l.cpu().numpy(), lens[:1234])
    o, l, n = P.pcap_index(dev(buf), cap=0)
    assert n == 5000 and o.numel() == 0


def test_fake_chains_in_payloads(P):
    """Every payload is itself a run of plausible record headers (a pcap inside the pcap), so a
    region that starts inside a payload guesses the fake chain; the fix-up must recover."""
    rng = np.random.default_rng(3)
    pays = []
    for i in range(3000):
        inner = bytearray()
        for _ in range(int(rng.integers(1, 6))):
            L = int(rng.integers(1, 40))
            inner += struct.pack("<IIII", 1, 2, L, L) + rng.integers(0, 256, L, dtype=np.uint8).tobytes()
        pays.append(bytes(inner))
    check_index(P, records(pays), "nested fake chains")


def test_zero_payloads_large_and_empty_records(P):
    rng = np.random.default_rng(4)
    pays = []
    for i in range(4000):
        r = rng.random()
        if r < 0.05:
            pays.append(b"")                               # incl_len 0 (never "plausible")
        elif r < 0.10:
            pays.append(bytes(int(rng.integers(4096, 65536))))  # spans several regions, all zeros
        elif r < 0.15:
            pays.append(rng.integers(0, 256, int(rng.integers(5000, 20000)), dtype=np.uint8).tobytes())
        else:
            pays.append(bytes(int(rng.integers(1, 300))))
    ts = [(int(rng.integers(0, 2**31)), int(rng.integers(0, 2**32))) for _ in pays]  # some usec >= 1e6
    check_index(P, records(pays, ts=ts, snap_trunc=[int(x) for x in rng.integers(0, 3, len(pays))]),
                "zero/large/empty")


def test_random_captures(P):
    rng = np.random.default_rng(5)
    for trial in range(6):
        n = int(rng.integers(1, 3000))
        hi = [20, 200, 1600, 9000, 70000, 16][trial]
        pays = [rng.integers(0, 256, int(rng.integers(0, hi)), dtype=np.uint8).tobytes() for _ in range(n)]
        check_index(P, records(pays), f"random {trial}")


def test_device_index_then_parse(P):
    """Capture in HBM -> device index -> indexed parse, every column == oracle, at C4's bench
    size (2^20 records, tests/pcap.rs:7-37 format)."""
    buf, offs, lens = gen.gen_c4(1 << 20, seed=21)
    d = dev(buf)
    o, l, n = P.pcap_index(d)
    g = P.parse(d, offsets=o, lens=l, columns="all")
    ref = oracle.parse_batch(buf, len(offs), offsets=offs, lens=lens, nthreads=8)
    for k, ov in ref.items():
        gv = g[k].cpu().numpy()
        if k in ("hdr_type", "hdr_off"):
            valid = np.arange(schema.MAX_HDRS)[:, None] < ref["n_hdrs"].astype(np.int64)[None, :]
            assert not (valid & (gv != ov)).any(), k
        else:
            assert np.array_equal(gv, ov), k


def test_one_ctx_growing_and_shrinking_captures():
    """one ctx indexes captures whose region count grows within the scratch
    buffer's slack and shrinks again, over many epochs.  The scan-block states must never sit on an
    earlier call's per-region words (file positions / prefixes that can look 'published' in the
    current epoch): the scratch layout is fixed by the allocated capacity, not by each call's K."""
    import pktgpu
    P2 = pktgpu.Parser(0)  # a fresh ctx: its scratch is first sized by the smallest capture
    try:
        caps = {}
        for n in (200, 5400, 6600, 200, 7000, 5800, 40, 8000):  # ~9 to ~360 4-KiB regions
            caps[n] = gen.gen_c4(n, seed=900 + n)
        order = [200, 5400, 6600, 200, 7000, 5800, 40, 8000] * 5
        for rep, n in enumerate(order):
            buf, offs, lens = caps[n]
            o, l, m = P2.pcap_index(dev(buf))
            assert m == n, (rep, n, m)
            assert np.array_equal(o.cpu().numpy(), offs), (rep, n)
            assert np.array_equal(l.cpu().numpy(), lens), (rep, n)
    finally:
        P2.close()


def test_parse_pcap_async_two_ctx(P):
    """pkt_parse_pcap_async / pkt_parse_pcap_result: captures queued alternately on two ctxs and two
    streams (one in flight per ctx), each result equal to the host indexer + oracle; an error
    capture parses nothing and its result raises."""
    import torch
    import pktgpu
    P2 = pktgpu.Parser(0)
    try:
        ps, ss = [P, P2], [torch.cuda.Stream(), torch.cuda.Stream()]
        caps = [gen.gen_c4(n, seed=90 + n) for n in (30000, 4097, 65536, 1, 20000)]
        bad = records([b"\x01" * 60, b"\x02" * 70, b"\x03" * 80])[:-3]
        jobs = [(c[0], len(c[1]), c) for c in caps] + [(np.frombuffer(bad, np.uint8), 8, None)]
        slots = [None, None]
        def finish(j):
            buf_d, res, o, l, c = slots[j]
            ss[j].synchronize()
            if c is None:
                with pytest.raises(RuntimeError):
                    ps[j].pcap_result()
                assert (res["status"].cpu().numpy() == 0xEE).all()
                return
            assert ps[j].pcap_result() == len(c[1])
            assert np.array_equal(o.cpu().numpy(), c[1]) and np.array_equal(l.cpu().numpy(), c[2])
            ref = oracle.parse_batch(c[0], len(c[1]), offsets=c[1], lens=c[2], columns=list(res), nthreads=8)
            for k, ov in ref.items():
                gv = res[k].cpu().numpy()
                if k in ("hdr_type", "hdr_off"):
                    valid = np.arange(schema.MAX_HDRS)[:, None] < ref["n_hdrs"].astype(np.int64)[None, :]
                    assert not (valid & (gv != ov)).any(), k
                else:
                    assert np.array_equal(gv, ov), k
        for k, (buf, cap, c) in enumerate(jobs):
            j = k % 2
            if slots[j] is not None:
                finish(j)
            cols = ["status"] if c is None else ["chain", "ipv4", "udp", "tcp"]
            res = ps[j].alloc(cap, cols)
            res["status"].fill_(0xEE)
            bd = dev(buf)
            o = torch.empty(cap, dtype=torch.uint64, device="cuda")
            l = torch.empty(cap, dtype=torch.uint32, device="cuda")
            ss[j].wait_stream(torch.cuda.current_stream())
            ps[j].parse_pcap_async(bd, cap, res, o, l, stream=ss[j])
            slots[j] = (bd, res, o, l, c)
        for j in (0, 1):
            finish(j)
        # the scratch belongs to a queued capture until its result is taken
        buf, offs, lens = caps[0]
        bd, m = dev(buf), len(offs)
        res = P.alloc(m, ["status"])
        o = torch.empty(m, dtype=torch.uint64, device="cuda")
        l = torch.empty(m, dtype=torch.uint32, device="cuda")
        P.parse_pcap_async(bd, m, res, o, l)
        with pytest.raises(RuntimeError):
            P.parse_pcap_async(bd, m, res, o, l)
        with pytest.raises(RuntimeError):
            P.parse_pcap(bd, m)
        assert P.pcap_result() == m
        with pytest.raises(RuntimeError):
            P.pcap_result()
    finally:
        P2.close()


def test_parse_pcap_fused_vs_oracle(P):
    """pkt_parse_pcap: device index + parse in one call, the parse taking the record count from the
    device (one host synchronisation).  Columns sized for cap > count: slot rows strided by cap and
    nothing written past the count; cap < count; the errors parse nothing."""
    import torch
    n = 50000
    buf, offs, lens = gen.gen_c4(n, seed=71)
    cap = n + 777
    res = P.alloc(cap, "all")
    for v in res.values():
        v.view(torch.uint8).fill_(0xEE)
    m, g, o, l = P.parse_pcap(dev(buf), cap, out=res)
    assert m == n
    assert np.array_equal(o[:n].cpu().numpy(), offs) and np.array_equal(l[:n].cpu().numpy(), lens)
    ref = oracle.parse_batch(buf, n, offsets=offs, lens=lens, nthreads=8)
    for k, ov in ref.items():
        gv = g[k].cpu().numpy()
        if k in ("hdr_type", "hdr_off"):
            valid = np.arange(schema.MAX_HDRS)[:, None] < ref["n_hdrs"].astype(np.int64)[None, :]
            assert not (valid & (gv[:, :n] != ov)).any(), k
        else:
            assert np.array_equal(gv[:n], ov), k
            assert (gv[n:].view(np.uint8) == 0xEE).all(), k  # past the count: untouched
    # the same call through an output descriptor built once (out_struct: what bench.py's pcap step
    # passes), into fresh columns: the same columns
    res2 = P.alloc(cap, "all")
    m2, g2, _, _ = P.parse_pcap(dev(buf), cap, out=P.out_struct(res2))
    assert m2 == n and isinstance(g2, P._lib.PktOut)
    for k in ("status", "n_hdrs", "payload_off", "hdr_mask", "ipv4_src", "udp_dst"):
        assert np.array_equal(res2[k][:n].cpu().numpy(), g[k][:n].cpu().numpy()), k
    m, g, o, l = P.parse_pcap(dev(buf), 1000, columns=["chain"])
    assert m == n and np.array_equal(o.cpu().numpy(), offs[:1000])
    ref = oracle.parse_batch(buf, 1000, offsets=offs[:1000], lens=lens[:1000], columns=list(g), nthreads=8)
    for k in ("status", "n_hdrs", "payload_off", "payload_len"):
        assert np.array_equal(g[k].cpu().numpy(), ref[k]), k
    good = records([b"\x01" * 60, b"\x02" * 70, b"\x03" * 80])
    for bad in (good[:-3], b"\x00" * 40):
        res = P.alloc(8, ["status"])
        res["status"].fill_(0xEE)
        with pytest.raises(RuntimeError):
            P.parse_pcap(dev(bad), 8, out=res)
        assert (res["status"].cpu().numpy() == 0xEE).all()  # an error parses nothing


def test_parse_pcap_span_staging_cap_past_count(P):
    """pkt_parse_pcap with wave-span staging (pkt_ctx_set_staging 2, parse_span_kernel) and
    cap > count — the span kernel takes the device-produced count: the records up to it equal the
    oracle, and no column (slot rows included) is written past it; whole waves past the count exit."""
    import torch
    n = 50000 + 37  # a partial last wave, then 12 whole waves past the count
    buf, offs, lens = gen.gen_c4(n, seed=73)
    cap = n + 777
    res = P.alloc(cap, "all")
    for v in res.values():
        v.view(torch.uint8).fill_(0xEE)
    P.set_staging(2)
    try:
        m, g, o, l = P.parse_pcap(dev(buf), cap, out=res)
    finally:
        P.set_staging(0)
    assert m == n
    ref = oracle.parse_batch(buf, n, offsets=offs, lens=lens, nthreads=8)
    for k, ov in ref.items():
        gv = g[k].cpu().numpy()
        if k in ("hdr_type", "hdr_off"):
            valid = np.arange(schema.MAX_HDRS)[:, None] < ref["n_hdrs"].astype(np.int64)[None, :]
            assert not (valid & (gv[:, :n] != ov)).any(), k
            assert (gv[:, n:].view(np.uint8) == 0xEE).all(), k
        else:
            assert np.array_equal(gv[:n], ov), k
            assert (gv[n:].view(np.uint8) == 0xEE).all(), k


def test_epoch_wrap_past_2_16_calls():
    """The scan blocks' published states carry a 16-bit call epoch (pktgpu_pcap.hip, BlkDesc) and the
    scratch is cleared once when it wraps: 2^16 + 3 blocking calls on one ctx over a capture of several
    scan blocks (with fake chains, so some regions are re-walked), the index checked against the host
    indexer on the calls around the wrap and at the end — a state left by an older call must never
    pass for the current one."""
    import ctypes
    import torch
    import pktgpu
    Q = pktgpu.Parser(0)  # a fresh ctx: its epoch starts at 0
    try:
        rng = np.random.default_rng(5)
        pays = []
        for i in range(9000):
            pays.append(bytes(rng.integers(0, 256, int(rng.integers(40, 300)), dtype=np.uint8)))
            if i % 97 == 0:  # a plausible-looking record header inside the payload (a fake chain)
                pays[-1] = struct.pack("<IIII", 0, 5, 20, 20) + pays[-1][16:]
        buf = records(pays)
        o_ref, l_ref = gen.pcap_index_py(buf)
        d = dev(buf)
        n = len(o_ref)
        o = torch.empty(n, dtype=torch.uint64, device="cuda")
        l = torch.empty(n, dtype=torch.uint32, device="cuda")
        cnt = ctypes.c_uint64()
        s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        L = Q._L
        checks = {1, (1 << 16) - 2, (1 << 16) - 1, 1 << 16, (1 << 16) + 1, (1 << 16) + 3}
        for call in range(1, (1 << 16) + 4):
            if call in checks:
                o.fill_(0)
                l.fill_(0)
            rc = L.pkt_pcap_index_device(Q._ctx, d.data_ptr(), d.numel(), o.data_ptr(), l.data_ptr(), n,
                                         ctypes.byref(cnt), s)
            assert rc == 0, call
            if call in checks:
                assert cnt.value == n, call
                assert np.array_equal(o.cpu().numpy(), o_ref) and np.array_equal(l.cpu().numpy(), l_ref), call
    finally:
        Q.close()


def test_scan64_composition_same_index():
    """files under 4 GiB take the 32-bit scan compositions; pkt_ctx_set_pcap_scan64 forces
    the 64-bit instantiation (the only one files >= 4 GiB run) so it stays pinned by the same captures:
    the golden capture, fake chains, zero / large / empty records, random captures, a C4 replay, the
    error cases, and a capture in HBM -> index -> parse == oracle."""
    import pktgpu
    import torch
    Q = pktgpu.Parser(0)
    try:
        Q.set_pcap_scan64(True)
        check_index(Q, open(os.path.join(GOLD, "ref22.pcap"), "rb").read(), "ref22 scan64")
        test_fake_chains_in_payloads(Q)
        test_zero_payloads_large_and_empty_records(Q)
        test_random_captures(Q)
        test_header_only_and_tails(Q)
        test_errors_match_host(Q)
        buf, offs, lens = gen.gen_c4(300_000, seed=64)
        o, l, m = Q.pcap_index(dev(buf))
        assert m == 300_000 and np.array_equal(o.cpu().numpy(), offs) and np.array_equal(l.cpu().numpy(), lens)
        g = Q.parse(dev(buf), offsets=o, lens=l, columns="all")
        torch.cuda.synchronize()
        ref = oracle.parse_batch(buf, len(offs), offsets=offs, lens=lens, nthreads=8)
        for k in ("status", "n_hdrs", "payload_off", "payload_len", "ipv4_csum_calc"):
            assert np.array_equal(g[k].cpu().numpy(), ref[k]), k
        Q.set_pcap_scan64(False)
        check_index(Q, open(os.path.join(GOLD, "ref22.pcap"), "rb").read(), "ref22 scan32 again")
    finally:
        Q.close()
    with pytest.raises(RuntimeError):
        P_ = pktgpu.Parser(0)
        try:
            P_._check(P_._L.pkt_ctx_set_pcap_scan64(P_._ctx, 2), "pkt_ctx_set_pcap_scan64")
        finally:
            P_.close()
