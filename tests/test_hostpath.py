"""Host-memory path (pkt_parse_host): host batch in, host columns out, chunk-pipelined through
the device — every column bit-exact against the oracle, including ragged last chunks, tails
shorter than one 16-byte chunk, indexed (pcap) batches and pinned buffers."""
import os

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


def check(g, o, label):
    for k, ov in o.items():
        gv = g[k]
        if k in ("hdr_type", "hdr_off"):
            valid = np.arange(schema.MAX_HDRS)[:, None] < o["n_hdrs"].astype(np.int64)[None, :]
            assert not (valid & (gv != ov)).any(), (label, k)
        else:
            assert np.array_equal(gv, ov), (label, k, np.nonzero(gv != ov)[0][:8])


@pytest.mark.parametrize("chunk", [0, 10000, 4096 * 3 + 5])
def test_c2_fixed_stride(P, chunk):
    n = 65537
    slab = gen.gen_c2(n, seed=3)
    g = P.parse_host(slab, stride=64, columns="all", chunk=chunk)
    check(g, oracle.parse_batch(slab, n, stride=64, nthreads=8), f"c2 chunk={chunk}")


def test_c3_stride_with_lens_and_odd_stride(P):
    rng = np.random.default_rng(5)
    n = 30001
    slab = gen.gen_c3(n, seed=5)
    lens = rng.integers(0, 129, n).astype(np.uint32)
    g = P.parse_host(slab, stride=128, lens=lens, chunk=7000)
    check(g, oracle.parse_batch(slab, n, stride=128, lens=lens, nthreads=8), "c3 lens")
    a = np.zeros((n, 72), np.uint8)
    a[:, :64] = gen.gen_c2(n, seed=6)
    g = P.parse_host(a, stride=72, chunk=9999)
    check(g, oracle.parse_batch(a, n, stride=72, nthreads=8), "stride 72")


def test_pcap_indexed(P):
    buf, offs, lens = gen.gen_c4(50000, seed=8)
    g = P.parse_host(buf, offsets=offs, lens=lens, chunk=7777)
    check(g, oracle.parse_batch(buf, len(offs), offsets=offs, lens=lens, nthreads=8), "c4")
    pc = open(os.path.join(GOLD, "ref22.pcap"), "rb").read()
    o2, l2 = gen.pcap_index_py(pc)
    arr = np.frombuffer(pc, np.uint8)
    for entry in ("parse", "parse_ethernet", "parse_ipv4"):
        g = P.parse_host(arr, offsets=o2, lens=l2, entry=entry, chunk=5)
        check(g, oracle.parse_batch(arr, 22, offsets=o2, lens=l2, entry=entry), f"ref22 {entry}")


def test_tiny_tails(P):
    """A last chunk holding fewer than 16 bytes (and one holding none) still parses exactly."""
    c2 = gen.gen_c2(3, seed=9).reshape(-1)
    for total in (64 + 6, 64 * 2 + 13, 64 * 2, 64 * 2 + 1, 20, 14, 1):
        slab = c2[:total].copy()
        n = (total + 63) // 64 + 1  # one packet past the end
        g = P.parse_host(slab, stride=64, n=n, chunk=1)
        check(g, oracle.parse_batch(slab, n, stride=64), f"tail {total}")


def test_pinned_buffers(P):
    import pktgpu
    n = 1 << 17
    src = gen.gen_c2(n, seed=10).reshape(-1)
    slab = P.host_empty(src.shape, np.uint8)
    slab[:] = src
    cols = pktgpu.resolve_columns(["chain", "ether", "ipv4", "udp"])
    out = {c: P.host_empty(schema.column_shape(c, n), schema.column_dtype(c)) for c in cols}
    for c in out:
        out[c][...] = 0
    g = P.parse_host(slab, stride=64, columns=cols, out=out, chunk=1 << 15)
    check(g, oracle.parse_batch(src, n, stride=64, columns=cols, nthreads=8), "pinned")


def test_pinned_indexed_zero_copy(P):
    """Pinned slab, offsets, lens and columns: the zero-copy route (one launch over the link); a
    pageable slab with pinned columns: the export pipeline (chunks copied in, parsed on the device,
    columns exported by 16-byte chunks; odd chunk sizes) — the same results."""
    buf, offs, lens = gen.gen_c4(40000, seed=11)
    h = P.host_empty(buf.shape, np.uint8)
    h[:] = buf
    ho = P.host_empty(offs.shape, np.uint64)
    ho[:] = offs
    hl = P.host_empty(lens.shape, np.uint32)
    hl[:] = lens
    out = {c: P.host_empty(schema.column_shape(c, len(offs)), schema.column_dtype(c)) for c in schema.COLUMN_NAMES}
    ref = oracle.parse_batch(buf, len(offs), offsets=offs, lens=lens, nthreads=8)
    g = P.parse_host(h, offsets=ho, lens=hl, out=out)
    check(g, ref, "pinned c4 zero copy")
    for chunk in (0, 4097):
        for c in out:
            out[c][...] = 0
        g = P.parse_host(buf, offsets=offs, lens=lens, out=out, chunk=chunk)
        check(g, ref, f"pageable slab, pinned columns: export chunk={chunk}")
    # mixed: pinned slab, pageable columns -> the staged pipeline, same results
    g = P.parse_host(h, offsets=ho, lens=hl, columns="all", chunk=9999)
    check(g, oracle.parse_batch(buf, len(offs), offsets=offs, lens=lens, nthreads=8), "pinned slab only")


@pytest.mark.parametrize("staging", [1, 2])
def test_pinned_async_parse_batch(P, staging):
    """pkt_parse_batch on pinned host buffers (no pkt_parse_host): the kernel reads the slab and
    writes the columns over the link, asynchronously on the caller's stream."""
    import torch
    buf, offs, lens = gen.gen_c4(30000, seed=12)
    n = len(offs)
    h, ho, hl = (P.host_empty(a.shape, a.dtype) for a in (buf, offs, lens))
    h[:], ho[:], hl[:] = buf, offs, lens
    out = {c: P.host_empty(schema.column_shape(c, n), schema.column_dtype(c)) for c in schema.COLUMN_NAMES}
    for c in out:
        out[c][...] = 0
    b = P._lib.PktBatch()
    b.slab, b.slab_len = h.ctypes.data, h.size
    b.offsets, b.lens, b.n = ho.ctypes.data, hl.ctypes.data, n
    o = P._lib.PktOut()
    for c, a in out.items():
        setattr(o, c, a.ctypes.data if a.size else None)
    s = torch.cuda.Stream()
    P.set_staging(staging)
    try:
        P.launch(b, 0, o, stream=s)
        s.synchronize()
    finally:
        P.set_staging(0)
    check(out, oracle.parse_batch(buf, n, offsets=offs, lens=lens, nthreads=8), f"async staging={staging}")


@pytest.mark.parametrize("pinned", [True, False])
def test_pcap_host_end_to_end(P, pinned):
    """pkt_parse_pcap_host — a capture in host memory (tests/pcap.rs:7-37 format) ->
    device copy -> device index -> all-column parse -> host columns, one blocking call — equals the
    host indexer + the oracle at 2^16 records; pinned columns take the kernel's direct writes over
    the link, pageable ones the staged pipeline.  Slot columns are strided by cap."""
    n = 1 << 16
    buf, offs, lens = gen.gen_c4(n, seed=31)
    cap = n + 123  # room to spare: the slot rows are strided by cap, not by the count
    if pinned:
        hb = P.host_empty((buf.size,), np.uint8)
        hb[:] = buf
        out = {c: P.host_empty(schema.column_shape(c, cap), schema.column_dtype(c)) for c in schema.COLUMN_NAMES}
    else:
        hb, out = buf, None
    m, g, (o2, l2) = P.parse_pcap_host(hb, cap, out=out)
    assert m == n
    assert np.array_equal(o2, offs) and np.array_equal(l2, lens)
    ref = oracle.parse_batch(buf, n, offsets=offs, lens=lens, nthreads=8)
    got = {k: (v[:, :n] if k in ("hdr_type", "hdr_off") else v[:n]) for k, v in g.items()}
    check(got, ref, f"pcap host pinned={pinned}")


def test_pcap_host_cap_and_errors(P):
    buf, offs, lens = gen.gen_c4(5000, seed=32)
    m, g, (o2, l2) = P.parse_pcap_host(buf, 1234, columns=["chain", "ipv4"])
    assert m == 5000 and np.array_equal(o2, offs[:1234]) and np.array_equal(l2, lens[:1234])
    ref = oracle.parse_batch(buf, 1234, offsets=offs[:1234], lens=lens[:1234], columns=list(g), nthreads=8)
    check(g, ref, "cap < count")
    pc = open(os.path.join(GOLD, "ref22.pcap"), "rb").read()
    for bad in (pc[:-3], b"\x00" * 40):
        with pytest.raises(RuntimeError):
            P.parse_pcap_host(bad, 64)
    m, g, _ = P.parse_pcap_host(pc, 22, columns=["chain"])
    assert m == 22 and int(g["status"].max()) == 0


def test_pcap_host_async_two_ctx(P):
    """pkt_parse_pcap_host_async / _result: captures in pinned host memory queued alternately on two
    ctxs (one in flight per ctx, one capture's copy in overlapping the other's columns out), every
    result equal to the oracle; an error capture parses nothing and its result raises; pageable
    columns are refused."""
    import pktgpu
    P2 = pktgpu.Parser(0)
    try:
        ps = [P, P2]
        caps = [gen.gen_c4(n, seed=60 + n) for n in (20000, 1, 65536, 4097)]
        pc = open(os.path.join(GOLD, "ref22.pcap"), "rb").read()
        jobs = [(c[0], len(c[1]), c) for c in caps] + [(np.frombuffer(pc[:-3], np.uint8), 64, None)]
        slots = [None, None]

        def finish(j):
            res, hb, c = slots[j]
            if c is None:
                with pytest.raises(RuntimeError):
                    ps[j].pcap_host_result()
                assert (res["status"] == 0xEE).all()  # an error parses nothing
                return
            n = len(c[1])
            assert ps[j].pcap_host_result() == n
            ref = oracle.parse_batch(c[0], n, offsets=c[1], lens=c[2], columns=list(res), nthreads=8)
            check(res, ref, f"async host capture n={n}")

        for k, (buf, cap, c) in enumerate(jobs):
            j = k % 2
            if slots[j] is not None:
                finish(j)
            hb = ps[j].host_empty((buf.size,), np.uint8)
            hb[:] = buf
            cols = ["status"] if c is None else list(schema.COLUMN_NAMES)
            res = {col: ps[j].host_empty(schema.column_shape(col, cap), schema.column_dtype(col)) for col in cols}
            res["status"][:] = 0xEE
            ps[j].parse_pcap_host_async(hb, cap, res)
            slots[j] = (res, hb, c)
        for j in (0, 1):
            finish(j)
        buf, offs, lens = caps[0]
        with pytest.raises(RuntimeError):  # pageable columns: refused
            P.parse_pcap_host_async(P.host_empty((buf.size,), np.uint8), len(offs),
                                    {"status": np.zeros(len(offs), np.uint8)})
    finally:
        P2.close()


def test_pcap_host_small_pieces_records_longer_than_a_piece(P):
    """pkt_parse_pcap_host at the smallest piece (4096 B) over records of up to 9 KB: pieces that add
    no record (their prefix's count does not move: an empty parse range and an empty export), records
    and record headers split across several pieces, a file length that is no multiple of the piece;
    every column, the index and the count equal the host indexer + the oracle."""
    import struct
    rng = np.random.default_rng(41)
    tm = [pk.to_vec() for pk in gen.reference_22_packets()]
    out_b = bytearray(gen.PCAP_GLOBAL_HEADER)
    for i in range(1500):
        body = tm[i % len(tm)] + bytes(int(rng.integers(0, 9000 if i % 5 == 0 else 300)))
        out_b += struct.pack("<IIII", i, 0, len(body), len(body)) + body
    buf = np.frombuffer(bytes(out_b), np.uint8)
    offs, lens = gen.pcap_index_py(bytes(out_b))
    n = len(offs)
    hb = P.host_empty((buf.size,), np.uint8)
    hb[:] = buf
    out = {c: P.host_empty(schema.column_shape(c, n), schema.column_dtype(c)) for c in schema.COLUMN_NAMES}
    P.set_host_piece(4096)
    try:
        assert buf.size % 4096 != 0 and int(lens.max()) > 2 * 4096
        m, g, (o2, l2) = P.parse_pcap_host(hb, n, out=out)
        assert m == n
        assert np.array_equal(o2, offs) and np.array_equal(l2, lens)
        ref = oracle.parse_batch(buf, n, offsets=offs, lens=lens, nthreads=8)
        check(g, ref, "pcap host pieces of 4096 B, long records")
    finally:
        P.set_host_piece(0)


@pytest.mark.parametrize("piece", [65537, 1 << 20])
def test_pcap_host_pieces_vs_oracle(P, piece):
    """pkt_parse_pcap_host copies a capture in pieces and parses each prefix's new
    records while the next pieces copy in.  At 2^16 records with pieces of 65537 bytes (odd: the piece
    boundaries fall inside records and inside record headers) and of 1 MiB, every column, the index
    and the count equal the host indexer + the oracle; a capture whose last record runs past the end is
    still an error (the last prefix is the whole file, indexed with pkt_pcap_index's errors)."""
    n = 1 << 16
    buf, offs, lens = gen.gen_c4(n, seed=34)
    cap = n + 77
    hb = P.host_empty((buf.size,), np.uint8)
    hb[:] = buf
    out = {c: P.host_empty(schema.column_shape(c, cap), schema.column_dtype(c)) for c in schema.COLUMN_NAMES}
    P.set_host_piece(piece)
    try:
        assert buf.size > 2 * piece
        m, g, (o2, l2) = P.parse_pcap_host(hb, cap, out=out)
        assert m == n
        assert np.array_equal(o2, offs) and np.array_equal(l2, lens)
        ref = oracle.parse_batch(buf, n, offsets=offs, lens=lens, nthreads=8)
        got = {k: (v[:, :n] if k in ("hdr_type", "hdr_off") else v[:n]) for k, v in g.items()}
        check(got, ref, f"pcap host pieces of {piece} B")
        bad = P.host_empty((buf.size - 3,), np.uint8)
        bad[:] = buf[:-3]  # the last record runs past the end of the file
        with pytest.raises(RuntimeError):
            P.parse_pcap_host(bad, cap, out=out)
    finally:
        P.set_host_piece(0)
