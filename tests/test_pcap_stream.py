"""The capture path fed as its bytes arrive (pkt_pcap_stream_*, and pkt_parse_pcap_host's pieces that
run on the same steps): every step indexes only the new bytes, from the device-side carry of the step
before (its first uncounted record start and record count), never re-walking from offset 24.

The records, counts and errors must equal the host indexer's over the whole capture (gen.pcap_index_py,
pinned by tests/golden/ref22.pcap; format tests/pcap.rs:7-37) and every column the oracle's
(reference src/parser/fast.rs:5-227), whatever the push sizes: pushes of one byte, pushes that split
record headers and the global header, records longer than many steps, captures built to defeat the
indexer's guess (fake record chains inside payloads, zero payloads), polls between pushes that see
exactly the records wholly inside the bytes so far."""
import os
import struct

import numpy as np
import pytest

import oracle
from pktgpu import gen, schema

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
SLOT = ("hdr_type", "hdr_off")


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.fail("no GPU visible: -m gpu tests need an MI355X")


def _check(g, ref, n, label):
    for k, ov in ref.items():
        gv = g[k].cpu().numpy() if hasattr(g[k], "cpu") else np.asarray(g[k])
        gv = gv[:, :n] if k in SLOT else gv[:n]
        if k in SLOT:
            valid = np.arange(schema.MAX_HDRS)[:, None] < ref["n_hdrs"].astype(np.int64)[None, :]
            assert not (valid & (gv != ov)).any(), f"{label} {k}"
        else:
            assert np.array_equal(gv, ov), f"{label} {k}"


def _records(payloads, ts=None):
    out = bytearray(gen.PCAP_GLOBAL_HEADER)
    for i, p in enumerate(payloads):
        sec, usec = ts[i] if ts else (i, 0)
        out += struct.pack("<IIII", sec, usec, len(p), len(p)) + bytes(p)
    return bytes(out)


def _whole_before(offs, lens, L):
    """Records wholly inside the first L bytes (the stream's count after L bytes)."""
    return int(np.searchsorted(offs.astype(np.int64) + lens.astype(np.int64), L, side="right"))


def _run(buf, sizes, step_bytes, pinned=False, polls=True, scan64=False, cap=None):
    from pktgpu.stream import PcapStream
    offs, lens = gen.pcap_index_py(bytes(buf))
    n = len(offs)
    cap = cap or max(n, 1)
    st = PcapStream(0, max_bytes=len(buf) + 64, cap=cap, columns="all", out="pinned" if pinned else None,
                    step_bytes=step_bytes)
    try:
        if scan64:
            assert st._L.pkt_ctx_set_pcap_scan64(st.ctx(), 1) == 0
        a = np.frombuffer(bytes(buf), np.uint8)
        pos, k = 0, 0
        while pos < a.size:
            m = int(sizes[k % len(sizes)])
            st.push(a[pos:pos + m])
            pos = min(a.size, pos + m)
            k += 1
            if polls and k % 7 == 3:
                c, idx = st.poll(index=True)
                want = _whole_before(offs, lens, pos)
                assert c == want, (pos, c, want)
                assert np.array_equal(idx[0], offs[:min(c, cap)]) and np.array_equal(idx[1], lens[:min(c, cap)])
        c, (o2, l2) = st.finish()
        assert c == n
        assert np.array_equal(o2, offs[:cap]) and np.array_equal(l2, lens[:cap])
        m = min(n, cap)
        if m:
            ref = oracle.parse_batch(np.frombuffer(bytes(buf), np.uint8), m, offsets=offs[:m], lens=lens[:m], nthreads=8)
            _check(st.out, ref, m, f"stream step={step_bytes} pinned={pinned}")
    finally:
        st.close()


def test_golden_capture_byte_by_byte():
    """ref22.pcap (the reference's 22 packets, tests/lib.rs:220-680) pushed one byte at a time with a
    step per byte: the global header arrives in 24 pushes, every record header in 16."""
    pc = open(os.path.join(GOLD, "ref22.pcap"), "rb").read()
    _run(pc, [1], 1)


@pytest.mark.parametrize("step", [1, 4096, 65536, 0])
@pytest.mark.parametrize("pinned", [False, True])
def test_c4_random_push_sizes(step, pinned):
    """A 20 000-record C4 replay pushed in random sizes (1 B .. 200 KB), a step every `step` new bytes
    (0 = the 4 MiB default: one step at the end), polled every few pushes; device and pinned columns."""
    buf, _, _ = gen.gen_c4(20_000, seed=500 + step)
    rng = np.random.default_rng(step + 7)
    sizes = rng.integers(1, 200_000, 64)
    sizes[::5] = rng.integers(1, 40, len(sizes[::5]))
    _run(buf, sizes, step, pinned=pinned)


def test_staged_and_direct_pushes_interleaved():
    """Pushes under 1 MiB go through the stream's pinned staging ring, larger ones are copied directly
    (include/pktgpu.h): a C4 capture pushed as small / 1 MiB / 2-3 MiB / tiny pieces in turn, with
    steps of 256 KiB and polls between, must keep the bytes in order (staged bytes flushed before a
    direct copy) and give the host indexer's records and the oracle's columns."""
    buf, _, _ = gen.gen_c4(40_000, seed=808)
    sizes = [70_000, 1 << 20, 5, (2 << 20) + 333, 123_457, 1, (1 << 20) - 1, (3 << 20) + 7, 64, 999_999]
    _run(buf, sizes, 256 << 10)
    _run(buf, sizes[::-1], 0, pinned=True)


def test_long_records_and_fake_chains():
    """Records up to 70 KB (many steps of 4 KiB pass inside one record), payloads that are themselves
    chains of plausible record headers, zero-filled payloads; pushed in 3000-byte pieces with a step per
    push, so most steps' first region lies inside a record that started several steps before."""
    rng = np.random.default_rng(9)
    pays = []
    for i in range(1500):
        r = rng.random()
        if r < 0.1:
            pays.append(bytes(int(rng.integers(4096, 70000))))
        elif r < 0.3:
            inner = bytearray()
            for _ in range(int(rng.integers(1, 6))):
                L = int(rng.integers(1, 40))
                inner += struct.pack("<IIII", 1, 2, L, L) + rng.integers(0, 256, L, dtype=np.uint8).tobytes()
            pays.append(bytes(inner))
        else:
            pays.append(rng.integers(0, 256, int(rng.integers(1, 400)), dtype=np.uint8).tobytes())
    _run(_records(pays), [3000], 1)
    _run(_records(pays), [4096 * 3 + 5, 17, 9000], 4096, scan64=True)


def test_cap_below_count_and_tails():
    """cap < records: the index and columns of the first cap records, the count of all; a trailing
    partial record header (< 16 B) is ignored at finish."""
    buf, _, _ = gen.gen_c4(3000, seed=77)
    _run(bytes(buf) + b"\x07" * 11, [777], 1000, cap=1234)


def test_errors():
    """A record running past the end of the capture is an error at finish (not at a poll before it);
    a bad magic is an error; a push past max_bytes is refused; after an error every call raises."""
    from pktgpu.stream import PcapStream
    buf, offs, lens = gen.gen_c4(2000, seed=78)
    st = PcapStream(0, max_bytes=buf.size, cap=2000, columns=["chain"])
    try:
        st.push(buf[:-3])
        c, _ = st.poll()
        assert c == 1999
        with pytest.raises(RuntimeError):
            st.finish()
    finally:
        st.close()
    bad = bytearray(buf[:5000].tobytes())
    bad[0] ^= 0xFF
    st = PcapStream(0, max_bytes=len(bad), cap=2000, columns=["chain"], step_bytes=1024)
    try:
        st.push(bytes(bad))
        with pytest.raises(RuntimeError):
            st.finish()
    finally:
        st.close()
    st = PcapStream(0, max_bytes=100, cap=10, columns=["chain"])
    try:
        st.push(buf[:60])
        with pytest.raises(RuntimeError):
            st.push(buf[60:200])
    finally:
        st.close()


@pytest.mark.parametrize("piece", [4096, 5000, 1 << 16, 3 << 20])
def test_host_pieces_every_size(piece):
    """pkt_parse_pcap_host runs on the same steps (one per piece): at 2^16 C4 records and piece sizes
    from one region to several MiB, the index, the count and every column == host indexer + oracle."""
    import pktgpu
    P = pktgpu.Parser(0)
    try:
        n = 1 << 16
        buf, offs, lens = gen.gen_c4(n, seed=35)
        hb = P.host_empty((buf.size,), np.uint8)
        hb[:] = buf
        out = {c: P.host_empty(schema.column_shape(c, n), schema.column_dtype(c)) for c in schema.COLUMN_NAMES}
        P.set_host_piece(piece)
        m, g, (o2, l2) = P.parse_pcap_host(hb, n, out=out)
        assert m == n and np.array_equal(o2, offs) and np.array_equal(l2, lens)
        _check(g, oracle.parse_batch(buf, n, offsets=offs, lens=lens, nthreads=8), n, f"host pieces {piece}")
    finally:
        P.close()
