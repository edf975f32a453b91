"""GPU parity tests: the HIP path (through the C ABI) against the oracle, bit for bit.

Every test calls libpktgpu's kernels on a real MI355X and compares with oracle/pkt_oracle.c
on the same seeded input.  Slot columns (hdr_type/hdr_off) are compared for the slots the
packet owns (j < n_hdrs); everything else is compared whole.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

import oracle  # noqa: E402
import pyref  # noqa: E402
from pktgpu import gen, schema  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(REPO, "tests", "golden")
H = schema.HDR_ID


@pytest.fixture(scope="module")
def P():
    if not torch.cuda.is_available():
        pytest.fail("no GPU visible: -m gpu tests need an MI355X")
    import pktgpu
    return pktgpu.Parser(0)


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def to_host(res):
    torch.cuda.synchronize()
    return {k: v.cpu().numpy() for k, v in res.items()}


def gpu_parse(P, slab, n, stride=None, offsets=None, lens=None, entry="parse", columns="all",
              window=0):
    ds = dev(np.ascontiguousarray(slab, np.uint8).reshape(-1))
    do = dev(offsets.astype(np.uint64)) if offsets is not None else None
    dl = dev(lens.astype(np.uint32)) if lens is not None else None
    P.set_window(window)
    try:
        res = P.parse(ds, stride=stride, n=n, offsets=do, lens=dl, entry=entry, columns=columns)
        return to_host(res)
    finally:
        P.set_window(0)


def compare(g, o, label=""):
    n = len(o["status"]) if "status" in o else None
    for k, ov in o.items():
        gv = g[k]
        if k in ("hdr_type", "hdr_off"):
            nh = o["n_hdrs"].astype(np.int64)
            valid = np.arange(schema.MAX_HDRS)[:, None] < nh[None, :]
            bad = np.nonzero(valid & (gv != ov))
            assert bad[0].size == 0, f"{label} {k}: first mismatch slot={bad[0][:5]} pkt={bad[1][:5]}"
        else:
            if not np.array_equal(gv, ov):
                idx = np.nonzero((gv != ov).reshape(len(ov), -1).any(axis=1))[0]
                raise AssertionError(f"{label} {k}: {idx.size} mismatches, first pkts {idx[:8]}: "
                                     f"gpu={gv[idx[:4]]} oracle={ov[idx[:4]]}")
    return n


def both(P, slab, n, stride=None, offsets=None, lens=None, entry="parse", columns="all", window=0,
         label=""):
    import pktgpu
    cols = pktgpu.resolve_columns(columns)
    g = gpu_parse(P, slab, n, stride, offsets, lens, entry, cols, window)
    o = oracle.parse_batch(slab, n, stride=stride, offsets=offsets, lens=lens, entry=entry,
                           columns=cols, nthreads=8)
    compare(g, o, label)
    return g, o


# ------------------------------------------------------------------ golden 22 packets
def test_ref22_pcap_all_columns(P):
    pc = open(os.path.join(GOLD, "ref22.pcap"), "rb").read()
    offs, lens = gen.pcap_index_py(pc)
    slab = np.frombuffer(pc, np.uint8)
    g, _ = both(P, slab, 22, offsets=offs, lens=lens, label="ref22")
    import json
    exp = json.load(open(os.path.join(GOLD, "ref22_expected.json")))
    for i, e in enumerate(exp):
        got = [[schema.HDR_NAMES[g["hdr_type"][j, i]], int(g["hdr_off"][j, i])]
               for j in range(g["n_hdrs"][i])]
        assert got == e["hdrs"], e["name"]
        assert (g["payload_off"][i], g["payload_len"][i]) == (e["payload_off"], e["payload_len"])


@pytest.mark.parametrize("window", [0, 16, 32, 64, 256])
def test_ref22_windows(P, window):
    """Small windows force the global-memory fallback of the walk and the field reads."""
    pc = open(os.path.join(GOLD, "ref22.pcap"), "rb").read()
    offs, lens = gen.pcap_index_py(pc)
    both(P, np.frombuffer(pc, np.uint8), 22, offsets=offs, lens=lens, window=window,
         label=f"w{window}")


def test_packet_slice_view_payload(P):
    """tests/lib.rs:818-827 through the GPU: fast::parse(..).payload() == [0..9]."""
    import pktgpu
    pl = bytes(range(10))
    v = gen.test_tcp_packet_with_payload(pl).to_vec()
    slab = np.frombuffer(v, np.uint8)
    g = gpu_parse(P, slab, 1, stride=len(v))
    sl = pktgpu.packet_slice(g, 0, v)
    assert sl.payload() == pl
    assert sl.to_vec() == v and sl.len() == len(v)
    assert [h.name() for h in sl.hdrs] == ["Ether", "IPv4", "TCP"]
    assert sl["IPv4"].ttl() == 64 and sl["TCP"].dst() == 8888 and sl["Ether"].etype() == 0x800


# ------------------------------------------------------------------ benchmark configs
@pytest.mark.parametrize("n", [1, 63, 64, 65, 255, 257, 4097, 1 << 16])
def test_c2_sizes(P, n):
    slab = gen.gen_c2(n, seed=n)
    both(P, slab, n, stride=64, label=f"c2 n={n}")


def test_c2_full_1m(P):
    """Config 2 at its full size (2^20 x 64 B), every column, against the oracle."""
    n = 1 << 20
    slab = gen.gen_c2(n)
    g, o = both(P, slab, n, stride=64, label="c2 1M")
    assert (g["status"] == 0).all() and (g["n_hdrs"] == 3).all()
    good = g["ipv4_header_checksum"] == g["ipv4_csum_calc"]
    assert 0.98 < good.mean() < 1.0  # 1 % corrupted checksums in the generator


def test_c3_full_1m(P):
    n = 1 << 20
    slab = gen.gen_c3(n)
    g, _ = both(P, slab, n, stride=128, label="c3 1M")
    assert set(np.unique(g["n_hdrs"])) == {3, 4, 5}


@pytest.mark.parametrize("staging", [0, 2])
def test_c4_pcap(P, staging):
    """Config 4 at its bench size: 2^20 pcap records of the 22 templates, every column."""
    n = 1 << 20
    buf, offs, lens = gen.gen_c4(n, seed=4)
    P.set_staging(staging)
    try:
        both(P, buf, n, offsets=offs, lens=lens, label=f"c4 staging={staging}")
    finally:
        P.set_staging(0)


def test_c2_chain_only_and_subsets(P):
    n = 5000
    slab = gen.gen_c2(n, seed=9)
    for cols in (["chain"], ["status", "payload_len"], ["ipv4_csum_calc"], ["ether", "udp"]):
        both(P, slab, n, stride=64, columns=cols, label=str(cols))


def test_c4_chain_only_and_subsets(P):
    """Indexed batches with column subsets (chain-only, status-only, chain + one header group,
    status + one field group: the runtime-checked kernel and the chain kernel) vs the oracle, and
    the ref22 capture (every template, every alignment phase) with the chain columns."""
    n = 1 << 18
    buf, offs, lens = gen.gen_c4(n, seed=44)
    for cols in (["chain"], ["status", "payload_len"], ["chain", "ipv6"], ["status", "udp"]):
        both(P, buf, n, offsets=offs, lens=lens, columns=cols, label=f"c4 {cols}")
    pc = open(os.path.join(GOLD, "ref22.pcap"), "rb").read()
    o22, l22 = gen.pcap_index_py(pc)
    both(P, np.frombuffer(pc, np.uint8), 22, offsets=o22, lens=l22, columns=["chain"], label="ref22 chain")


# ------------------------------------------------------------------ entries and edge cases
@pytest.mark.parametrize("entry", schema.ENTRIES)
def test_entries_random_and_templates(P, entry):
    rng = np.random.default_rng(100 + schema.ENTRY_ID[entry])
    pkts = [p.to_vec() for p in gen.reference_22_packets()]
    pkts += [rng.integers(0, 256, int(rng.integers(0, 200)), dtype=np.uint8).tobytes()
             for _ in range(3000)]
    buf = b"".join(pkts)
    lens = np.array([len(p) for p in pkts], np.uint32)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    slab = np.frombuffer(buf + bytes(16), np.uint8)
    both(P, slab, len(pkts), offsets=offs, lens=lens, entry=entry, label=entry)


def test_truncated_prefixes(P):
    """Every prefix (0..len) of every template, in one fixed-stride batch with lens."""
    pkts = [p.to_vec() for p in gen.reference_22_packets()]
    stride = 288
    rows, lens = [], []
    for v in pkts:
        for L in range(0, len(v) + 1):
            r = np.zeros(stride, np.uint8)
            r[:len(v)] = np.frombuffer(v, np.uint8)  # bytes past len present but not packet
            rows.append(r)
            lens.append(L)
    slab = np.stack(rows)
    lens = np.array(lens, np.uint32)
    g, o = both(P, slab, len(lens), stride=stride, lens=lens, label="prefixes")
    assert (g["status"] == schema.TRUNCATED).sum() > 1000


def test_empty_batch(P):
    import pktgpu
    ds = dev(np.zeros(64, np.uint8))
    res = P.parse(ds, stride=64, n=0)
    torch.cuda.synchronize()
    assert res["status"].numel() == 0
    del pktgpu


def _stack_packets():
    """VLAN stacks of 0-19 tags (whole and truncated) and MPLS stacks of 1-18 labels, at a 256-B
    stride with lengths: chains past the depth limit and far past 8 headers."""
    eth = gen.ethernet("00:00:00:00:00:01", "00:00:00:00:00:02", 0x8100).data
    tag = gen.vlan(1, 0, 7, 0x8100).data
    last = gen.vlan(0, 0, 5, 0x0800).data
    ip = gen.ipv4(5, 0, 1, 64, 0, 17, "1.1.1.1", "2.2.2.2", 28).data
    udp = gen.udp(1, 2, 8).data
    pkts = []
    for k in range(0, 20):
        pkts.append(eth + tag * k + last + ip + udp)
        pkts.append(eth + tag * k + last + ip[:-1])
    # MPLS stacks
    e8847 = gen.ethernet("00:00:00:00:00:01", "00:00:00:00:00:02", 0x8847).data
    for k in range(0, 18):
        pkts.append(e8847 + gen.mpls_raw(5, 0, 0, 9).data * k + gen.mpls_raw(6, 0, 1, 9).data +
                    bytes([0x45, 1, 2, 3]) + ip + udp)
    stride = 256
    slab = np.zeros((len(pkts), stride), np.uint8)
    lens = np.zeros(len(pkts), np.uint32)
    for i, p in enumerate(pkts):
        slab[i, :len(p)] = np.frombuffer(p, np.uint8)
        lens[i] = len(p)
    return slab, lens, stride


def test_depth_limit_and_stacks(P):
    slab, lens, stride = _stack_packets()
    g, o = both(P, slab, len(lens), stride=stride, lens=lens, label="stacks")
    assert (g["status"] == schema.DEPTH_LIMIT).sum() > 5 and (g["status"] == 0).sum() > 5


def test_gre_option_combinations(P):
    inner = gen.create_udp_packet("00:01:02:03:04:05", "00:06:07:08:09:0a", False, 0, 0, 5,
                                  "1.1.1.1", "2.2.2.2", 0, 64, 0, 0, [], 53, 1000, False, b"x" * 8)
    inner.remove(0)
    pkts = []
    for c in (0, 1):
        for k in (0, 1):
            for s in (0, 1):
                p = gen.create_gre_packet("00:01:02:03:04:05", "00:06:07:08:09:0a", False, 0, 0, 5,
                                          "3.3.3.3", "4.4.4.4", 0, 64, 0, 0, [], c, 0, k, s, 0, 0, 0,
                                          0x1111, 0x2222, 0x33333333, 0x44444444, b"", inner).to_vec()
                for L in (len(p), 38, 42, 46, 50):
                    pkts.append(p[:L])
    buf = b"".join(pkts)
    lens = np.array([len(p) for p in pkts], np.uint32)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    both(P, np.frombuffer(buf + bytes(16), np.uint8), len(pkts), offsets=offs, lens=lens, label="gre")


def test_fuzz_mutated_templates(P):
    rng = np.random.default_rng(2024)
    pkts = [p.to_vec() for p in gen.reference_22_packets()]
    keys = [12, 13, 23, 20, 36, 37, 38, 34, 35, 16, 45, 46, 53, 57, 60, 61]
    out = []
    for _ in range(40000):
        v = bytearray(pkts[int(rng.integers(0, len(pkts)))])
        for _ in range(int(rng.integers(1, 5))):
            k = int(rng.choice(keys)) if rng.random() < 0.6 else int(rng.integers(0, len(v)))
            if k < len(v):
                v[k] = int(rng.choice([0x00, 0x01, 0x04, 0x06, 0x08, 0x11, 0x29, 0x2F, 0x3A, 0x81,
                                       0x86, 0x88, 0xAA, 0xDD, 0xBE, 0x22, 0xEB, 0x12, 0xB5, 0xF0,
                                       int(rng.integers(0, 256))]))
        out.append(bytes(v[:int(rng.integers(max(0, len(v) - 60), len(v) + 1))]))
    buf = b"".join(out)
    lens = np.array([len(p) for p in out], np.uint32)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    g, _ = both(P, np.frombuffer(buf + bytes(16), np.uint8), len(out), offsets=offs, lens=lens,
                label="fuzz")
    # spot-check against the independent Python walk too
    for i in range(0, len(out), 997):
        st, hdrs, po, pl = pyref.parse(out[i])
        assert schema.STATUS_NAMES[g["status"][i]] == st


def test_misaligned_slab_view_rejected(P):
    ds = dev(np.zeros(256, np.uint8))
    with pytest.raises(RuntimeError):
        P.parse(ds[1:], stride=64, n=2)


# ------------------------------------------------------------------ getters and checksum
def test_extract_fields_vs_oracle(P):
    pc = open(os.path.join(GOLD, "ref22.pcap"), "rb").read()
    offs, lens = gen.pcap_index_py(pc)
    buf, offs4, lens4 = gen.gen_c4(20000, seed=77)
    slab = buf
    g = gpu_parse(P, slab, len(offs4), offsets=offs4, lens=lens4, columns=["chain"])
    specs = []
    for t in range(1, len(schema.HDR_NAMES)):
        if t == H["STP"]:
            continue
        for name, s, e in oracle.field_table(t):
            specs.append((t, 0, s, e))
    specs += [(H["IPv4"], 1, 96, 127), (H["Ether"], 1, 0, 47), (H["IPv6"], 0, 0, 71),
              (H["IPv6"], 1, 64, 191), (H["ARP"], 0, 3, 66)]
    import pktgpu  # noqa: F401
    vals, found = P.extract_fields(dev(slab), {k: dev(g[k]) for k in ("n_hdrs", "hdr_type", "hdr_off")},
                                   specs, offsets=dev(offs4), lens=dev(lens4))
    torch.cuda.synchronize()
    ov, of = oracle.extract_fields(slab, len(offs4), g, specs, offsets=offs4, lens=lens4)
    for k, sp in enumerate(specs):
        assert np.array_equal(vals[k].cpu().numpy(), ov[k]), sp
        assert np.array_equal(found[k].cpu().numpy(), of[k]), sp
    del pc, offs, lens


def test_extract_and_set_fields_deep_chains(P):
    """Getters and setters on headers deep in the chain (slot >= 8: the kernels keep the first 8
    slots in LDS and read deeper ones from the chain columns), vs the oracle."""
    slab, lens, stride = _stack_packets()
    n = len(lens)
    g = gpu_parse(P, slab, n, stride=stride, lens=lens, columns=["chain"])
    ch = {k: g[k] for k in ("n_hdrs", "hdr_type", "hdr_off")}
    specs = [(H["Vlan"], k, 4, 15) for k in range(0, 16, 3)] + [(H["MPLS"], k, 0, 19) for k in range(0, 16, 5)]
    specs += [(H["IPv4"], 0, 96, 127), (H["UDP"], 0, 0, 15), (H["Ether"], 0, 96, 111)]
    vals, found = P.extract_fields(dev(slab), {k: dev(v) for k, v in ch.items()}, specs, stride=stride,
                                   lens=dev(lens))
    torch.cuda.synchronize()
    ov, of = oracle.extract_fields(slab, n, ch, specs, stride=stride, lens=lens)
    for k, sp in enumerate(specs):
        assert np.array_equal(vals[k].cpu().numpy(), ov[k]), sp
        assert np.array_equal(found[k].cpu().numpy(), of[k]), sp
    rng = np.random.default_rng(11)
    sv = [rng.integers(0, 2**63, n, dtype=np.uint64) for _ in specs]
    ds = dev(slab.reshape(-1).copy())
    P.set_fields(ds, {k: dev(v) for k, v in ch.items()}, specs, [dev(v) for v in sv], n=n, stride=stride,
                 lens=dev(lens))
    torch.cuda.synchronize()
    want = slab.reshape(-1).copy()
    oracle.set_fields(want, n, ch, specs, sv, stride=stride, lens=lens)
    assert np.array_equal(ds.cpu().numpy(), want)


def test_ipv4_checksum_batch_sweep(P):
    """tests/lib.rs:151-204 on the device: 25 400 builder headers -> Packet::ipv4_checksum."""
    payload = bytes(range(100))
    ips = [f"{k}.{k}.{k}.1" for k in range(10, 20)]
    hdrs = []
    for sip in ips:
        for dip in ips:
            for ttl in range(1, 255):
                hdrs.append(gen.ipv4(5, 0, 115, ttl, 0, 6, sip, dip, 140).data)
    a = np.frombuffer(b"".join(hdrs), np.uint8)
    out = P.ipv4_checksum(dev(a), stride=20).cpu().numpy()
    stored = np.array([int.from_bytes(h[10:12], "big") for h in hdrs])
    assert np.array_equal(out, stored)
    rng = np.random.default_rng(3)
    r = rng.integers(0, 256, (50000, 24), dtype=np.uint8)
    out = P.ipv4_checksum(dev(r), stride=24).cpu().numpy()
    want = np.array([oracle.ipv4_checksum(r[i, :20].tobytes()) for i in range(0, 50000, 50)])
    assert np.array_equal(out[::50], want)


# ------------------------------------------------------------------ to_vec (config 1, Q2)
def test_c1_roundtrip_to_vec(P):
    """Config 1: 1 024 x 64 B parse + serialise round trip (tests/lib.rs:790-802 shape) on the
    device: every packet's to_vec equals its bytes."""
    n = 1024
    slab = gen.gen_c2(n, seed=1).reshape(-1)
    ds = dev(slab)
    res = P.parse(ds, stride=64, columns=["chain"])
    out, ln = P.to_vec(ds, res, stride=64)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), slab)
    assert (ln.cpu().numpy() == 64).all()


def test_to_vec_templates_and_gre_reorder_vs_oracle(P):
    inner = gen.create_udp_packet("00:01:02:03:04:05", "00:06:07:08:09:0a", False, 0, 0, 5,
                                  "1.1.1.1", "2.2.2.2", 0, 64, 0, 0, [], 53, 1000, False, b"x" * 8)
    inner.remove(0)
    pkts = [p.to_vec() for p in gen.reference_22_packets()]
    for c, k, s in ((1, 1, 1), (1, 0, 1), (0, 1, 1), (1, 1, 0)):
        pkts.append(gen.create_gre_packet("00:01:02:03:04:05", "00:06:07:08:09:0a", False, 0, 0, 5,
                                          "3.3.3.3", "4.4.4.4", 0, 64, 0, 0, [], c, 0, k, s, 0, 0, 0,
                                          0x1111, 0x2222, 0x33333333, 0x44444444, b"", inner).to_vec())
    pkts.append(pkts[0][:30])  # truncated: not written
    buf = b"".join(pkts)
    lens = np.array([len(p) for p in pkts], np.uint32)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    slab = np.frombuffer(buf + bytes(16), np.uint8)
    ds, do, dl = dev(slab), dev(offs), dev(lens)
    res = P.parse(ds, offsets=do, lens=dl, columns=["chain"])
    out, ln = P.to_vec(ds, res, offsets=do, lens=dl)
    torch.cuda.synchronize()
    o, ln = out.cpu().numpy(), ln.cpu().numpy()
    reordered = 0
    for i, p in enumerate(pkts):
        try:
            want = oracle.slow_parse_to_vec(p)
        except ValueError:
            assert ln[i] == 0
            continue
        got = o[offs[i]:offs[i] + ln[i]].tobytes()
        assert got == want, i
        reordered += got != p
    assert reordered == 4  # the four GRE packets, each with >= 2 options (Q2)


@pytest.mark.parametrize("shift", [0, 1, 6])
def test_to_vec_c4_dst_layouts_vs_oracle(P, shift):
    """C4 records (plus Q2 GRE packets and truncated ones) serialised into a packed destination
    whose records start `shift` bytes off the source's 16-byte phase: the kernel's aligned
    16-byte path (shift 0 keeps the phase), its dword path and the Q2 gather all equal the
    oracle's slow::parse(..).to_vec() (tests/lib.rs:790-802)."""
    n = 1 << 16
    slab, offs, lens = gen.gen_c4(n, seed=11)
    rng = np.random.default_rng(shift)
    cut = rng.random(n) < 0.02  # some truncated records: nothing written, out_len 0
    lens = np.where(cut, (lens * rng.random(n)).astype(np.uint32), lens).astype(np.uint32)
    ds, do, dl = dev(slab), dev(offs), dev(lens)
    res = P.parse(ds, offsets=do, lens=dl, columns=["chain"])
    dst_off = (offs + np.uint64(shift)) if shift == 0 else \
        (np.concatenate([[0], np.cumsum(lens.astype(np.uint64) + np.uint64(3))[:-1]]) + np.uint64(shift))
    dst_len = int(dst_off[-1]) + int(lens[-1]) + 64
    dst = torch.full((dst_len,), 0xEE, dtype=torch.uint8, device="cuda")
    out, ln = P.to_vec(ds, res, offsets=do, lens=dl, dst=dst, dst_offsets=dev(dst_off.astype(np.uint64)))
    torch.cuda.synchronize()
    o, ln = out.cpu().numpy(), ln.cpu().numpy()
    want, wl = oracle.round_trip_batch(slab, n, offsets=offs, lens=lens, slow=True, nthreads=8)
    assert np.array_equal(ln, wl)
    for i in range(n):
        a, b, k = int(offs[i]), int(dst_off[i]), int(wl[i])
        assert o[b:b + k].tobytes() == want[a:a + k].tobytes(), i
    # nothing outside the written records changed
    mask = np.ones(dst_len, bool)
    for i in range(n):
        mask[int(dst_off[i]):int(dst_off[i]) + int(wl[i])] = False
    assert (o[mask] == 0xEE).all()


@pytest.mark.parametrize("gap", [16, 5])
def test_to_vec_input_layout_edges_vs_oracle(P, gap):
    """to_vec into the input's own layout (dst_offsets NULL) of an indexed batch: with 16-byte gaps
    between the records (a capture's record headers) no 16-byte chunk holds two records' bytes and
    the partial edge chunks are read-modify-written whole; with 5-byte gaps neighbouring records share
    chunks and the kernel keeps the byte-exact edge stores.  Every to_vec equals the oracle and no
    byte outside the written packets changes."""
    n = 20000
    slab0, offs0, lens = gen.gen_c4(n, seed=77 + gap)
    rng = np.random.default_rng(gap)
    cut = rng.random(n) < 0.02  # truncated records: nothing written
    lens = np.where(cut, np.maximum(1, (lens * rng.random(n)).astype(np.uint32)), lens).astype(np.uint32)
    offs = np.concatenate([[24 + gap], 24 + gap + np.cumsum(lens.astype(np.uint64) + np.uint64(gap))[:-1]]).astype(np.uint64)
    total = int(offs[-1]) + int(lens[-1]) + 32
    buf = np.zeros(total, np.uint8)
    for i in range(n):
        a, b = int(offs0[i]), int(offs[i])
        buf[b:b + int(lens[i])] = slab0[a:a + int(lens[i])]
    ds, do, dl = dev(buf), dev(offs), dev(lens)
    res = P.parse(ds, offsets=do, lens=dl, columns=["chain"])
    dst = torch.full((total,), 0xEE, dtype=torch.uint8, device="cuda")
    out, ln = P.to_vec(ds, res, offsets=do, lens=dl, dst=dst)
    torch.cuda.synchronize()
    o, ln = out.cpu().numpy(), ln.cpu().numpy()
    want, wl = oracle.round_trip_batch(buf, n, offsets=offs, lens=lens, slow=True, nthreads=8)
    assert np.array_equal(ln, wl)
    mask = np.ones(total, bool)
    for i in range(n):
        a, k = int(offs[i]), int(wl[i])
        assert o[a:a + k].tobytes() == want[a:a + k].tobytes(), i
        mask[a:a + k] = False
    assert (o[mask] == 0xEE).all()


def test_to_vec_long_packets_both_chunk_maps_vs_oracle(P):
    """Waves whose outputs exceed the kernel's per-wave start map (> 2048 16-byte chunks: 64
    records of ~1.4 KB) next to waves of short records (the map path), in a pcap-like layout with
    16-byte gaps, plus truncated records: every to_vec equals the oracle's slow::parse(..).to_vec()
    and no gap byte of the destination changes (tests/lib.rs:790-802 round trip)."""
    n = 512
    pkts = []
    for i in range(n):
        big = (i // 64) % 2 == 0
        pay = bytes((i * 7 + j) & 0xFF for j in range(1400 - (i % 9) if big else i % 50))
        pkts.append(gen.create_udp_packet("00:01:02:03:04:05", "00:06:07:08:09:0a", False, 0, 0, 5,
                                          "1.1.1.1", "2.2.2.2", 0, 64, 0, 0, [], 1000 + i, 2000, False,
                                          pay).to_vec())
    for i in range(3, n, 97):
        pkts[i] = pkts[i][:20]  # truncated: not written, out_len 0
    lens = np.array([len(x) for x in pkts], np.uint32)
    offs = np.concatenate([[16], 16 + np.cumsum(lens.astype(np.uint64) + np.uint64(16))[:-1]]).astype(np.uint64)
    total = int(offs[-1]) + int(lens[-1]) + 16
    buf = bytearray(total)
    for i, x in enumerate(pkts):
        buf[int(offs[i]):int(offs[i]) + len(x)] = x
    slab = np.frombuffer(bytes(buf), np.uint8)
    ds, do, dl = dev(slab), dev(offs), dev(lens)
    res = P.parse(ds, offsets=do, lens=dl, columns=["chain"])
    dst = torch.full((total,), 0xEE, dtype=torch.uint8, device="cuda")
    out, ln = P.to_vec(ds, res, offsets=do, lens=dl, dst=dst)
    torch.cuda.synchronize()
    o, ln = out.cpu().numpy(), ln.cpu().numpy()
    mask = np.ones(total, bool)
    for i, x in enumerate(pkts):
        try:
            want = oracle.slow_parse_to_vec(x)
        except ValueError:
            assert ln[i] == 0, i
            continue
        assert ln[i] == len(want), i
        assert o[int(offs[i]):int(offs[i]) + len(want)].tobytes() == want, i
        mask[int(offs[i]):int(offs[i]) + len(want)] = False
    assert (o[mask] == 0xEE).all()


@pytest.mark.parametrize("layout", ["capture", "lead_gap_exact_dst", "dense_windows", "far_gap"])
def test_to_vec_capture_windows_vs_oracle(P, layout):
    """to_vec into a capture's own layout goes by destination window (4 KiB per wave, the records'
    starts mapped per window): C4 records, Q2 GRE packets (list order != wire order, gathered by the
    window holding their start), truncated records (nothing written, out_len 0) and 1.4 KB records
    crossing windows, with 16-byte record headers between them.  Layouts: a pcap (24-byte global
    header first); a 100 KB lead before the first record and a destination ending at the last
    record's last byte (its final 16-byte chunk partial); > 64 records starting in one window (36-byte
    records: the window takes them 64 at a time); one gap of 600 KB (a record spanning more than the
    window table allows: to_vec_kernel takes the batch).  Each equals the oracle's
    slow::parse(..).to_vec() (tests/lib.rs:790-802) and no other destination byte changes."""
    inner = gen.create_udp_packet("00:01:02:03:04:05", "00:06:07:08:09:0a", False, 0, 0, 5,
                                  "1.1.1.1", "2.2.2.2", 0, 64, 0, 0, [], 53, 1000, False, b"x" * 8)
    inner.remove(0)
    q2 = [gen.create_gre_packet("00:01:02:03:04:05", "00:06:07:08:09:0a", False, 0, 0, 5, "3.3.3.3", "4.4.4.4",
                                0, 64, 0, 0, [], c, 0, k, s, 0, 0, 0, 0x1111, 0x2222, 0x33333333, 0x44444444,
                                b"", inner).to_vec() for c, k, s in ((1, 1, 1), (1, 0, 1), (0, 1, 1), (1, 1, 0))]
    rng = np.random.default_rng(len(layout))
    s4, o4, l4 = gen.gen_c4(6000, seed=90 + len(layout))
    pk = []
    for i in range(6000):
        r = rng.random()
        if r < 0.03:
            pk.append(q2[int(rng.integers(0, 4))])
        elif layout == "dense_windows" and r < 0.6:
            pk.append(q2[0][:20] if r < 0.3 else bytes(s4[int(o4[i]):int(o4[i]) + 20]))  # 36-byte records
        elif r < 0.05:
            pk.append(bytes(s4[int(o4[i]):int(o4[i]) + int(rng.integers(1, 40))]))
        elif r < 0.07:
            pk.append(gen.create_udp_packet("00:01:02:03:04:05", "00:06:07:08:09:0a", False, 0, 0, 5, "1.1.1.1",
                                            "2.2.2.2", 0, 64, 0, 0, [], 7, 9, False, bytes(1400 - i % 13)).to_vec())
        else:
            pk.append(bytes(s4[int(o4[i]):int(o4[i]) + int(l4[i])]))
    n = len(pk)
    lens = np.array([len(x) for x in pk], np.uint64)
    gaps = np.full(n, 16, np.uint64)
    gaps[0] = {"capture": 40, "lead_gap_exact_dst": 100_000, "dense_windows": 40, "far_gap": 40}[layout]
    if layout == "far_gap":
        gaps[n // 2] = 600_000
    offs = np.cumsum(gaps) + np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    end = int(offs[-1] + lens[-1])
    total = end if layout == "lead_gap_exact_dst" else end + 40
    buf = rng.integers(0, 256, total, dtype=np.uint8)
    for i, x in enumerate(pk):
        buf[int(offs[i]):int(offs[i]) + len(x)] = np.frombuffer(x, np.uint8)
    ds, do, dl = dev(buf), dev(offs), dev(lens.astype(np.uint32))
    res = P.parse(ds, offsets=do, lens=dl, columns=["chain"])
    dst = torch.full((total,), 0xEE, dtype=torch.uint8, device="cuda")
    out, ln = P.to_vec(ds, res, offsets=do, lens=dl, dst=dst)
    torch.cuda.synchronize()
    o, ln = out.cpu().numpy(), ln.cpu().numpy()
    mask = np.ones(total, bool)
    reordered = 0
    for i, x in enumerate(pk):
        try:
            want = oracle.slow_parse_to_vec(x)
        except ValueError:
            assert ln[i] == 0, i
            continue
        a = int(offs[i])
        assert ln[i] == len(want), i
        assert o[a:a + len(want)].tobytes() == want, i
        reordered += want != x
        mask[a:a + len(want)] = False
    assert reordered > 0
    assert (o[mask] == 0xEE).all()


@pytest.mark.parametrize("layout", ["packed", "gaps_shift", "truncated", "exact_end", "q2_fallback"])
def test_to_vec_dst_layouts_in_order_vs_oracle(P, layout):
    """to_vec into a destination layout of its own (dst_offsets), records in order: chunks holding the
    end of one record and the start of the next (their source alignments differ).  Layouts: packed
    back to back (the bench's); 1-9 byte gaps and an odd start; records truncated to 17-40 bytes (not
    parsed: nothing written, their bytes left untouched); a destination ending at the last record's
    last byte; a batch holding a Q2 GRE packet.  Every to_vec and out_len equals the oracle's
    slow::parse(..).to_vec() (tests/lib.rs:790-802) and no other destination byte changes.  (Round 6
    measured a by-window kernel for these layouts and kept to_vec_kernel: profiles/ab/r06zr_*.)"""
    s4, o4, l4 = gen.gen_c4(30000, seed=70 + len(layout))
    rng = np.random.default_rng(len(layout))
    pk = [bytes(s4[int(o4[i]):int(o4[i]) + int(l4[i])]) for i in range(len(o4))]
    if layout == "truncated":
        for i in rng.choice(len(pk), 1500, replace=False):
            pk[i] = pk[i][:int(rng.integers(17, 41))]
    if layout == "q2_fallback":
        inner = gen.create_udp_packet("00:01:02:03:04:05", "00:06:07:08:09:0a", False, 0, 0, 5,
                                      "1.1.1.1", "2.2.2.2", 0, 64, 0, 0, [], 53, 1000, False, b"x" * 8)
        inner.remove(0)
        pk[777] = gen.create_gre_packet("00:01:02:03:04:05", "00:06:07:08:09:0a", False, 0, 0, 5, "3.3.3.3",
                                        "4.4.4.4", 0, 64, 0, 0, [], 1, 0, 1, 1, 0, 0, 0, 0x1111, 0x2222,
                                        0x33333333, 0x44444444, b"", inner).to_vec()
    n = len(pk)
    lens = np.array([len(x) for x in pk], np.uint64)
    offs = np.concatenate([[0], np.cumsum(lens + np.uint64(16))[:-1]]).astype(np.uint64) + np.uint64(40)
    buf = np.zeros(int(offs[-1] + lens[-1]) + 64, np.uint8)
    for i, x in enumerate(pk):
        buf[int(offs[i]):int(offs[i]) + len(x)] = np.frombuffer(x, np.uint8)
    gaps = rng.integers(1, 10, n).astype(np.uint64) if layout == "gaps_shift" else np.zeros(n, np.uint64)
    start = np.uint64(5 if layout == "gaps_shift" else 0)
    doff = np.concatenate([[0], np.cumsum(lens + gaps)[:-1]]).astype(np.uint64) + start
    end = int(doff[-1] + lens[-1])
    dst_len = end if layout == "exact_end" else end + 100
    ds, do, dl = dev(buf), dev(offs), dev(lens.astype(np.uint32))
    res = P.parse(ds, offsets=do, lens=dl, columns=["chain"])
    dst = torch.full((dst_len,), 0xEE, dtype=torch.uint8, device="cuda")
    out, ln = P.to_vec(ds, res, offsets=do, lens=dl, dst=dst, dst_offsets=dev(doff))
    torch.cuda.synchronize()
    o, ln = out.cpu().numpy(), ln.cpu().numpy()
    mask = np.ones(dst_len, bool)
    for i, x in enumerate(pk):
        try:
            want = oracle.slow_parse_to_vec(x)
        except ValueError:
            assert ln[i] == 0, i
            continue
        a = int(doff[i])
        assert ln[i] == len(want), i
        assert o[a:a + len(want)].tobytes() == want, i
        mask[a:a + len(want)] = False
    assert (o[mask] == 0xEE).all()


def test_to_vec_capture_empty_last_record_at_a_window_start(P):
    """A capture-layout batch whose last record is empty and starts exactly at a 4 KiB boundary: an
    empty record sends the batch to to_vec_kernel (the window path would have no window to write its
    out_len); every out_len (0 for the empty record) and every to_vec equals the oracle."""
    s4, o4, l4 = gen.gen_c4(200, seed=123)
    pk = [bytes(s4[int(o4[i]):int(o4[i]) + int(l4[i])]) for i in range(200)]
    lens = np.array([len(x) for x in pk] + [0], np.uint64)
    offs = np.zeros(len(lens), np.uint64)
    offs[0] = 40
    for i in range(1, len(lens) - 1):
        offs[i] = offs[i - 1] + lens[i - 1] + np.uint64(16)
    end = int(offs[-2] + lens[-2])
    offs[-1] = np.uint64((end + 16 + 4095) // 4096 * 4096)
    total = int(offs[-1]) + 64
    buf = np.zeros(total, np.uint8)
    for i, x in enumerate(pk):
        buf[int(offs[i]):int(offs[i]) + len(x)] = np.frombuffer(x, np.uint8)
    ds, do, dl = dev(buf), dev(offs), dev(lens.astype(np.uint32))
    res = P.parse(ds, offsets=do, lens=dl, columns=["chain"])
    dst = torch.full((total,), 0xEE, dtype=torch.uint8, device="cuda")
    out, ln = P.to_vec(ds, res, offsets=do, lens=dl, dst=dst)
    torch.cuda.synchronize()
    o, ln = out.cpu().numpy(), ln.cpu().numpy()
    assert ln[-1] == 0
    for i, x in enumerate(pk):
        want = oracle.slow_parse_to_vec(x)
        assert ln[i] == len(want) and o[int(offs[i]):int(offs[i]) + len(want)].tobytes() == want, i


# ------------------------------------------------------------------ mixed inputs
def test_mixed_inputs_bit_exact(P):
    """The reference pcap, a C4 replay, C3/C2 slabs and random/truncated records under three
    entries: every column equals the oracle."""
    pc = open(os.path.join(GOLD, "ref22.pcap"), "rb").read()
    offs, lens = gen.pcap_index_py(pc)
    both(P, np.frombuffer(pc, np.uint8), 22, offsets=offs, lens=lens, label="ref22")
    buf, offs, lens = gen.gen_c4(50000, seed=41)
    both(P, buf, len(offs), offsets=offs, lens=lens, label="c4")
    slab = gen.gen_c3(50001, seed=42)
    both(P, slab, 50001, stride=128, label="c3")
    slab = gen.gen_c2(4099, seed=43)
    both(P, slab, 4099, stride=64, label="c2")
    rng = np.random.default_rng(44)
    pk = [rng.integers(0, 256, int(rng.integers(0, 90)), dtype=np.uint8).tobytes() for _ in range(5000)]
    pk += [p.to_vec()[:int(rng.integers(10, 120))] for p in gen.reference_22_packets() for _ in range(50)]
    b = b"".join(pk)
    ln = np.array([len(x) for x in pk], np.uint32)
    of = np.concatenate([[0], np.cumsum(ln)[:-1]]).astype(np.uint64)
    for entry in ("parse", "parse_ethernet", "parse_ipv4"):
        both(P, np.frombuffer(b + bytes(16), np.uint8), len(pk), offsets=of, lens=ln, entry=entry,
             label=f"mix {entry}")


# ------------------------------------------------------------------ register fast path
def _fastpath_mix(n, stride, seed):
    """C2-shaped packets with the fields the fast-path classifier reads mutated (EtherType,
    IP protocol, UDP dst incl. 4789) and lengths clustered around the UDP (42) and TCP (54)
    header ends, so waves mix fast and walked lanes and every boundary is crossed."""
    rng = np.random.default_rng(seed)
    a = gen.gen_c2(n, seed=seed, stride=stride)
    tcp = rng.random(n) < 0.35
    a[tcp, 23] = 6
    r = rng.random(n)
    a[r < 0.04, 12:14] = [0x86, 0xDD]
    a[(r >= 0.04) & (r < 0.08), 12:14] = [0x81, 0x00]
    a[(r >= 0.08) & (r < 0.10), 12:14] = [0x08, 0x01]
    a[(r >= 0.10) & (r < 0.12), 12:14] = [0x05, 0xDB]  # < 1500: Dot3
    p = rng.random(n)
    a[p < 0.03, 23] = rng.choice([1, 4, 41, 47, 58, 0x11, 0x06], int((p < 0.03).sum()))
    a[(p >= 0.03) & (p < 0.06), 36:38] = [0x12, 0xB5]  # VXLAN port
    lens = np.where(rng.random(n) < 0.5, rng.integers(36, 60, n), rng.integers(0, stride + 1, n))
    return a, lens.astype(np.uint32)


@pytest.mark.parametrize("fast", [1, 0])
def test_fastpath_classifier_boundaries(P, fast):
    """Fixed stride with per-packet lengths: fast path on and off both equal the oracle."""
    P.set_fastpath(fast)
    try:
        for stride in (64, 72, 80, 104, 128):  # 72, 104: every other packet 16-byte aligned
            n = 40003
            a, lens = _fastpath_mix(n, stride, seed=stride + fast)
            for entry in ("parse", "parse_ethernet", "parse_ipv4"):
                both(P, a, n, stride=stride, lens=lens, entry=entry, label=f"s{stride} {entry} f{fast}")
            both(P, a, n, stride=stride, label=f"s{stride} full f{fast}")
            # aligned indexed batch (offsets multiples of 16) and a misaligned one
            offs = (np.arange(n, dtype=np.uint64) * stride)
            both(P, a, n, offsets=offs, lens=lens, label=f"idx s{stride} f{fast}")
            both(P, np.concatenate([np.zeros(8, np.uint8), a.reshape(-1), np.zeros(8, np.uint8)]), n,
                 offsets=offs + 8, lens=lens, label=f"idx+8 s{stride} f{fast}")
    finally:
        P.set_fastpath(1)


def test_fastpath_windows_and_columns(P):
    """Narrow windows (no fast path below 64 B) and every column subset agree with the oracle."""
    n = 20000
    a, lens = _fastpath_mix(n, 64, seed=77)
    for w in (16, 32, 48, 64):
        both(P, a, n, stride=64, lens=lens, window=w, label=f"w{w}")
    for cols in (["status"], ["chain"], ["ether"], ["ipv4"], ["udp"], ["tcp"], ["chain", "udp", "tcp"],
                 ["ipv4_csum_calc", "udp_dst", "hdr_off", "n_hdrs"]):
        both(P, a, n, stride=64, lens=lens, columns=cols, label=f"cols {cols}")


# ------------------------------------------------------------------ launch modes (grid, staging)
def _mode_cases(P, label):
    """Every launch mode must agree with the oracle on the same mixes: golden pcap, C4 pcap
    (indexed, unaligned records), C3/C2 fixed stride, the fast-path mix with per-packet lengths,
    and random/truncated records back to back."""
    pc = open(os.path.join(GOLD, "ref22.pcap"), "rb").read()
    offs, lens = gen.pcap_index_py(pc)
    both(P, np.frombuffer(pc, np.uint8), 22, offsets=offs, lens=lens, label=f"ref22 {label}")
    buf, offs, lens = gen.gen_c4(30011, seed=51)
    both(P, buf, len(offs), offsets=offs, lens=lens, label=f"c4 {label}")
    both(P, buf, len(offs), offsets=offs, lens=lens, columns=["chain"], label=f"c4 chain {label}")
    slab = gen.gen_c3(20011, seed=52)
    both(P, slab, 20011, stride=128, label=f"c3 {label}")
    slab = gen.gen_c2(70001, seed=53)
    both(P, slab, 70001, stride=64, columns=["chain", "ether", "ipv4", "udp"], label=f"c2 {label}")
    a, ln = _fastpath_mix(20000, 64, seed=54)
    both(P, a, 20000, stride=64, lens=ln, label=f"fastmix {label}")
    rng = np.random.default_rng(55)
    pk = [rng.integers(0, 256, int(rng.integers(0, 90)), dtype=np.uint8).tobytes() for _ in range(3000)]
    pk += [p.to_vec()[:int(rng.integers(10, 300))] for p in gen.reference_22_packets() for _ in range(40)]
    b = b"".join(pk)
    ln = np.array([len(x) for x in pk], np.uint32)
    of = np.concatenate([[0], np.cumsum(ln)[:-1]]).astype(np.uint64)
    for entry in ("parse", "parse_ipv4", "parse_gre"):
        both(P, np.frombuffer(b + bytes(16), np.uint8), len(pk), offsets=of, lens=ln, entry=entry,
             label=f"mix {entry} {label}")
    # records out of order and far apart (wave ranges beyond the span region: window fallback)
    perm = rng.permutation(len(pk))
    both(P, np.frombuffer(b + bytes(16), np.uint8), len(pk), offsets=of[perm], lens=ln[perm],
         label=f"shuffled {label}")
    # one long record per wave (> 16 KiB range) next to short ones
    big = np.zeros(40000, np.uint8)
    big[:64] = gen.gen_c2(1, seed=56)[0]
    of2 = np.array([0, 20000, 39000, 100, 200], np.uint64)
    ln2 = np.array([40000, 64, 1000, 64, 50], np.uint32)
    both(P, big, 5, offsets=of2, lens=ln2, label=f"long {label}")


@pytest.mark.parametrize("staging", [1, 2])
def test_staging_modes_bit_exact(P, staging):
    """Per-lane windows (1) and wave spans (2) give identical columns; staging 3 (round 3's
    pipelined windows) is gone and rejected."""
    with pytest.raises(RuntimeError):
        P.set_staging(3)
    P.set_staging(staging)
    try:
        _mode_cases(P, f"st{staging}")
        for w in (16, 64, 144):
            P.set_window(w)
            buf, offs, lens = gen.gen_c4(5003, seed=57 + w)
            both(P, buf, len(offs), offsets=offs, lens=lens, window=w, label=f"c4 w{w} st{staging}")
    finally:
        P.set_staging(0)
        P.set_window(0)


@pytest.mark.parametrize("window", [80, 96, 112, 144])
def test_lockstep_window_widths(P, window):
    """The lockstep walk is compiled for 6, 7, 9 and 17 chunks (window requests up to 80, 96,
    128 and 256 B); 112 and 144 are widened to 9 and 17 chunks: every width is bit-exact on C4."""
    buf, offs, lens = gen.gen_c4(20011, seed=window)
    both(P, buf, len(offs), offsets=offs, lens=lens, window=window, label=f"c4 w{window}")


@pytest.mark.parametrize("staging", [0, 2])
@pytest.mark.parametrize("n", [1, 63, 64, 65, 1000, 65537])
def test_indexed_sizes_and_wide_ranges(P, n, staging):
    """Indexed batches around the wave / block sizes, with jumbo records (wave ranges past the
    span staging's 16 KiB: its per-lane fallback) mixed with tiny, empty and truncated ones."""
    rng = np.random.default_rng(n)
    tm = [p.to_vec() for p in gen.reference_22_packets()]
    pk = []
    for k in range(n):
        u = rng.random()
        if u < 0.02:
            pk.append(tm[int(rng.integers(0, 22))] + bytes(int(rng.integers(1000, 9000))))  # jumbo
        elif u < 0.04:
            pk.append(tm[int(rng.integers(0, 22))][:int(rng.integers(0, 40))])               # truncated
        else:
            pk.append(tm[int(rng.integers(0, 22))])
    buf = gen.pcap_bytes(pk)
    offs, lens = gen.pcap_index_py(buf)
    P.set_staging(staging)
    try:
        both(P, np.frombuffer(buf, np.uint8), n, offsets=offs, lens=lens, label=f"st{staging} n={n}")
        both(P, np.frombuffer(buf, np.uint8), n, offsets=offs, lens=lens, columns=["chain"], label=f"st{staging} chain n={n}")
    finally:
        P.set_staging(0)


@pytest.mark.parametrize("walk", [1, 2])
def test_walk_modes_bit_exact(P, walk):
    """Waterfall (1) and lockstep (2) walks give identical columns on every mix, every entry,
    truncations, depth limits and GRE option combinations; and with wave spans."""
    P.set_walk(walk)
    try:
        _mode_cases(P, f"wk{walk}")
        rng = np.random.default_rng(61)
        tm = [p.to_vec() for p in gen.reference_22_packets()]
        for entry in schema.ENTRIES:
            pk = [t[int(rng.integers(0, 14)):] for t in tm] + [rng.integers(0, 256, int(rng.integers(0, 80)), dtype=np.uint8).tobytes() for _ in range(300)]
            b = b"".join(pk)
            ln = np.array([len(x) for x in pk], np.uint32)
            of = np.concatenate([[0], np.cumsum(ln)[:-1]]).astype(np.uint64)
            both(P, np.frombuffer(b + bytes(16), np.uint8), len(pk), offsets=of, lens=ln, entry=entry,
                 label=f"{entry} wk{walk}")
        for st in (2,):
            P.set_staging(st)
            buf, offs, lens = gen.gen_c4(20011, seed=62)
            both(P, buf, len(offs), offsets=offs, lens=lens, label=f"c4 st{st} wk{walk}")
    finally:
        P.set_walk(0)
        P.set_staging(0)


def _vlan_fastpath_mix(n, seed):
    """C3-shaped packets (0-2 VLAN tags, IPv4, TCP|UDP) with per-packet lengths around every
    fast-path bound (42/54 + 4v), UDP dst 4789 at the tag-shifted offset, a third tag, and
    EtherTypes after the tags mutated, so every branch of the VLAN fast-path classifier is hit."""
    rng = np.random.default_rng(seed)
    a = gen.gen_c3(n, seed=seed)
    tags = np.zeros(n, np.int64)
    tags[(a[:, 12] == 0x81) & (a[:, 13] == 0)] = 1
    tags[(tags == 1) & (a[:, 16] == 0x81) & (a[:, 17] == 0)] = 2
    l4 = 34 + 4 * tags
    udp = a[np.arange(n), 23 + 4 * tags] == 17
    r = rng.random(n)
    m = (r < 0.05) & udp  # VXLAN port at the shifted UDP dst
    a[np.nonzero(m)[0], (l4 + 2)[m]] = 0x12
    a[np.nonzero(m)[0], (l4 + 3)[m]] = 0xB5
    m = (r >= 0.05) & (r < 0.08) & (tags == 2)  # a third tag
    a[np.nonzero(m)[0], 20] = 0x81
    a[np.nonzero(m)[0], 21] = 0x00
    m = (r >= 0.08) & (r < 0.11) & (tags >= 1)  # EtherType after the first tag neither IPv4 nor Vlan
    a[np.nonzero(m)[0], 16] = 0x86
    a[np.nonzero(m)[0], 17] = 0xDD
    m = (r >= 0.11) & (r < 0.14)  # protocol neither TCP nor UDP
    a[np.nonzero(m)[0], (23 + 4 * tags)[m]] = 47
    bound = l4 + np.where(udp, 8, 20)
    lens = np.where(rng.random(n) < 0.6, bound + rng.integers(-3, 3, n), rng.integers(0, 129, n))
    return a, np.clip(lens, 0, 128).astype(np.uint32)


@pytest.mark.parametrize("fast", [1, 0])
def test_vlan_fastpath_boundaries(P, fast):
    """The fast path for Ether/0-2 Vlan/IPv4/TCP|UDP agrees with the walk (and the oracle) at every
    length bound, shifted VXLAN port, third tag and non-IPv4 EtherType after a tag."""
    P.set_fastpath(fast)
    try:
        n = 60001
        a, lens = _vlan_fastpath_mix(n, seed=70 + fast)
        for entry in ("parse", "parse_ethernet"):
            both(P, a, n, stride=128, lens=lens, entry=entry, label=f"vlan {entry} f{fast}")
        both(P, a, n, stride=128, label=f"vlan full f{fast}")
        both(P, a, n, stride=128, lens=lens, columns=["chain", "vlan", "ipv4", "tcp", "udp"],
             label=f"vlan cols f{fast}")
    finally:
        P.set_fastpath(1)


@pytest.mark.parametrize("same", [True, False])
def test_parse_batches_vs_oracle(P, same):
    """pkt_parse_batches — K = 3 batches in one call.  Equal sizes with one packed
    output buffer each (a common column distance) take ONE launch over the three batches' tiles;
    different sizes fall back to one launch per batch.  Every batch must equal the oracle."""
    import torch
    from pktgpu.mgpu import packed_bytes, packed_views
    cols = schema.columns_of(["chain", "ether", "ipv4", "udp"])
    sizes = [1 << 17] * 3 if same else [70001, 1, 130000]
    bts, outs, refs = [], [], []
    for k, n in enumerate(sizes):
        slab = gen.gen_c2(n, seed=300 + k)
        t = torch.from_numpy(slab.reshape(-1)).cuda()
        buf = torch.full((packed_bytes(cols, n),), 0xEE, dtype=torch.uint8, device="cuda")
        bts.append((t, n, 64, None, None))
        outs.append(packed_views(buf, cols, n))
        refs.append(oracle.parse_batch(slab, n, stride=64, columns=cols, nthreads=8))
    P.parse_batches(bts, outs)
    for k in range(3):
        compare({c: v.cpu().numpy() for c, v in outs[k].items()}, refs[k], f"batch {k} same={same}")
    # indexed (C4) batches of equal size, all columns, one launch
    bts, outs, refs = [], [], []
    for k in range(3):
        buf, offs, lens = gen.gen_c4(40000, seed=310 + k)
        bts.append((torch.from_numpy(buf).cuda(), 40000, None, torch.from_numpy(offs).cuda(),
                    torch.from_numpy(lens).cuda()))
        b = torch.full((packed_bytes("all", 40000),), 0xEE, dtype=torch.uint8, device="cuda")
        outs.append(packed_views(b, "all", 40000))
        refs.append(oracle.parse_batch(buf, 40000, offsets=offs, lens=lens, nthreads=8))
    P.parse_batches(bts, outs)
    for k in range(3):
        compare({c: v.cpu().numpy() for c, v in outs[k].items()}, refs[k], f"c4 batch {k}")


def test_parse_batches_ipv6_alignment(P):
    """pkt_parse_batches' one-launch path addresses batch k's columns as batch 0's + a
    common distance, so it is taken only when that distance keeps the IPv6 address columns 16-byte
    aligned.  Distance % 16 == 0 (but not a multiple of 256): one launch, every batch == oracle;
    distance % 16 == 8: the per-batch path validates each batch and rejects the misaligned one."""
    import torch
    from pktgpu.mgpu import packed_bytes, packed_views
    n = 4096
    ins, refs = [], []
    for k in range(2):
        buf, offs, lens = gen.gen_c4(n, seed=320 + k)
        ins.append((torch.from_numpy(buf).cuda(), n, None, torch.from_numpy(offs).cuda(),
                    torch.from_numpy(lens).cuda()))
        refs.append(oracle.parse_batch(buf, n, offsets=offs, lens=lens, nthreads=8))
    nb = (packed_bytes("all", n) + 255) // 256 * 256
    for pad, ok in ((16, True), (8, False)):
        dist = nb + pad
        big = torch.full((2 * dist + 256,), 0xEE, dtype=torch.uint8, device="cuda")
        outs = [packed_views(big[k * dist:], "all", n) for k in range(2)]
        if ok:
            P.parse_batches(ins, outs)
            for k in range(2):
                compare({c: v.cpu().numpy() for c, v in outs[k].items()}, refs[k], f"pad {pad} batch {k}")
        else:
            with pytest.raises(RuntimeError):
                P.parse_batches(ins, outs)
