"""GPU packet generation (pkt_gen_*, pktgpu.pktgen) against the host builders and the oracle.

Every one of the 22 templates of create_packet_test (tests/lib.rs:220-671, built by the
utils.rs:7-876 builders restated in pktgpu/gen.py) is generated with its builder arguments varied
per packet.  Two checks per template:
  - sampled packets are byte-equal to the BUILDER called with that packet's arguments (the
    reference's "new packet in every iteration" loop, tests/lib.rs:762-768);
  - the whole batch equals the oracle's clone + set_bit_range (headers.rs:315-324) +
    Packet::ipv4_checksum refresh (packet.rs:93-107) of every packet (oracle/pkt_oracle.c).
"""
import numpy as np
import pytest

import oracle
from pktgpu import gen

import pktgen_templates as T

pytestmark = pytest.mark.gpu

@pytest.fixture(scope="module")
def P():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.fail("no GPU visible")
    import pktgpu
    return pktgpu.Parser(0)


@pytest.mark.parametrize("name", gen.REFERENCE_22_NAMES)
def test_template_generation_matches_builder_and_oracle(P, name):
    import torch
    from pktgpu import pktgen
    tpl = T.template_bytes(name)
    n, first = 4096, 1000
    gf, values, host_vals, csum, build = T.make_case(name, n, first)
    G = pktgen.Generator(P, tpl, gf, csum=csum)
    stride = G.default_stride() + 16
    dvals = {j: torch.from_numpy(v).cuda() for j, v in values.items()}
    out = G.run(n, stride, values=dvals, first=first).cpu().numpy().reshape(n, stride)
    # whole batch vs the oracle
    want = T.oracle_batch(tpl, n, stride, [(f.hdr, f.occurrence, f.start, f.end) for f in gf], host_vals, csum)
    bad = np.nonzero((out != want).any(axis=1))[0]
    assert bad.size == 0, f"{name}: {bad.size} packets differ from the oracle, first {bad[:5]}"
    # sampled packets vs the builder called with that packet's arguments
    for i in list(range(0, n, 211)) + [n - 1]:
        want_b = build(T.builder_args(name, host_vals, i)).to_vec()
        assert out[i, :len(tpl)].tobytes() == want_b, (name, i)
        assert not out[i, len(tpl):].any()


def test_gen_udp_matches_host_builder(P):
    """Every packet equals create_udp_packet(...) with that packet's field values."""
    import torch
    from pktgpu import pktgen
    n = 20000
    rng = np.random.default_rng(12)
    f = {"eth_dst": rng.integers(0, 2**48, n, dtype=np.uint64),
         "eth_src": rng.integers(0, 2**48, n, dtype=np.uint64),
         "ipv4_diffserv": rng.integers(0, 256, n).astype(np.uint64),
         "ipv4_identification": rng.integers(0, 65536, n).astype(np.uint64),
         "ipv4_ttl": rng.integers(1, 256, n).astype(np.uint64),
         "ipv4_src": rng.integers(0, 2**32, n, dtype=np.uint64),
         "ipv4_dst": rng.integers(0, 2**32, n, dtype=np.uint64),
         "udp_src": rng.integers(0, 65536, n).astype(np.uint64),
         "udp_dst": rng.integers(0, 65536, n).astype(np.uint64)}
    slab = pktgen.gen_udp(P, n, {k: torch.from_numpy(v).cuda() for k, v in f.items()})
    got = slab.cpu().numpy().reshape(n, 64)
    for i in list(range(0, n, 997)) + [n - 1]:
        want = gen.create_udp_packet(T.mac(f["eth_dst"][i]), T.mac(f["eth_src"][i]), False, 10, 3, 5,
                                     T.ip4(f["ipv4_src"][i]), T.ip4(f["ipv4_dst"][i]), int(f["ipv4_diffserv"][i]),
                                     int(f["ipv4_ttl"][i]), int(f["ipv4_identification"][i]), 0x4000, [],
                                     int(f["udp_dst"][i]), int(f["udp_src"][i]), False, bytes(range(22))).to_vec()
        assert got[i].tobytes() == want, i
    r = oracle.parse_batch(got, n, stride=64)
    assert (r["status"] == 0).all()
    assert np.array_equal(r["ipv4_header_checksum"], r["ipv4_csum_calc"])
    assert np.array_equal(r["udp_dst"], f["udp_dst"].astype(np.uint16))


def test_reference_update_clone_loop(P):
    """tests/lib.rs:778-787: Ether etype = i % 0xFFFF on test_tcp_packet, cloned, to_vec — for
    1M packets, split over two runs (the counter continues through `first`)."""
    from pktgpu import pktgen
    tpl = pktgen.test_tcp_template()
    assert len(tpl) == 154
    n = 1 << 20
    G = pktgen.Generator(P, tpl, [pktgen.Field("Ether", "etype", kind="inc", count=0xFFFF)])
    a = G.run(n // 2, 160).cpu().numpy().reshape(-1, 160)
    b = G.run(n // 2, 160, first=n // 2).cpu().numpy().reshape(-1, 160)
    out = np.concatenate([a, b])
    et = (out[:, 12].astype(np.int64) << 8) | out[:, 13]
    assert np.array_equal(et, np.arange(n) % 0xFFFF)
    t = np.frombuffer(tpl, np.uint8)
    assert (out[:, :12] == t[:12]).all() and (out[:, 14:154] == t[14:]).all() and not out[:, 154:].any()


def test_clone_and_edge_fields(P):
    """No fields = n clones; fields that straddle 16-byte pieces at odd offsets (SNAP at 17),
    overlapping fields (later wins), 64-bit fields, RANDOM continuity across runs."""
    import torch
    from pktgpu import pktgen
    tpl = T.template_bytes("snap")
    n = 3000
    G0 = pktgen.Generator(P, tpl)
    c = G0.run(n, 32).cpu().numpy().reshape(n, 32)
    assert (c[:, :len(tpl)] == np.frombuffer(tpl, np.uint8)).all() and not c[:, len(tpl):].any()
    fs = [pktgen.Field("SNAP", (0, 39), kind="random", base=7),         # bytes 17..21: pieces 1
          pktgen.Field("Dot3", (40, 103), kind="random", base=9),       # 64 bits across bytes 5..12
          pktgen.Field("Dot3", (44, 47), kind="inc", base=3, step=5),   # overlaps the previous one
          pktgen.Field("LLC", (4, 19), kind="values")]                  # bytes 14..16 straddle
    v = torch.from_numpy(np.arange(n, dtype=np.uint64) * np.uint64(2654435761)).cuda()
    G = pktgen.Generator(P, tpl, fs)
    out = G.run(n, 32, values={3: v}, first=5).cpu().numpy().reshape(n, 32)
    g = np.arange(5, 5 + n, dtype=np.uint64)
    hv = [fs[0].value(g), fs[1].value(g), fs[2].value(g), fs[3].value(g, v.cpu().numpy())]
    want = T.oracle_batch(tpl, n, 32, [(f.hdr, f.occurrence, f.start, f.end) for f in fs], hv, [])
    assert np.array_equal(out, want)
    # the same packets from two runs with `first` continuing
    a = G.run(1000, 32, values={3: v}, first=5).cpu().numpy().reshape(1000, 32)
    b = G.run(n - 1000, 32, values={3: v[1000:]}, first=1005).cpu().numpy().reshape(n - 1000, 32)
    assert np.array_equal(np.concatenate([a, b]), out)


def test_generator_errors(P):
    import pktgpu
    from pktgpu import pktgen
    tpl = pktgen.udp_template()
    with pytest.raises(RuntimeError, match="header not in"):
        pktgen.Generator(P, tpl, [pktgen.Field("TCP", "src")])
    with pytest.raises(RuntimeError, match="bad generator field"):
        pktgen.Generator(P, tpl, [pktgen.Field("IPv6", "src")])  # 128-bit: split it into halves
    with pytest.raises(RuntimeError, match="checksum mask"):
        pktgen.Generator(P, tpl, csum=[1])
    with pytest.raises(RuntimeError, match="does not parse"):
        pktgen.Generator(P, tpl[:30])
    G = pktgen.Generator(P, tpl)
    with pytest.raises(RuntimeError, match="stride"):
        G.run(10, 48)
    with pytest.raises(RuntimeError, match="stride"):
        G.run(10, 72)
    with pytest.raises(RuntimeError, match="value array"):
        pktgen.Generator(P, tpl, [pktgen.Field("UDP", "src")]).run(10)
    assert isinstance(P, pktgpu.Parser)


def test_broadcast_clones_template(P):
    import torch
    from pktgpu import pktgen
    tpl = pktgen.udp_template()
    src = torch.from_numpy(np.frombuffer(tpl, np.uint8).copy()).cuda()
    out = P.broadcast(src, 1000, 80).cpu().numpy().reshape(1000, 80)
    want = np.zeros(80, np.uint8)
    want[:len(tpl)] = np.frombuffer(tpl, np.uint8)
    assert (out == want).all()


@pytest.mark.parametrize("name", ["erspan3", "vxlan_tcp", "snap"])
def test_wide_stride_takes_piece_kernel(P, name):
    """Strides over 1 KiB go through the lane-per-piece kernel (fields and checksum rebuilt per
    piece): same packets as the region kernel and the oracle."""
    import torch
    from pktgpu import pktgen
    tpl = T.template_bytes(name)
    n, first = 2000, 3
    gf, values, host_vals, csum, _ = T.make_case(name, n, first)
    G = pktgen.Generator(P, tpl, gf, csum=csum)
    dv = {j: torch.from_numpy(v).cuda() for j, v in values.items()}
    narrow = G.default_stride()
    a = G.run(n, narrow, values=dv, first=first).cpu().numpy().reshape(n, narrow)
    b = G.run(n, 1040, values=dv, first=first).cpu().numpy().reshape(n, 1040)
    assert np.array_equal(b[:, :narrow], a) and not b[:, narrow:].any()
    want = T.oracle_batch(tpl, n, narrow, [(f.hdr, f.occurrence, f.start, f.end) for f in gf], host_vals, csum)
    assert np.array_equal(a, want)
