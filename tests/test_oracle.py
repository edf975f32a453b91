"""CPU tests: pin the oracle (oracle/pkt_oracle.c) to the reference's own known answers.

Every assertion here is a value a reference test asserts (file:line cited), or a property the
reference's code fixes (quirks Q1-Q7 of SURVEY §8), or agreement with the independent Python
restatement tests/pyref.py.  No GPU is used.
"""
import json
import os

import numpy as np
import pytest

import oracle
import pyref
from pktgpu import gen, schema

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
KAT = json.load(open(os.path.join(GOLD, "kat_reference.json")))
H = schema.HDR_ID


def verify_ref(v):
    """tests/lib.rs:13-24 ipv4_checksum_verify (sums ALL words, same fold)."""
    s = 0
    for i in range(0, len(v), 2):
        s += (v[i] << 8) | v[i + 1]
    while s >> 16:
        s = ((s >> 16) + s) & 0xFFFF
    return (~s) & 0xFFFF


def one(pkt, entry="parse", columns=None):
    a = np.frombuffer(bytes(pkt), np.uint8) if len(pkt) else np.zeros(1, np.uint8)
    r = oracle.parse_batch(a, 1, stride=len(pkt), lens=np.array([len(pkt)], np.uint32),
                           entry=entry, columns=columns)
    return {k: v[..., 0] if k in ("hdr_type", "hdr_off") else v[0] for k, v in r.items()}


def chain(r):
    return [(schema.HDR_NAMES[r["hdr_type"][j]], int(r["hdr_off"][j])) for j in range(r["n_hdrs"])]


# ------------------------------------------------------------------ bit_range KATs
def test_tester_bit_extraction():
    """headers.rs:856-881 test_header_get."""
    t = KAT["tester"]
    b = bytes(t["bytes"])
    for name, (s, e, want) in t["fields"].items():
        assert oracle.bit_range(b, e, s) == want, name
    s, e, want = t["byte4_as_u32"]
    assert oracle.bit_range(b, e, s) & 0xFFFFFFFF == want
    s, e, want = t["byte16_bytes"]
    assert [oracle.bit_range(b, i + 7, i) for i in range(s, e + 1, 8)] == want


def test_bit_range_q8_release_semantics():
    """headers.rs:262 with a width > 64: the release build keeps the low (w mod 64 or 64) bits."""
    b = bytes(range(1, 41))
    low64 = int.from_bytes(b[8:16], "big")
    assert oracle.bit_range(b, 127, 0) == low64                    # w=128 -> shift 0
    w72 = pyref.bit_range_py(b, 0, 71) & (2**64 - 1)
    assert oracle.bit_range(b, 71, 0) == w72 & 0xFF                # w=72 -> shift 56


@pytest.mark.parametrize("case,hdr", [("ether_default", "Ether"), ("ether_from", "Ether"),
                                      ("vlan_default", "Vlan"), ("vlan_from", "Vlan"),
                                      ("arp_default", "ARP"), ("vxlan_default", "Vxlan")])
def test_header_kats(case, hdr):
    """tests/lib.rs:58-116, 139-149, 206-218 (getters on default / given bytes)."""
    k = KAT[case]
    b = bytes(k["bytes"])
    table = {n: (s, e) for n, s, e in oracle.field_table(H[hdr])}
    for f, want in k.items():
        if f == "bytes":
            continue
        s, e = table[f]
        assert oracle.bit_range(b, e, s) == want, (case, f)


def test_vxlan_builder():
    """tests/lib.rs:145-148: Packet::vxlan(2000) has flags 8, vni 2000."""
    v = gen.vxlan_hdr(2000).data
    t = {n: (s, e) for n, s, e in oracle.field_table(H["Vxlan"])}
    assert oracle.bit_range(v, t["flags"][1], t["flags"][0]) == 8
    assert oracle.bit_range(v, t["vni"][1], t["vni"][0]) == 2000


def test_field_tables_match_schema():
    for t in range(1, schema.HDR_SIZES.__len__()):
        ft = oracle.field_table(t)
        assert ft, t
        assert max(e for _, _, e in ft) < 8 * schema.HDR_SIZES[t]


# ------------------------------------------------------------------ checksum KATs
def test_ipv4_builder_checksum_verifies():
    """tests/lib.rs:130-131."""
    h = gen.ipv4(*KAT["ipv4_builder"]["args"]).data
    assert verify_ref(h) == 0
    assert oracle.ipv4_checksum(h) == int.from_bytes(h[10:12], "big")


def test_ipv4_checksum_sweep_25400():
    """tests/lib.rs:151-204: 10 src x 10 dst x ttl 1..254 — the oracle's checksum equals the
    builder's stored field, verifies to 0, and matches Packet::ipv4(5,0,115,ttl,0,6,..,140)."""
    payload = bytes(range(100))
    ips = [f"{k}.{k}.{k}.1" for k in range(10, 20)]
    n = 0
    for sip in ips:
        for dip in ips:
            for ttl in range(1, 255):
                pkt = gen.create_tcp_packet("00:01:02:03:04:05", "00:06:07:08:09:0a", False, 10, 3,
                                            5, sip, dip, 0, ttl, 115, 0, [], 80, 9090, 100, 101, 0,
                                            0, 1, 0, 0, False, payload)
                ip = pkt["IPv4"].data
                stored = int.from_bytes(ip[10:12], "big")
                assert oracle.ipv4_checksum(ip) == stored
                assert verify_ref(ip) == 0
                ip2 = gen.ipv4(5, 0, 115, ttl, 0, 6, sip, dip, 140).data
                assert int.from_bytes(ip2[10:12], "big") == stored
                n += 1
    assert n == 25400


def test_checksum_q1_fold():
    """packet.rs:102-104: ((s>>16)+s)&0xFFFF drops the end-around carry of hi+lo (Q1).
    Find headers where that differs from RFC 1071 and check the oracle takes the quirk."""
    rng = np.random.default_rng(7)
    hits = 0
    for _ in range(40000):
        h = rng.integers(0, 256, 20, dtype=np.uint8).tobytes()
        s = sum((h[i] << 8) | h[i + 1] for i in range(0, 20, 2) if i != 10)
        quirk = (~(((s >> 16) + s) & 0xFFFF)) & 0xFFFF
        rfc = s
        while rfc >> 16:
            rfc = (rfc >> 16) + (rfc & 0xFFFF)
        rfc = (~rfc) & 0xFFFF
        assert oracle.ipv4_checksum(h) == quirk
        hits += quirk != rfc
    assert hits > 0


# ------------------------------------------------------------------ walk KATs
def test_worked_example():
    """create_udp_packet(...) bytes and its parse."""
    k = KAT["worked_example"]
    p = gen.create_udp_packet("00:01:02:03:04:05", "00:06:07:08:09:0a", False, 10, 3, 5,
                              "192.168.0.199", "192.168.0.1", 0, 64, 0, 0x4000, [], 1234, 9090,
                              False, bytes(range(22))).to_vec()
    assert p.hex() == k["bytes_hex"]
    r = one(p)
    assert r["status"] == schema.OK
    assert [o for _, o in chain(r)] == k["hdr_offsets"]
    assert r["ipv4_header_checksum"] == k["ipv4_csum"] == r["ipv4_csum_calc"]
    assert (r["udp_src"], r["udp_dst"], r["udp_length"]) == (k["udp_src"], k["udp_dst"], k["udp_len"])
    assert (r["payload_off"], r["payload_len"]) == (k["payload_off"], k["payload_len"])


def test_reference_22_roundtrip():
    """tests/lib.rs:674-679: slow::parse(bytes).compare(pkt) for the 22 packets."""
    for name, p in zip(gen.REFERENCE_22_NAMES, gen.reference_22_packets()):
        v = p.to_vec()
        assert oracle.slow_parse_to_vec(v) == v, name


def test_reference_22_golden_chains():
    exp = json.load(open(os.path.join(GOLD, "ref22_expected.json")))
    pc = open(os.path.join(GOLD, "ref22.pcap"), "rb").read()
    offs, lens = gen.pcap_index_py(pc)
    r = oracle.parse_batch(np.frombuffer(pc, np.uint8), len(exp), offsets=offs, lens=lens)
    for i, e in enumerate(exp):
        assert schema.STATUS_NAMES[r["status"][i]] == e["status"]
        got = [[schema.HDR_NAMES[r["hdr_type"][j, i]], int(r["hdr_off"][j, i])]
               for j in range(r["n_hdrs"][i])]
        assert got == e["hdrs"], e["name"]
        assert (r["payload_off"][i], r["payload_len"][i]) == (e["payload_off"], e["payload_len"])


def test_golden_pcap_is_reproducible():
    pkts = [p.to_vec() for p in gen.reference_22_packets()]
    assert gen.pcap_bytes(pkts) == open(os.path.join(GOLD, "ref22.pcap"), "rb").read()


@pytest.mark.parametrize("entry", ["parse", "parse_ethernet"])
def test_payload_extraction(entry):
    """tests/lib.rs:818-837: fast/slow parse payload() == the 10-byte payload."""
    pl = bytes(KAT["payload_test"]["payload"])
    v = gen.test_tcp_packet_with_payload(pl).to_vec()
    r = one(v, entry)
    assert v[r["payload_off"]:r["payload_off"] + r["payload_len"]] == pl
    assert oracle.slow_parse_to_vec(v).endswith(pl)


# ------------------------------------------------------------------ quirks
def test_q2_gre_option_order_and_to_vec_reorder():
    """fast.rs:154-163: list is GRE, SeqNum, Key, ChksumOffset; to_vec reorders the bytes."""
    inner = gen.create_udp_packet("00:01:02:03:04:05", "00:06:07:08:09:0a", False, 0, 0, 5,
                                  "1.1.1.1", "2.2.2.2", 0, 64, 0, 0, [], 53, 1000, False, b"x" * 8)
    inner.remove(0)
    p = gen.create_gre_packet("00:01:02:03:04:05", "00:06:07:08:09:0a", False, 0, 0, 5, "3.3.3.3",
                              "4.4.4.4", 0, 64, 0, 0, [], 1, 0, 1, 1, 0, 0, 0, 0x1111, 0x2222,
                              0x33333333, 0x44444444, b"", inner).to_vec()
    r = one(p)
    assert chain(r) == [("Ether", 0), ("IPv4", 14), ("GRE", 34), ("GRESequenceNum", 46),
                        ("GREKey", 42), ("GREChksumOffset", 38), ("IPv4", 50), ("UDP", 70)]
    rt = oracle.slow_parse_to_vec(p)
    assert len(rt) == len(p) and rt != p
    assert rt[38:42] == p[46:50] and rt[46:50] == p[38:42]


def test_q3_mpls_bos_consumes_next_label():
    """fast.rs:63-83."""
    eth = gen.ethernet("00:00:00:00:00:01", "00:00:00:00:00:02", 0x8847).data
    l1 = gen.mpls_raw(100, 0, 0, 64).data
    l2 = gen.mpls_raw(200, 0, 1, 64).data
    ip = gen.ipv4(5, 0, 1, 64, 0, 17, "1.1.1.1", "2.2.2.2", 28).data
    extra = bytes([0x12, 0x34, 0x56, 0x78])
    udp = gen.udp(1, 2, 8).data
    # after the bos label, 4 more bytes are taken as MPLS, then arr[4]>>4 picks the parser
    p = eth + l1 + l2 + extra + ip + udp
    r = one(p)
    assert chain(r)[:4] == [("Ether", 0), ("MPLS", 14), ("MPLS", 18), ("MPLS", 22)]
    # high nibble of ip[0] = 4 -> IPv4 at 26
    assert chain(r)[4:] == [("IPv4", 26), ("UDP", 46)]
    # nibble not 4/6 -> Ethernet
    p2 = eth + l2 + extra + gen.ethernet("00:00:00:00:00:03", "00:00:00:00:00:04", 0x1234).data
    assert chain(one(p2)) == [("Ether", 0), ("MPLS", 14), ("MPLS", 18), ("Ether", 22)]
    # bos with nothing after the extra 4 bytes: arr[4] panics
    assert one(eth + l2 + extra)["status"] == schema.TRUNCATED


def test_q4_ihl_and_tcp_offset_ignored():
    ip = bytearray(gen.ipv4(6, 0, 1, 64, 0, 6, "1.1.1.1", "2.2.2.2", 44).data)
    p = gen.ethernet("00:00:00:00:00:01", "00:00:00:00:00:02", 0x0800).data + bytes(ip) + \
        gen.tcp(1, 2, 3, 4, 15, 0, 0, 0, 0, 0).data + bytes(4)
    r = one(p)
    assert chain(r) == [("Ether", 0), ("IPv4", 14), ("TCP", 34)]
    assert r["ipv4_ihl"] == 6 and r["tcp_data_startset"] == 15 and r["payload_off"] == 54


def test_q5_dot3_and_unknown_etypes():
    p = bytes(12) + bytes([0x05, 0xDB]) + bytes([0xAA, 0xAA, 0x03]) + bytes(5) + b"pl"
    assert chain(one(p)) == [("Dot3", 0), ("LLC", 14), ("SNAP", 17)]
    p = bytes(12) + bytes([0x05, 0xDC]) + bytes(20)  # 1500 -> Ethernet, unknown etype
    r = one(p)
    assert chain(r) == [("Ether", 0)] and r["payload_off"] == 14
    for et in (0x88A8, 0x88BE, 0x22EB):  # QinQ, ERSPAN types: payload after Ether (Q5)
        p = bytes(12) + et.to_bytes(2, "big") + bytes(30)
        assert chain(one(p)) == [("Ether", 0)]


def test_q6_protocol_maps():
    e4 = gen.ethernet("00:00:00:00:00:01", "00:00:00:00:00:02", 0x0800).data
    e6 = gen.ethernet("00:00:00:00:00:01", "00:00:00:00:00:02", 0x86DD).data
    ip58 = gen.ipv4(5, 0, 1, 64, 0, 58, "1.1.1.1", "2.2.2.2", 24).data
    assert chain(one(e4 + ip58 + bytes(4))) == [("Ether", 0), ("IPv4", 14)]
    ip6_1 = gen.ipv6(0, 0, 1, 64, "::1", "::2", 4).data
    assert chain(one(e6 + ip6_1 + bytes(4))) == [("Ether", 0), ("IPv6", 14)]
    ip6_58 = gen.ipv6(0, 0, 58, 64, "::1", "::2", 4).data
    assert chain(one(e6 + ip6_58 + bytes(4))) == [("Ether", 0), ("IPv6", 14), ("ICMP", 54)]
    # UDP *source* 4789 does not trigger VXLAN, destination does
    u = gen.udp(4789, 53, 8).data
    ip = gen.ipv4(5, 0, 1, 64, 0, 17, "1.1.1.1", "2.2.2.2", 28).data
    assert chain(one(e4 + ip + u)) == [("Ether", 0), ("IPv4", 14), ("UDP", 34)]


def test_q7_truncation_at_every_length():
    """Every prefix of every template either parses like pyref or is TRUNCATED where pyref
    (= the reference's slice indexing) panics."""
    for p in gen.reference_22_packets():
        v = p.to_vec()
        for L in range(0, min(len(v), 140) + 1):
            st, hdrs, po, pl = pyref.parse(v[:L])
            r = one(v[:L])
            assert schema.STATUS_NAMES[r["status"]] == st
            if st == "OK":
                assert chain(r) == [tuple(h) for h in hdrs]
                assert (r["payload_off"], r["payload_len"]) == (po, pl)
            else:
                assert r["n_hdrs"] == 0 and r["hdr_mask"] == 0 and r["payload_len"] == 0


def test_depth_limit():
    eth = gen.ethernet("00:00:00:00:00:01", "00:00:00:00:00:02", 0x8100).data
    tag = gen.vlan(0, 0, 5, 0x8100).data
    last = gen.vlan(0, 0, 5, 0x0800).data
    ip = gen.ipv4(5, 0, 1, 64, 0, 99, "1.1.1.1", "2.2.2.2", 20).data
    p14 = eth + tag * 13 + last + ip  # 1 + 14 + 1 = 16 headers: fits
    r = one(p14)
    assert r["status"] == schema.OK and r["n_hdrs"] == 16
    p15 = eth + tag * 14 + last + ip  # 17 headers
    assert one(p15)["status"] == schema.DEPTH_LIMIT
    # the 17th header truncated: its bounds check comes first -> TRUNCATED
    assert one(p15[:-1])["status"] == schema.TRUNCATED
    # the 17th header fits but a later one is truncated: depth is hit first (forward order)
    assert one(eth + tag * 15 + last + ip[:-1])["status"] == schema.DEPTH_LIMIT
    assert one(eth + tag * 3)["status"] == schema.TRUNCATED


@pytest.mark.parametrize("entry", schema.ENTRIES)
def test_entries_vs_pyref(entry):
    rng = np.random.default_rng(schema.ENTRY_ID[entry])
    pkts = [p.to_vec() for p in gen.reference_22_packets()]
    cases = pkts + [rng.integers(0, 256, int(rng.integers(0, 120)), dtype=np.uint8).tobytes()
                    for _ in range(200)]
    for v in cases:
        st, hdrs, po, pl = pyref.parse(v, entry)
        r = one(v, entry)
        assert schema.STATUS_NAMES[r["status"]] == st
        if st == "OK":
            assert chain(r) == [tuple(h) for h in hdrs]
            assert (r["payload_off"], r["payload_len"]) == (po, pl)


def test_fuzz_mutated_templates_vs_pyref():
    """Byte-level mutations of the 22 templates (hits every dispatch arm)."""
    rng = np.random.default_rng(11)
    pkts = [p.to_vec() for p in gen.reference_22_packets()]
    keys = [12, 13, 14 + 9, 14 + 6, 36, 37, 38, 34, 35, 16, 45]
    for _ in range(3000):
        v = bytearray(pkts[int(rng.integers(0, len(pkts)))])
        for _ in range(int(rng.integers(1, 4))):
            k = int(rng.choice(keys)) if rng.random() < 0.6 else int(rng.integers(0, len(v)))
            if k < len(v):
                v[k] = int(rng.choice([0x00, 0x01, 0x04, 0x06, 0x08, 0x11, 0x29, 0x2F, 0x3A, 0x81,
                                       0x86, 0x88, 0xAA, 0xDD, 0xBE, 0x22, 0xEB, 0x12, 0xB5,
                                       int(rng.integers(0, 256))]))
        v = bytes(v[:int(rng.integers(max(0, len(v) - 40), len(v) + 1))])
        st, hdrs, po, pl = pyref.parse(v)
        r = one(v)
        assert schema.STATUS_NAMES[r["status"]] == st
        if st == "OK":
            assert chain(r) == [tuple(h) for h in hdrs]
            assert (r["payload_off"], r["payload_len"]) == (po, pl)


def test_fields_vs_pyref_getters():
    """Field columns of the first header of each type == the make_header! getters."""
    rng = np.random.default_rng(5)
    slab = gen.gen_c3(512, seed=99)
    r = oracle.parse_batch(slab, 512, stride=128)
    for i in range(512):
        v = slab[i].tobytes()
        st, hdrs, _, _ = pyref.parse(v)
        first = {}
        for name, o in hdrs:
            first.setdefault(name, o)
        o = first["IPv4"]
        assert r["ipv4_src"][i] == pyref.bit_range_py(v[o:], 96, 127)
        assert r["ipv4_csum_calc"][i] == gen.ipv4_checksum(v[o:o + 20])
        if "TCP" in first:
            o = first["TCP"]
            assert r["tcp_seq_no"][i] == pyref.bit_range_py(v[o:], 32, 63)
            assert r["tcp_flags"][i] == v[o + 13]
            assert r["udp_src"][i] == 0
        if "Vlan" in first:
            o = first["Vlan"]
            assert r["vlan_vid"][i] == pyref.bit_range_py(v[o:], 4, 15)
    del rng


def test_extract_fields_oracle():
    pc = open(os.path.join(GOLD, "ref22.pcap"), "rb").read()
    offs, lens = gen.pcap_index_py(pc)
    slab = np.frombuffer(pc, np.uint8)
    r = oracle.parse_batch(slab, 22, offsets=offs, lens=lens)
    specs = [(H["Vxlan"], 0, 32, 55), (H["IPv4"], 1, 96, 127), (H["ERSPAN3"], 0, 95, 95),
             (H["IPv6"], 0, 64, 191)]
    vals, found = oracle.extract_fields(slab, 22, r, specs, offsets=offs, lens=lens)
    names = gen.REFERENCE_22_NAMES
    assert vals[0][names.index("vxlan_udp")] == 2000 and found[0][names.index("tcp")] == 0
    assert vals[1][names.index("ip4ip4")] == int.from_bytes(bytes([10, 10, 10, 1]), "big")
    assert vals[2][names.index("erspan3")] == 1
    # IPv6 src "AAAA::1": Q8 low 64 bits of the 128-bit field
    assert vals[3][names.index("tcpv6")] == 1


def test_multithreaded_oracle_matches_single():
    slab = gen.gen_c2(4096, seed=3)
    a = oracle.parse_batch(slab, 4096, stride=64, nthreads=1)
    b = oracle.parse_batch(slab, 4096, stride=64, nthreads=4)
    for k in a:
        assert np.array_equal(a[k], b[k]), k
