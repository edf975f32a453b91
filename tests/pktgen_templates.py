"""The 22 create_packet_test templates (tests/lib.rs:220-671) as generator cases: for each, the
builder arguments that vary, the header field each one lands in (headers.rs:529-827 tables), the
IPv4 checksums the builder computes (utils.rs:233-236), and the builder itself (pktgpu/gen.py's
restatement of utils.rs:7-876).  Shared by tests/test_pktgen.py (GPU) and
tests/test_pktgen_model.py (CPU: the case tables against the builders and the oracle)."""
import ipaddress

import numpy as np

import oracle
from pktgpu import gen

PAYLOAD = bytes(range(100))
M1, M2 = "00:01:02:03:04:05", "00:06:07:08:09:0a"


def mac(x):
    return ":".join(f"{(int(x) >> (40 - 8 * k)) & 0xFF:02x}" for k in range(6))


def ip4(x):
    return ".".join(str((int(x) >> (24 - 8 * k)) & 0xFF) for k in range(4))


def ip6(hi, lo):
    return str(ipaddress.IPv6Address((int(hi) << 64) | int(lo)))


# ---- builder-argument maps: (arg, header, field, occurrence, value range) and the builder
ETH = [("ed", "Ether", "dst", 0, 1 << 48), ("es", "Ether", "src", 0, 1 << 48)]
IP4 = [("is", "IPv4", "src", 0, 1 << 32), ("id", "IPv4", "dst", 0, 1 << 32), ("tos", "IPv4", "diffserv", 0, 256),
       ("ttl", "IPv4", "ttl", 0, 256), ("ipid", "IPv4", "identification", 0, 1 << 16)]
IP6 = [("tc", "IPv6", "traffic_class", 0, 256), ("fl", "IPv6", "flow_label", 0, 1 << 20),
       ("hl", "IPv6", "hop_limit", 0, 256), ("sh", "IPv6", (64, 127), 0, 1 << 64),
       ("sl", "IPv6", (128, 191), 0, 1 << 64), ("dh", "IPv6", (192, 255), 0, 1 << 64),
       ("dl", "IPv6", (256, 319), 0, 1 << 64)]


def l4(hdr, occ=0):
    return [("dp", hdr, "dst", occ, 1 << 16), ("sp", hdr, "src", occ, 1 << 16)]


def occ1(fields):
    return [(a + "1", h, f, o + 1, r) for a, h, f, o, r in fields]


def _tcp(v, ed=None, es=None):
    return gen.create_tcp_packet(mac(v.get("ed", 0x000102030405)) if ed is None else ed,
                                 mac(v.get("es", 0x00060708090A)) if es is None else es, False, 10, 3, 5,
                                 ip4(v["is"]), ip4(v["id"]), v["tos"], v["ttl"], v["ipid"], 0, [], v["dp"], v["sp"],
                                 v.get("seq", 100), v.get("ack", 101), 5, 0, 0x10, 2, 0, False, PAYLOAD)


def _udp(v, sfx=""):
    g = lambda k, d: v.get(k + sfx, d)  # noqa: E731
    return gen.create_udp_packet(mac(g("ed", 0x000102030405)), mac(g("es", 0x00060708090A)), False, 10, 3, 5,
                                 ip4(g("is", 0xC0A800C7)), ip4(g("id", 0xC0A80001)), g("tos", 0), g("ttl", 64),
                                 g("ipid", 0), 0x4000, [], g("dp", 1234), g("sp", 9090), False, PAYLOAD)


def _v6(v, builder, *tail):
    return builder(mac(v.get("ed", 0x000102030405)), mac(v.get("es", 0x00060708090A)), False, 10, 3,
                   v.get("tc", 5), v.get("fl", 4), v.get("hl", 64),
                   ip6(v.get("sh", 0xAAAA << 48), v.get("sl", 1)), ip6(v.get("dh", 0xBBBB << 48), v.get("dl", 1)), *tail)


def _ip4_outer(v, builder, *tail):
    return builder(mac(v.get("ed", 0x000102030405)), mac(v.get("es", 0x00060708090A)), False, 10, 3, 5,
                   ip4(v.get("is", 0xC0A800C7)), ip4(v.get("id", 0xC0A80001)), v.get("tos", 0), v.get("ttl", 64),
                   v.get("ipid", 0), 0x4000, [], *tail)


def _strip(p):
    p = p.clone()
    p.remove(0)
    return p


def _udpv6(v, sfx=""):
    w = {k[:-len(sfx)]: x for k, x in v.items() if k.endswith(sfx)} if sfx else v
    return _v6(w, gen.create_udpv6_packet, w.get("dp", 1234), w.get("sp", 9090), False, PAYLOAD)


def _llc(v, snap):
    p = gen.Packet()
    d = bytearray([0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 0x0, 86])
    d[0:6] = int(v["ed"]).to_bytes(6, "big")
    d[6:12] = int(v["es"]).to_bytes(6, "big")
    p.push(gen.Hdr("Dot3", bytes(d)))
    if snap:
        p.push(gen.Hdr("LLC", bytes([0xAA, 0xAA, 0x03])))
        p.push(gen.Hdr("SNAP", int(v["oui"]).to_bytes(3, "big") + int(v["code"]).to_bytes(2, "big")))
    else:
        p.push(gen.Hdr("LLC", bytes([0x0, 0x04, 0x0])))
    return p


TCP_EXTRA = [("seq", "TCP", "seq_no", 0, 1 << 32), ("ack", "TCP", "ack_no", 0, 1 << 32)]
DOT3 = [("ed", "Dot3", "dst", 0, 1 << 48), ("es", "Dot3", "src", 0, 1 << 48)]
ARP = ETH + [("op", "ARP", "opcode", 0, 1 << 16), ("smac", "ARP", "sender_hw_addr", 0, 1 << 48),
             ("sip", "ARP", "sender_proto_addr", 0, 1 << 32), ("tmac", "ARP", "target_hw_addr", 0, 1 << 48),
             ("tip", "ARP", "target_proto_addr", 0, 1 << 32)]
VX = [("sp", "UDP", "src", 0, 1 << 16), ("vni", "Vxlan", "vni", 0, 1 << 24)]
INNER_UDP4 = [("ed1", "Ether", "dst", 1, 1 << 48), ("is1", "IPv4", "src", 1, 1 << 32), ("ttl1", "IPv4", "ttl", 1, 256),
              ("dp1", "UDP", "dst", 1, 1 << 16), ("sp1", "UDP", "src", 1, 1 << 16)]
INNER_TCP4 = [("ed1", "Ether", "dst", 1, 1 << 48), ("is1", "IPv4", "src", 1, 1 << 32), ("ttl1", "IPv4", "ttl", 1, 256),
              ("dp1", "TCP", "dst", 0, 1 << 16), ("sp1", "TCP", "src", 0, 1 << 16)]
ER2 = [("sq", "GRESequenceNum", "seqnum", 0, 1 << 32), ("evlan", "ERSPAN2", "vlan", 0, 1 << 12),
       ("cos", "ERSPAN2", "cos", 0, 8), ("sid", "ERSPAN2", "session_id", 0, 1 << 10),
       ("idx", "ERSPAN2", "index", 0, 1 << 20)]
ER3 = [("evlan", "ERSPAN3", "vlan", 0, 1 << 12), ("sid", "ERSPAN3", "session_id", 0, 1 << 10),
       ("ts", "ERSPAN3", "timestamp", 0, 1 << 32), ("sgt", "ERSPAN3", "sgt", 0, 1 << 16),
       ("pinfo", "ERSPANPLATFORM", "info", 0, 1 << 58)]


def _vxlan_inner_udp(v):
    inner = {"ed": v["ed1"], "is": v["is1"], "ttl": v["ttl1"], "dp": v["dp1"], "sp": v["sp1"]}
    return _udp(inner)


def _vxlan_inner_tcp(v):
    return _tcp({"ed": v["ed1"], "is": v["is1"], "id": 0x0B0B0B01, "tos": 0, "ttl": v["ttl1"], "ipid": 115,
                 "dp": v["dp1"], "sp": v["sp1"]})


# name -> (fields, ipv4 checksum occurrences refreshed, builder(v) -> Packet)
TEMPLATES = {
    "tcp": (ETH + IP4 + l4("TCP") + TCP_EXTRA, [0], lambda v: _tcp(v)),
    "udp": (ETH + IP4 + l4("UDP"), [0], lambda v: _udp(v)),
    "icmp": (ETH + IP4 + [("it", "ICMP", "icmp_type", 0, 256), ("ic", "ICMP", "icmp_code", 0, 256)], [0],
             lambda v: _ip4_outer(v, gen.create_icmp_packet, v["it"], v["ic"], [], False, PAYLOAD)),
    "tcpv6": (ETH + IP6 + l4("TCP") + TCP_EXTRA, [],
              lambda v: _v6(v, gen.create_tcpv6_packet, v["dp"], v["sp"], v["seq"], v["ack"], 5, 0, 1, 0, 0, PAYLOAD)),
    "udpv6": (ETH + IP6 + l4("UDP"), [], lambda v: _udpv6(v)),
    "icmpv6": (ETH + IP6 + [("it", "ICMP", "icmp_type", 0, 256), ("ic", "ICMP", "icmp_code", 0, 256)], [],
               lambda v: _v6(v, gen.create_icmpv6_packet, v["it"], v["ic"], [], False, PAYLOAD)),
    # outer IPv4 checksum is stale by construction (Q9, utils.rs:542-543): outer IPv4 not varied
    "vxlan_udp": (ETH + VX + INNER_UDP4, [1],
                  lambda v: _ip4_outer(v, gen.create_vxlan_packet, gen.VXLAN_PORT, v["sp"], False, v["vni"],
                                       _vxlan_inner_udp(v))),
    # Q12: the inner packet is emitted twice, so only outer fields vary
    "vxlanv6_udp": (ETH + IP6 + VX, [],
                    lambda v: _v6(v, gen.create_vxlanv6_packet, gen.VXLAN_PORT, v["sp"], False, v["vni"],
                                  _udp({}))),
    "vxlan_tcp": (ETH + VX + INNER_TCP4, [1],
                  lambda v: _ip4_outer(v, gen.create_vxlan_packet, gen.VXLAN_PORT, v["sp"], False, v["vni"],
                                       _vxlan_inner_tcp(v))),
    "vxlanv6_tcp": (ETH + IP6 + VX, [],
                    lambda v: _v6(v, gen.create_vxlanv6_packet, gen.VXLAN_PORT, v["sp"], False, v["vni"],
                                  _tcp({"is": 0x0A0A0A01, "id": 0x0B0B0B01, "tos": 0, "ttl": 64, "ipid": 115,
                                        "dp": 1234, "sp": 9090}))),
    "arp_req": (ARP, [], lambda v: gen.create_arp_packet(mac(v["ed"]), mac(v["es"]), False, 10, 3, v["op"],
                                                         mac(v["smac"]), mac(v["tmac"]), ip4(v["sip"]), ip4(v["tip"]),
                                                         PAYLOAD)),
    "arp_resp": (ARP, [], lambda v: gen.create_arp_packet(mac(v["ed"]), mac(v["es"]), False, 10, 3, v["op"],
                                                          mac(v["smac"]), mac(v["tmac"]), ip4(v["sip"]), ip4(v["tip"]),
                                                          PAYLOAD)),
    "ip4ip4": (ETH + IP4 + occ1([f for f in IP4 if f[0] in ("is", "ttl")]) + l4("TCP"), [0, 1],
               lambda v: _ip4_outer(v, gen.create_ipv4ip_packet,
                                    _strip(_tcp({"is": v["is1"], "id": 0x0B0B0B01, "tos": 0, "ttl": v["ttl1"],
                                                 "ipid": 115, "dp": v["dp"], "sp": v["sp"]})))),
    "ip4ip6": (ETH + IP4 + [f for f in IP6 if f[0] in ("hl", "sl", "dh")] + l4("UDP"), [0],
               lambda v: _ip4_outer(v, gen.create_ipv4ip_packet,
                                    _strip(_udpv6({"hl": v["hl"], "sl": v["sl"], "dh": v["dh"], "dp": v["dp"],
                                                   "sp": v["sp"]})))),
    "ip6ip4": (ETH + IP6 + [("is1", "IPv4", "src", 0, 1 << 32), ("ttl1", "IPv4", "ttl", 0, 256)] + l4("UDP"), [0],
               lambda v: _v6(v, gen.create_ipv6ip_packet,
                             _strip(_udp({"is": v["is1"], "ttl": v["ttl1"], "dp": v["dp"], "sp": v["sp"]})))),
    "ip6ip6": (ETH + IP6 + [("hl1", "IPv6", "hop_limit", 1, 256), ("sl1", "IPv6", (128, 191), 1, 1 << 64)] + l4("TCP"),
               [], lambda v: _v6(v, gen.create_ipv6ip_packet,
                                 _strip(_v6({"hl": v["hl1"], "sl": v["sl1"]}, gen.create_tcpv6_packet, v["dp"], v["sp"],
                                            100, 101, 5, 0, 1, 0, 0, PAYLOAD)))),
    "llc": (DOT3, [], lambda v: _llc(v, False)),
    "snap": (DOT3 + [("oui", "SNAP", "oui", 0, 1 << 24), ("code", "SNAP", "code", 0, 1 << 16)], [],
             lambda v: _llc(v, True)),
    "greip4": (ETH + IP4 + occ1([f for f in IP4 if f[0] in ("is", "ttl")]) + l4("TCP"), [0, 1],
               lambda v: _ip4_outer(v, gen.create_gre_packet, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, b"",
                                    _strip(_tcp({"is": v["is1"], "id": 0x0B0B0B01, "tos": 0, "ttl": v["ttl1"],
                                                 "ipid": 115, "dp": v["dp"], "sp": v["sp"]})))),
    "greip6": (ETH + IP4 + [f for f in IP6 if f[0] in ("hl", "sh", "dl")] + l4("UDP"), [0],
               lambda v: _ip4_outer(v, gen.create_gre_packet, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, b"",
                                    _strip(_udpv6({"hl": v["hl"], "sh": v["sh"], "dl": v["dl"], "dp": v["dp"],
                                                   "sp": v["sp"]})))),
    "erspan2": (ETH + IP4 + ER2 + [("hl", "IPv6", "hop_limit", 0, 256)] + l4("UDP"), [0],
                lambda v: _ip4_outer(v, gen.create_erspan_2_packet, v["sq"], v["evlan"], v["cos"], 1, 0,
                                     v["sid"], v["idx"],
                                     _udpv6({"hl": v["hl"], "dp": v["dp"], "sp": v["sp"]}))),
    # Q12 again (inner ICMP packet twice): outer fields only
    "erspan3": (ETH + IP4 + ER3, [0],
                lambda v: _ip4_outer(v, gen.create_erspan_3_packet, 23, v["evlan"], 0, 1, 0, v["sid"], v["ts"],
                                     v["sgt"], 1, 4, v["pinfo"],
                                     _ip4_outer({}, gen.create_icmp_packet, 8, 0, [], False, PAYLOAD))),
}
assert list(TEMPLATES) == gen.REFERENCE_22_NAMES


def template_bytes(name):
    """The template = the builder with its reference_22 arguments (defaults of the lambdas)."""
    return gen.reference_22_packets()[gen.REFERENCE_22_NAMES.index(name)].to_vec()


def oracle_batch(tpl, n, stride, specs, values, csum):
    """clone + set_bit_range per field + checksum refresh, on the CPU oracle."""
    slab = np.zeros((n, stride), np.uint8)
    slab[:, :len(tpl)] = np.frombuffer(tpl, np.uint8)
    slab = slab.reshape(-1)
    lens = np.full(n, len(tpl), np.uint32)
    chain = oracle.parse_batch(slab, n, stride=stride, lens=lens, columns=["status", "n_hdrs", "hdr_type", "hdr_off"])
    assert (chain["status"] == 0).all()
    oracle.set_fields(slab, n, chain, specs, values, stride=stride, lens=lens)
    for occ in csum:
        oracle.ipv4_update_checksum(slab, n, chain, occ, stride=stride, lens=lens)
    return slab.reshape(n, stride)




def make_case(name, n, first, seed=None):
    """Generator fields (pktgpu.pktgen.Field) of template `name` with kinds cycling through
    values / inc / random, the per-field "values" arrays, and every field's host value per packet."""
    from pktgpu import pktgen
    fields, csum, build = TEMPLATES[name]
    rng = np.random.default_rng(sum(map(ord, name)) if seed is None else seed)
    kinds = ["values", "inc", "random"]
    gf, values, host_vals = [], {}, []
    g = np.arange(first, first + n, dtype=np.uint64)
    for j, (arg, hdr, fld, occ, hi) in enumerate(fields):
        kind = "values" if arg == "sq" else kinds[(j + len(name)) % 3]  # seqnum must stay nonzero
        f = pktgen.Field(hdr, fld, occ, kind=kind, base=int(rng.integers(0, 2**62)), step=int(rng.integers(1, 2**20)),
                         count=int(rng.integers(0, 3000)))
        if kind == "values":
            v = rng.integers(1 if arg == "sq" else 0, hi, n, dtype=np.uint64) if hi < 2**64 else \
                rng.integers(0, 2**63, n, dtype=np.uint64) * np.uint64(2) + rng.integers(0, 2, n, dtype=np.uint64)
            values[j] = v
            hv = f.value(g, v)
        else:
            hv = f.value(g)
        gf.append(f)
        host_vals.append(hv)
    return gf, values, host_vals, csum, build


def builder_args(name, host_vals, i):
    return {arg: int(host_vals[j][i]) for j, (arg, *_r) in enumerate(TEMPLATES[name][0])}
