"""Workload generation: the reference's packet builders and the synthetic slabs.

This module produces INPUT bytes only (it parses nothing).  Two parts:

1. A restatement of packet_rs's builders so the parity fixtures have exactly the bytes the
   reference's tests construct: `Packet::ethernet … snap` (src/packet.rs:405-643), the
   `utils::create_*_packet` generators (src/utils.rs:7-876) and `Packet::to_vec`
   (packet.rs:385-392).  Their quirks are kept: `udp_dst, udp_src` argument order
   (utils.rs:211-212), the stale VXLAN IPv4 checksum (utils.rs:542-543), the duplicated
   inner packet of the vxlanv6/erspan3 builders (Q12, utils.rs:582+594, 837+871),
   `set_payload` appending (packet.rs:178-181) and `set_seqnum_present(gre_seqnum)` writing
   the low bit of the sequence number (utils.rs:846).
2. Vectorised numpy generators for the benchmark configs of BASELINE.json (C2: Ether/IPv4/UDP
   64 B, C3: Ether/{0-2}xVlan/IPv4/TCP|UDP 128 B, C4: pcap replay of the 22 templates of
   tests/lib.rs:220-671), seeded so every run sees the same bytes.
"""
import ipaddress
import struct

import numpy as np

VXLAN_PORT = 4789

# --------------------------------------------------------------------------- string parsers
# packet.rs:19-58 (ConvertToBytes): parse failures print and yield 0 for that octet.


def to_mac_bytes(s):
    out = [0] * 6
    for i, v in enumerate(s.split(":")):
        try:
            out[i] = int(v, 16)
            if out[i] > 255:
                out[i] = 0
        except ValueError:
            out[i] = 0
    return bytes(out)


def to_ipv4_bytes(s):
    out = [0] * 4
    for i, v in enumerate(s.split(".")):
        try:
            x = int(v, 10)
            out[i] = x if x <= 255 else 0
        except ValueError:
            out[i] = 0
    return bytes(out)


def to_ipv6_bytes(s):
    try:
        return ipaddress.IPv6Address(s).packed
    except ValueError:
        return bytes(16)


def ipv4_checksum(v):
    """Packet::ipv4_checksum (packet.rs:93-107) — generator-side copy for building packets."""
    s = 0
    for i in range(0, len(v), 2):
        if i == 10:
            continue
        s += (v[i] << 8) | v[i + 1]
    while s >> 16:
        s = ((s >> 16) + s) & 0xFFFF
    return (~s) & 0xFFFF


# --------------------------------------------------------------------------- Packet model
class Hdr:
    """An owned header: name + bytes (make_header! owned half, headers.rs:297-511)."""

    __slots__ = ("name", "data")

    def __init__(self, name, data):
        self.name = name
        self.data = bytearray(data)

    def set_bits(self, start, end, value):
        # set_bit_range (headers.rs:315-324): LSB of value into bit `end`, walking upwards.
        for i in range(end, start - 1, -1):
            byte, bit = i // 8, 7 - i % 8
            self.data[byte] = (self.data[byte] & ~(1 << bit)) | ((value & 1) << bit)
            value >>= 1

    def get_bits(self, start, end):
        v = 0
        for i in range(start, end + 1):
            v = (v << 1) | ((self.data[i // 8] >> (7 - i % 8)) & 1)
        return v


class Packet:
    """packet_rs::Packet (lib.rs:129-134): ordered owned headers + payload."""

    def __init__(self):
        self.hdrs = []
        self.payload = bytearray()

    def push(self, h):
        self.hdrs.append(h)

    def remove(self, idx):
        if self.hdrs and idx < len(self.hdrs):
            del self.hdrs[idx]

    def set_payload(self, b):  # packet.rs:178-181 appends
        self.payload.extend(b)

    def __getitem__(self, name):  # packet.rs:61-67, first match
        for h in self.hdrs:
            if h.name == name:
                return h
        raise KeyError(name)

    def clone(self):  # clone_me (packet.rs:393-400); byte copies suffice here
        p = Packet()
        p.hdrs = [Hdr(h.name, h.data) for h in self.hdrs]
        p.payload = bytearray(self.payload)
        return p

    def __add__(self, other):  # packet.rs:75-84: other's headers appended, payload dropped
        self.hdrs.extend(Hdr(h.name, h.data) for h in other.hdrs)
        return self

    def to_vec(self):  # packet.rs:385-392
        out = bytearray()
        for h in self.hdrs:
            out += h.data
        out += self.payload
        return bytes(out)


# --------------------------------------------------------------------------- header builders
def ethernet(dst, src, etype):  # packet.rs:405-412
    return Hdr("Ether", to_mac_bytes(dst) + to_mac_bytes(src) + struct.pack(">H", etype))


def vlan(pcp, _cfi, vid, etype):  # packet.rs:447-454 (cfi ignored)
    d = bytearray(struct.pack(">H", vid & 0xFFFF))
    d[0] = (d[0] | (pcp << 5)) & 0xFF
    return Hdr("Vlan", bytes(d) + struct.pack(">H", etype))


def arp(opcode, sender_mac, target_mac, sender_ip, target_ip):  # packet.rs:425-446
    d = struct.pack(">HHBBH", 1, 0x0800, 6, 4, opcode)
    d += to_mac_bytes(sender_mac) + to_ipv4_bytes(sender_ip)
    d += to_mac_bytes(target_mac) + to_ipv4_bytes(target_ip)
    return Hdr("ARP", d)


def ipv4(ihl, tos, ident, ttl, frag, proto, src, dst, pktlen):  # packet.rs:455-484
    d = bytearray([0x40 | ihl, tos]) + struct.pack(">HHHBBH", pktlen, ident, frag, ttl, proto, 0)
    d += to_ipv4_bytes(src) + to_ipv4_bytes(dst)
    h = Hdr("IPv4", d)
    h.set_bits(80, 95, ipv4_checksum(d))
    return h


def ipv6(traffic_class, flow_label, next_hdr, hop_limit, src, dst, pktlen):  # packet.rs:485-506
    word = ((0x6 << 28) & 0xF0000000) | ((traffic_class << 20) & 0xFFFFFFFF) | flow_label
    d = struct.pack(">IHBB", word & 0xFFFFFFFF, pktlen & 0xFFFF, next_hdr, hop_limit)
    return Hdr("IPv6", d + to_ipv6_bytes(src) + to_ipv6_bytes(dst))


def udp(src, dst, length):  # packet.rs:507-516
    return Hdr("UDP", struct.pack(">HHHH", src, dst, length & 0xFFFF, 0))


def icmp(t, c):  # packet.rs:517-525
    return Hdr("ICMP", struct.pack(">BBH", t, c, 0))


def tcp(src, dst, seq, ack, data_offset, res, flags, window, chksum, urg):  # packet.rs:526-550
    b12 = ((data_offset << 4) | (res & 0xFF)) & 0xFF
    return Hdr("TCP", struct.pack(">HHIIBBHHH", src, dst, seq, ack, b12, flags, window, chksum, urg))


def vxlan_hdr(vni):  # packet.rs:551-558
    return Hdr("Vxlan", struct.pack(">II", 0x8 << 24, (vni << 8) & 0xFFFFFFFF))


def gre(c, r, k, s, strict, flags, ver, proto):  # packet.rs:559-578
    x = (c << 7) | (r << 6) | (k << 5) | (s << 4) | (strict << 3)
    y = ((flags << 3) | ver) & 0xFF
    return Hdr("GRE", bytes([x & 0xFF, y]) + struct.pack(">H", proto))


def gre_chksum_offset(chksum, offset):  # packet.rs:579-585
    return Hdr("GREChksumOffset", struct.pack(">HH", chksum, offset))


def gre_sequence_number(seq):  # packet.rs:586-591
    return Hdr("GRESequenceNum", struct.pack(">I", seq))


def gre_key(key):  # packet.rs:592-597
    return Hdr("GREKey", struct.pack(">I", key))


def erspan2(vlan_, cos, en, t, session_id, index):  # packet.rs:598-607
    b1 = ((1 << 12) | vlan_) & 0xFFFF
    b2 = ((cos << 13) | (en << 11) | (t << 10) | session_id) & 0xFFFF
    return Hdr("ERSPAN2", struct.pack(">HHI", b1, b2, index))


def erspan3(vlan_, cos, en, t, session_id, timestamp, sgt, ft_d_other):  # packet.rs:608-628
    b1 = ((2 << 12) | vlan_) & 0xFFFF
    b2 = ((cos << 13) | (en << 11) | (t << 10) | session_id) & 0xFFFF
    return Hdr("ERSPAN3", struct.pack(">HHIHH", b1, b2, timestamp, sgt, ft_d_other))


def mpls(label, exp, bos, ttl):  # packet.rs:629-633 (field shifts as written: Q11 of SURVEY row 11)
    w = ((label << 20) | (exp << 23) | (bos << 24) | ttl) & 0xFFFFFFFF
    return Hdr("MPLS", struct.pack(">I", w))


def mpls_raw(label, exp, bos, ttl):
    """An MPLS label laid out as the header's field table says (headers.rs:818-827)."""
    w = ((label & 0xFFFFF) << 12) | ((exp & 7) << 9) | ((bos & 1) << 8) | (ttl & 0xFF)
    return Hdr("MPLS", struct.pack(">I", w))


def snap(oui, code):  # packet.rs:634-643
    return Hdr("SNAP", struct.pack(">HBH", oui & 0xFFFF, (oui >> 16) & 0xFF, code))


# --------------------------------------------------------------------------- utils.rs
def create_eth_packet(eth_dst, eth_src, vlan_enable, vlan_vid, vlan_pcp, etype, payload):
    pkt = Packet()
    if vlan_enable:
        pkt.push(ethernet(eth_dst, eth_src, 0x8100))
        pkt.push(vlan(vlan_pcp, 0, vlan_vid, etype))
    else:
        pkt.push(ethernet(eth_dst, eth_src, etype))
    pkt.set_payload(payload)
    return pkt


def create_arp_packet(eth_dst, eth_src, vlan_enable, vlan_vid, vlan_pcp, opcode, sender_mac,
                      target_mac, sender_ip, target_ip, payload):
    pkt = create_eth_packet(eth_dst, eth_src, vlan_enable, vlan_vid, vlan_pcp, 0x0806, payload)
    pkt.push(arp(opcode, sender_mac, target_mac, sender_ip, target_ip))
    return pkt


def create_ipv4_packet(eth_dst, eth_src, vlan_enable, vlan_vid, vlan_pcp, ip_ihl, ip_src, ip_dst,
                       ip_proto, ip_tos, ip_ttl, ip_id, ip_frag, _ip_options, payload):
    pkt = create_eth_packet(eth_dst, eth_src, vlan_enable, vlan_vid, vlan_pcp, 0x0800, payload)
    pktlen = 20 + len(payload)
    pkt.push(ipv4(ip_ihl, ip_tos, ip_id, ip_ttl, ip_frag, ip_proto, ip_src, ip_dst, pktlen & 0xFFFF))
    return pkt


def create_ipv6_packet(eth_dst, eth_src, vlan_enable, vlan_vid, vlan_pcp, tc, fl, nh, hl, src, dst,
                       payload):
    pkt = create_eth_packet(eth_dst, eth_src, vlan_enable, vlan_vid, vlan_pcp, 0x86DD, payload)
    pkt.push(ipv6(tc, fl, nh, hl, src, dst, len(payload)))
    return pkt


def _ipv4_add_len(pkt, extra, recompute=True):
    ip = pkt["IPv4"]
    ip.set_bits(16, 31, (ip.get_bits(16, 31) + extra) & 0xFFFF)
    if recompute:
        ip.set_bits(80, 95, ipv4_checksum(ip.data))


def _ipv6_add_len(pkt, extra):
    ip = pkt["IPv6"]
    ip.set_bits(32, 47, (ip.get_bits(32, 47) + extra) & 0xFFFF)


def create_tcp_packet(eth_dst, eth_src, vlan_enable, vlan_vid, vlan_pcp, ip_ihl, ip_src, ip_dst,
                      ip_tos, ip_ttl, ip_id, ip_frag, ip_options, tcp_dst, tcp_src, tcp_seq_no,
                      tcp_ack_no, tcp_data_offset, tcp_res, tcp_flags, tcp_window, tcp_urgent_ptr,
                      _tcp_checksum, payload):
    pkt = create_ipv4_packet(eth_dst, eth_src, vlan_enable, vlan_vid, vlan_pcp, ip_ihl, ip_src,
                             ip_dst, 6, ip_tos, ip_ttl, ip_id, ip_frag, ip_options, payload)
    _ipv4_add_len(pkt, 20)
    pkt.push(tcp(tcp_src, tcp_dst, tcp_seq_no, tcp_ack_no, tcp_data_offset, tcp_res, tcp_flags,
                 tcp_window, 0, tcp_urgent_ptr))
    return pkt


def create_udp_packet(eth_dst, eth_src, vlan_enable, vlan_vid, vlan_pcp, ip_ihl, ip_src, ip_dst,
                      ip_tos, ip_ttl, ip_id, ip_frag, ip_options, udp_dst, udp_src, _udp_checksum,
                      payload):
    pkt = create_ipv4_packet(eth_dst, eth_src, vlan_enable, vlan_vid, vlan_pcp, ip_ihl, ip_src,
                             ip_dst, 17, ip_tos, ip_ttl, ip_id, ip_frag, ip_options, payload)
    _ipv4_add_len(pkt, 8)
    pkt.push(udp(udp_src, udp_dst, 8 + len(payload)))
    return pkt


def create_icmp_packet(eth_dst, eth_src, vlan_enable, vlan_vid, vlan_pcp, ip_ihl, ip_src, ip_dst,
                       ip_tos, ip_ttl, ip_id, ip_frag, ip_options, icmp_type, icmp_code, _data,
                       _csum, payload):
    pkt = create_ipv4_packet(eth_dst, eth_src, vlan_enable, vlan_vid, vlan_pcp, ip_ihl, ip_src,
                             ip_dst, 1, ip_tos, ip_ttl, ip_id, ip_frag, ip_options, payload)
    _ipv4_add_len(pkt, 4)
    pkt.push(icmp(icmp_type, icmp_code))
    return pkt


def _inner_proto(vec):
    return {4: 4, 6: 41}.get((vec[0] >> 4) & 0xF, 4)


def create_ipv4ip_packet(eth_dst, eth_src, vlan_enable, vlan_vid, vlan_pcp, ip_ihl, ip_src, ip_dst,
                         ip_tos, ip_ttl, ip_id, ip_frag, ip_options, inner):
    v = inner.to_vec()
    return create_ipv4_packet(eth_dst, eth_src, vlan_enable, vlan_vid, vlan_pcp, ip_ihl, ip_src,
                              ip_dst, _inner_proto(v), ip_tos, ip_ttl, ip_id, ip_frag, ip_options, v)


def create_ipv6ip_packet(eth_dst, eth_src, vlan_enable, vlan_vid, vlan_pcp, tc, fl, hl, src, dst,
                         inner):
    v = inner.to_vec()
    return create_ipv6_packet(eth_dst, eth_src, vlan_enable, vlan_vid, vlan_pcp, tc, fl,
                              _inner_proto(v), hl, src, dst, v)


def create_tcpv6_packet(eth_dst, eth_src, vlan_enable, vlan_vid, vlan_pcp, tc, fl, hl, src, dst,
                        tcp_dst, tcp_src, seq, ack, doff, res, flags, window, urg, payload):
    pkt = create_ipv6_packet(eth_dst, eth_src, vlan_enable, vlan_vid, vlan_pcp, tc, fl, 6, hl, src,
                             dst, payload)
    _ipv6_add_len(pkt, 20)
    pkt.push(tcp(tcp_src, tcp_dst, seq, ack, doff, res, flags, window, 0, urg))
    return pkt


def create_udpv6_packet(eth_dst, eth_src, vlan_enable, vlan_vid, vlan_pcp, tc, fl, hl, src, dst,
                        udp_dst, udp_src, _csum, payload):
    pkt = create_ipv6_packet(eth_dst, eth_src, vlan_enable, vlan_vid, vlan_pcp, tc, fl, 17, hl, src,
                             dst, payload)
    _ipv6_add_len(pkt, 8)
    u = udp(udp_src, udp_dst, 8 + len(payload))
    u.set_bits(48, 63, 0xFFFF)
    pkt.push(u)
    return pkt


def create_icmpv6_packet(eth_dst, eth_src, vlan_enable, vlan_vid, vlan_pcp, tc, fl, hl, src, dst,
                         icmp_type, icmp_code, _data, _csum, payload):
    pkt = create_ipv6_packet(eth_dst, eth_src, vlan_enable, vlan_vid, vlan_pcp, tc, fl, 58, hl, src,
                             dst, payload)
    _ipv6_add_len(pkt, 4)
    pkt.push(icmp(icmp_type, icmp_code))
    return pkt


def create_vxlan_packet(eth_dst, eth_src, vlan_enable, vlan_vid, vlan_pcp, ip_ihl, ip_src, ip_dst,
                        ip_tos, ip_ttl, ip_id, ip_frag, ip_options, udp_dst, udp_src, _csum,
                        vni, inner):
    v = inner.to_vec()
    pkt = create_ipv4_packet(eth_dst, eth_src, vlan_enable, vlan_vid, vlan_pcp, ip_ihl, ip_src,
                             ip_dst, 17, ip_tos, ip_ttl, ip_id, ip_frag, ip_options, v)
    _ipv4_add_len(pkt, 16, recompute=False)  # utils.rs:542-543: checksum left stale (Q9)
    pkt.push(udp(udp_src, udp_dst, 16 + len(v)))
    pkt.push(vxlan_hdr(vni))
    return pkt


def create_vxlanv6_packet(eth_dst, eth_src, vlan_enable, vlan_vid, vlan_pcp, tc, fl, hl, src, dst,
                          udp_dst, udp_src, _csum, vni, inner):
    v = inner.to_vec()
    pkt = create_ipv6_packet(eth_dst, eth_src, vlan_enable, vlan_vid, vlan_pcp, tc, fl, 17, hl, src,
                             dst, v)
    _ipv6_add_len(pkt, 16)
    u = udp(udp_src, udp_dst, 16 + len(v))
    u.set_bits(48, 63, 0xFFFF)
    pkt.push(u)
    pkt.push(vxlan_hdr(vni))
    return pkt + inner  # Q12: inner headers again, ahead of the payload copy


def create_gre_packet(eth_dst, eth_src, vlan_enable, vlan_vid, vlan_pcp, ip_ihl, ip_src, ip_dst,
                      ip_tos, ip_ttl, ip_id, ip_frag, ip_options, c, r, k, s, strict, flags, ver,
                      chksum, offset, key, seqnum, routing, inner):
    if inner is not None:
        v = inner.to_vec()
        proto = {4: 0x0800, 6: 0x86DD}.get((v[0] >> 4) & 0xF, 0)
    else:
        v, proto = b"", 0
    pktlen = 4 + 4 * c + 4 * k + 4 * s + (len(routing) if r else 0)
    pkt = create_ipv4_packet(eth_dst, eth_src, vlan_enable, vlan_vid, vlan_pcp, ip_ihl, ip_src,
                             ip_dst, 47, ip_tos, ip_ttl, ip_id, ip_frag, ip_options, v)
    _ipv4_add_len(pkt, pktlen)
    pkt.push(gre(c, r, k, s, strict, flags, ver, proto))
    if c:
        pkt.push(gre_chksum_offset(chksum, offset))
    if k:
        pkt.push(gre_key(key))
    if s:
        pkt.push(gre_sequence_number(seqnum))
    return pkt


def create_erspan_2_packet(eth_dst, eth_src, vlan_enable, vlan_vid, vlan_pcp, ip_ihl, ip_src,
                           ip_dst, ip_tos, ip_ttl, ip_id, ip_frag, ip_options, gre_seqnum, evlan,
                           cos, en, t, session_id, index, inner):
    v = inner.to_vec() if inner is not None else b""
    pktlen = 4 + 8 + (4 if gre_seqnum != 0 else 0) + (len(inner.to_vec()) if inner is not None else 0)
    pkt = create_ipv4_packet(eth_dst, eth_src, vlan_enable, vlan_vid, vlan_pcp, ip_ihl, ip_src,
                             ip_dst, 47, ip_tos, ip_ttl, ip_id, ip_frag, ip_options, v)
    _ipv4_add_len(pkt, pktlen)
    g = Hdr("GRE", bytes(4))
    g.set_bits(16, 31, 0x88BE)
    if gre_seqnum != 0:
        g.set_bits(3, 3, 1)
    pkt.push(g)
    if gre_seqnum != 0:
        pkt.push(gre_sequence_number(gre_seqnum))
    pkt.push(erspan2(evlan, cos, en, t, session_id, index))
    return pkt


def create_erspan_3_packet(eth_dst, eth_src, vlan_enable, vlan_vid, vlan_pcp, ip_ihl, ip_src,
                           ip_dst, ip_tos, ip_ttl, ip_id, ip_frag, ip_options, gre_seqnum, evlan,
                           cos, en, t, session_id, timestamp, sgt, ft_d_other, pltfm_id, pltfm_info,
                           inner):
    v = inner.to_vec() if inner is not None else b""
    pktlen = 4 + 12 + (4 if gre_seqnum != 0 else 0) + (8 if ft_d_other & 1 else 0)
    pktlen += len(inner.to_vec()) if inner is not None else 0
    pkt = create_ipv4_packet(eth_dst, eth_src, vlan_enable, vlan_vid, vlan_pcp, ip_ihl, ip_src,
                             ip_dst, 47, ip_tos, ip_ttl, ip_id, ip_frag, ip_options, v)
    _ipv4_add_len(pkt, pktlen)
    g = Hdr("GRE", bytes(4))
    g.set_bits(16, 31, 0x22EB)
    g.set_bits(3, 3, gre_seqnum)  # utils.rs:846: the low bit of the sequence number
    pkt.push(g)
    if gre_seqnum != 0:
        pkt.push(gre_sequence_number(gre_seqnum))
    pkt.push(erspan3(evlan, cos, en, t, session_id, timestamp, sgt, ft_d_other))
    if ft_d_other & 1:
        pkt.push(Hdr("ERSPANPLATFORM", struct.pack(">Q", ((pltfm_id << 58) | pltfm_info) & (2**64 - 1))))
    if inner is not None:
        pkt = pkt + inner  # Q12
    return pkt


# --------------------------------------------------------------------------- tests/lib.rs:220-671
REFERENCE_22_NAMES = [
    "tcp", "udp", "icmp", "tcpv6", "udpv6", "icmpv6", "vxlan_udp", "vxlanv6_udp", "vxlan_tcp",
    "vxlanv6_tcp", "arp_req", "arp_resp", "ip4ip4", "ip4ip6", "ip6ip4", "ip6ip6", "llc", "snap",
    "greip4", "greip6", "erspan2", "erspan3",
]


def reference_22_packets():
    """The 22 packets of create_packet_test (tests/lib.rs:220-671), as Packet objects, in the
    order of its `pkts` vector (lib.rs:648-671)."""
    payload = bytes(range(100))
    M1, M2 = "00:01:02:03:04:05", "00:06:07:08:09:0a"
    _tcp = create_tcp_packet(M1, M2, False, 10, 3, 5, "10.10.10.1", "11.11.11.1", 0, 64, 115, 0, [],
                             1234, 9090, 100, 101, 5, 0, 0x10, 2, 0, False, payload)
    _udp = create_udp_packet(M1, M2, False, 10, 3, 5, "192.168.0.199", "192.168.0.1", 0, 64, 0,
                             0x4000, [], 1234, 9090, False, payload)
    _icmp = create_icmp_packet(M1, M2, False, 10, 3, 5, "192.168.0.199", "192.168.0.1", 0, 64, 0,
                               0x4000, [], 8, 0, [], False, payload)
    _tcpv6 = create_tcpv6_packet(M1, M2, False, 10, 3, 5, 4, 64, "AAAA::1", "BBBB::1", 1234, 9090,
                                 100, 101, 5, 0, 1, 0, 0, payload)
    _udpv6 = create_udpv6_packet(M1, M2, False, 10, 3, 5, 4, 64, "AAAA::1", "BBBB::1", 1234, 9090,
                                 False, payload)
    _icmpv6 = create_icmpv6_packet(M1, M2, False, 10, 3, 5, 4, 64, "AAAA::1", "BBBB::1", 135, 0, [],
                                   False, payload)
    _vxlan_udp = create_vxlan_packet(M1, M2, False, 10, 3, 5, "192.168.0.199", "192.168.0.1", 0, 64,
                                     0, 0x4000, [], VXLAN_PORT, 9090, False, 2000, _udp.clone())
    _vxlan_tcp = create_vxlan_packet(M1, M2, False, 10, 3, 5, "192.168.0.199", "192.168.0.1", 0, 64,
                                     0, 0x4000, [], VXLAN_PORT, 9090, False, 2000, _tcp.clone())
    _vxlanv6_udp = create_vxlanv6_packet(M1, M2, False, 10, 3, 5, 4, 64, "AAAA::1", "BBBB::1",
                                         VXLAN_PORT, 9090, False, 2000, _udp.clone())
    _vxlanv6_tcp = create_vxlanv6_packet(M1, M2, False, 10, 3, 5, 4, 64, "AAAA::1", "BBBB::1",
                                         VXLAN_PORT, 9090, False, 2000, _tcp.clone())
    _arp_req = create_arp_packet("FF:FF:FF:FF:FF:FF", M2, False, 10, 3, 1, M2, "00:00:00:00:00:00",
                                 "10.10.10.1", "0.0.0.0", payload)
    _arp_resp = create_arp_packet(M2, M1, False, 10, 3, 2, M1, M2, "10.10.10.2", "10.10.10.1",
                                  payload)
    ip_tcp = _tcp.clone()
    ip_tcp.remove(0)
    ip_udp = _udp.clone()
    ip_udp.remove(0)
    ip_tcpv6 = _tcpv6.clone()
    ip_tcpv6.remove(0)
    ip_udpv6 = _udpv6.clone()
    ip_udpv6.remove(0)
    _ip4ip4 = create_ipv4ip_packet(M1, M2, False, 10, 3, 5, "192.168.0.199", "192.168.0.1", 0, 64,
                                   0, 0x4000, [], ip_tcp.clone())
    _ip4ip6 = create_ipv4ip_packet(M1, M2, False, 10, 3, 5, "192.168.0.199", "192.168.0.1", 0, 64,
                                   0, 0x4000, [], ip_udpv6.clone())
    _ip6ip4 = create_ipv6ip_packet(M1, M2, False, 10, 3, 5, 4, 64, "AAAA::1", "BBBB::1",
                                   ip_udp.clone())
    _ip6ip6 = create_ipv6ip_packet(M1, M2, False, 10, 3, 5, 4, 64, "AAAA::1", "BBBB::1",
                                   ip_tcpv6.clone())
    _greip4 = create_gre_packet(M1, M2, False, 10, 3, 5, "192.168.0.199", "192.168.0.1", 0, 64, 0,
                                0x4000, [], 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, b"", ip_tcp.clone())
    _greip6 = create_gre_packet(M1, M2, False, 10, 3, 5, "192.168.0.199", "192.168.0.1", 0, 64, 0,
                                0x4000, [], 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, b"", ip_udpv6.clone())
    _erspan2 = create_erspan_2_packet(M1, M2, False, 10, 3, 5, "192.168.0.199", "192.168.0.1", 0, 64,
                                      0, 0x4000, [], 23, 0, 0, 1, 0, 10, 10, _udpv6.clone())
    _erspan3 = create_erspan_3_packet(M1, M2, False, 10, 3, 5, "192.168.0.199", "192.168.0.1", 0, 64,
                                      0, 0x4000, [], 23, 0, 0, 1, 0, 10, 10, 10, 1, 4, 0xFFFFFFFF,
                                      _icmp.clone())
    _llc = Packet()
    _llc.push(Hdr("Dot3", bytes([0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 0x0, 86])))
    _llc.push(Hdr("LLC", bytes([0x0, 0x04, 0x0])))
    _snap = Packet()
    _snap.push(Hdr("Dot3", bytes([0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 0x0, 86])))
    _snap.push(Hdr("LLC", bytes([0xAA, 0xAA, 0x03])))
    _snap.push(Hdr("SNAP", bytes([0x0, 0x80, 0xC2, 0x8, 0x0])))
    return [_tcp, _udp, _icmp, _tcpv6, _udpv6, _icmpv6, _vxlan_udp, _vxlanv6_udp, _vxlan_tcp,
            _vxlanv6_tcp, _arp_req, _arp_resp, _ip4ip4, _ip4ip6, _ip6ip4, _ip6ip6, _llc, _snap,
            _greip4, _greip6, _erspan2, _erspan3]


def test_tcp_packet_with_payload(payload):
    """tests/lib.rs:682-709."""
    return create_tcp_packet("00:11:11:11:11:11", "00:06:07:08:09:0a", False, 10, 3, 5,
                             "10.10.10.1", "11.11.11.1", 0, 64, 115, 0, [], 8888, 9090, 100, 101, 5,
                             0, 2, 0, 0, False, payload)


# --------------------------------------------------------------------------- pcap (tests/pcap.rs)
PCAP_GLOBAL_HEADER = bytes([0xD4, 0xC3, 0xB2, 0xA1, 0x2, 0x0, 0x4, 0x0, 0, 0, 0, 0, 0, 0, 0, 0,
                            0xFF, 0xFF, 0, 0, 1, 0, 0, 0])


def pcap_bytes(packets, tv_sec=0, tv_usec=0):
    """tests/pcap.rs:7-37 layout (timestamps fixed so the bytes are reproducible)."""
    out = bytearray(PCAP_GLOBAL_HEADER)
    for p in packets:
        out += struct.pack("<IIII", tv_sec, tv_usec, len(p), len(p))
        out += p
    return bytes(out)


def pcap_index_py(buf):
    """(offsets, lens) of the records of a tests/pcap.rs-format buffer."""
    if buf[:4] != PCAP_GLOBAL_HEADER[:4]:
        raise ValueError("bad pcap magic")
    off, offs, lens = 24, [], []
    while off + 16 <= len(buf):
        incl = struct.unpack_from("<I", buf, off + 8)[0]
        if off + 16 + incl > len(buf):
            raise ValueError("truncated pcap record")
        offs.append(off + 16)
        lens.append(incl)
        off += 16 + incl
    return np.array(offs, np.uint64), np.array(lens, np.uint32)


# --------------------------------------------------------------------------- synthetic slabs
def _csum_rows(hdr):
    """Vectorised Packet::ipv4_checksum over rows of 20-byte headers (uint8 [n,20])."""
    w = (hdr[:, 0::2].astype(np.uint32) << 8) | hdr[:, 1::2].astype(np.uint32)
    w[:, 5] = 0  # byte offset 10 skipped
    s = w.sum(axis=1, dtype=np.uint32)
    s = ((s >> 16) + s) & 0xFFFF  # one fold reaches <= 0xFFFF (Q1)
    return (~s) & 0xFFFF


def _put16(a, col, v):
    a[:, col] = (v >> 8) & 0xFF
    a[:, col + 1] = v & 0xFF


def _put32(a, col, v):
    for k in range(4):
        a[:, col + k] = (v >> (24 - 8 * k)) & 0xFF


def _ipv4_rows(rng, n, proto, total_len, bad_csum_frac=0.01):
    h = np.zeros((n, 20), np.uint8)
    h[:, 0] = 0x45
    h[:, 1] = rng.integers(0, 256, n)  # tos
    _put16(h, 2, np.full(n, total_len, np.uint32) if np.isscalar(total_len) else total_len)
    _put16(h, 4, rng.integers(0, 65536, n).astype(np.uint32))  # id
    _put16(h, 6, np.full(n, 0x4000, np.uint32))  # frag (DF)
    h[:, 8] = rng.integers(1, 256, n)  # ttl in [1,255]
    h[:, 9] = proto
    h[:, 12:20] = rng.integers(0, 256, (n, 8))  # src, dst
    cs = _csum_rows(h)
    bad = rng.random(n) < bad_csum_frac
    cs = np.where(bad, rng.integers(0, 65536, n).astype(np.uint32), cs)
    _put16(h, 10, cs)
    return h


def _udp_dst(rng, n):
    d = rng.integers(0, 65536, n).astype(np.uint32)
    return np.where(d == VXLAN_PORT, d + 1, d)  # keep C2 on the Ether/IPv4/UDP chain


def gen_c2(n, seed=0x5EED0002, stride=64):
    """C2: n x 64 B Ether/IPv4/UDP (create_udp_packet layout, utils.rs:197-242): 14+20+8 header
    bytes + 22 payload bytes; random MACs, tos, id, ttl, IPs, ports; 1 % corrupt checksums."""
    assert stride >= 64
    rng = np.random.default_rng(seed)
    a = np.zeros((n, stride), np.uint8)
    a[:, 0:12] = rng.integers(0, 256, (n, 12))
    _put16(a, 12, np.full(n, 0x0800, np.uint32))
    a[:, 14:34] = _ipv4_rows(rng, n, 17, 20 + 8 + 22)
    _put16(a, 34, rng.integers(0, 65536, n).astype(np.uint32))  # udp src
    _put16(a, 36, _udp_dst(rng, n))
    _put16(a, 38, np.full(n, 30, np.uint32))
    a[:, 42:64] = np.arange(22, dtype=np.uint8)
    return a


def gen_c3(n, seed=0x5EED0003, stride=128):
    """C3: n x 128 B Ether -> {0,1,2} x Vlan (1/3 each) -> IPv4 -> TCP (90 %) | UDP (10 %),
    random fields, payload filling the slot."""
    rng = np.random.default_rng(seed)
    a = np.zeros((n, stride), np.uint8)
    a[:, 0:12] = rng.integers(0, 256, (n, 12))
    tags = rng.integers(0, 3, n)
    is_tcp = rng.random(n) < 0.9
    for k in range(3):
        idx = np.nonzero(tags == k)[0]
        if idx.size == 0:
            continue
        m = idx.size
        b = np.zeros((m, stride), np.uint8)
        o = 12
        for t in range(k):
            _put16(b, o, np.full(m, 0x8100, np.uint32))
            tci = rng.integers(0, 65536, m).astype(np.uint32)
            _put16(b, o + 2, tci)
            o += 4
        _put16(b, o, np.full(m, 0x0800, np.uint32))
        o += 2
        tcp_m = is_tcp[idx]
        l4 = np.where(tcp_m, 20, 8)
        total = np.full(m, stride - o, np.uint32)
        ip = _ipv4_rows(rng, m, 6, total)
        ip[~tcp_m, 9] = 17
        ip[:, 10:12] = 0
        cs = _csum_rows(ip)
        _put16(ip, 10, cs)
        b[:, o:o + 20] = ip
        o4 = o + 20
        b[:, o4:o4 + 20] = rng.integers(0, 256, (m, 20))
        ud = ~tcp_m
        if ud.any():
            sub = b[ud]
            _put16(sub, o4 + 2, _udp_dst(rng, sub.shape[0]))
            b[ud] = sub
        pl = o4 + l4
        cols = np.arange(stride)
        fill = (cols[None, :] >= pl[:, None])
        b[fill] = (cols[None, :].repeat(m, 0)[fill] & 0xFF).astype(np.uint8)
        b[:, 0:12] = a[idx, 0:12]
        a[idx] = b
    return a


def gen_c4(n, seed=0x5EED0004):
    """C4: pcap replay — n records drawn uniformly (seeded) from the 22 templates of
    tests/lib.rs:220-671, written in the tests/pcap.rs format.  Returns (pcap_bytes as a
    uint8 array, offsets uint64[n], lens uint32[n])."""
    rng = np.random.default_rng(seed)
    tmpl = [p.to_vec() for p in reference_22_packets()]
    choice = rng.integers(0, len(tmpl), n)
    tlen = np.array([len(t) for t in tmpl], np.int64)
    rec = 16 + tlen[choice]
    offs = 24 + np.concatenate([[0], np.cumsum(rec)[:-1]]) + 16
    total = 24 + int(rec.sum())
    buf = np.zeros(total, np.uint8)
    buf[:24] = np.frombuffer(PCAP_GLOBAL_HEADER, np.uint8)
    for t, tb in enumerate(tmpl):
        idx = np.nonzero(choice == t)[0]
        if idx.size == 0:
            continue
        L = len(tb)
        hdr = np.frombuffer(struct.pack("<IIII", 0, 0, L, L), np.uint8)
        pos = (offs[idx] - 16)[:, None] + np.arange(16)[None, :]
        buf[pos] = hdr
        pos = offs[idx][:, None] + np.arange(L)[None, :]
        buf[pos] = np.frombuffer(tb, np.uint8)
    return buf, offs.astype(np.uint64), tlen[choice].astype(np.uint32)
