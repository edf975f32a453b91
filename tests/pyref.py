"""Independent pure-Python restatement of packet_rs's fast::parse (tests only).

Written as a forward iterative walk (not the recursion of oracle/pkt_oracle.c) so that the
C oracle is cross-checked by a second, structurally different reading of
src/parser/fast.rs:5-227.  Small cases only (pure-Python loops).

parse(pkt, entry) -> (status, [(type_name, offset)], payload_off, payload_len)
"""
MAX_HDRS = 16
SIZES = {"Ether": 14, "Vlan": 4, "IPv4": 20, "IPv6": 40, "ICMP": 4, "TCP": 20, "UDP": 8,
         "ARP": 28, "Vxlan": 8, "Dot3": 14, "LLC": 3, "SNAP": 5, "GRE": 4,
         "GREChksumOffset": 4, "GRESequenceNum": 4, "GREKey": 4, "ERSPAN2": 8, "ERSPAN3": 12,
         "ERSPANPLATFORM": 8, "MPLS": 4}
ETYPE_NEXT = {0x8100: "vlan", 0x0806: "arp", 0x0800: "ipv4", 0x86DD: "ipv6", 0x8847: "mpls"}
V4_NEXT = {1: "icmp", 4: "ipv4", 6: "tcp", 17: "udp", 41: "ipv6", 47: "gre"}
V6_NEXT = {58: "icmp", 4: "ipv4", 6: "tcp", 17: "udp", 41: "ipv6", 47: "gre"}
GRE_NEXT = {0x0800: "ipv4", 0x86DD: "ipv6", 0x88BE: "erspan2", 0x22EB: "erspan3"}


class _Stop(Exception):
    def __init__(self, status):
        self.status = status


def parse(pkt, entry="parse"):
    n = len(pkt)
    hdrs = []

    def need(o, k):
        if o + k > n:
            raise _Stop("TRUNCATED")

    def push(name, o):
        if len(hdrs) >= MAX_HDRS:
            raise _Stop("DEPTH_LIMIT")
        hdrs.append((name, o))

    def be16(o):
        return (pkt[o] << 8) | pkt[o + 1]

    state, o = entry.replace("parse_", "") if entry != "parse" else "parse", 0
    if state == "ethernet":
        state = "ether"
    try:
        while True:
            if state == "parse":
                need(o, 14)
                state = "dot3" if be16(o + 12) < 1500 else "ether"
            elif state == "dot3":
                need(o, 14); push("Dot3", o); o += 14; state = "llc"
            elif state == "llc":
                need(o, 3); push("LLC", o)
                snap = pkt[o] == 0xAA and pkt[o + 1] == 0xAA and pkt[o + 2] == 0x03
                o += 3; state = "snap" if snap else "accept"
            elif state == "snap":
                need(o, 5); push("SNAP", o); o += 5; state = "accept"
            elif state in ("ether", "vlan"):
                name, size, eo = ("Ether", 14, 12) if state == "ether" else ("Vlan", 4, 2)
                need(o, size); push(name, o)
                et = be16(o + eo); o += size; state = ETYPE_NEXT.get(et, "accept")
            elif state == "mpls":
                need(o, 4); push("MPLS", o)
                bos = pkt[o + 2] & 1; o += 4; state = "mpls_bos" if bos else "mpls"
            elif state == "mpls_bos":
                need(o, 4); push("MPLS", o); need(o, 5)
                nib = pkt[o + 4] >> 4; o += 4
                state = {4: "ipv4", 6: "ipv6"}.get(nib, "ether")
            elif state == "ipv4":
                need(o, 20); push("IPv4", o)
                p = pkt[o + 9]; o += 20; state = V4_NEXT.get(p, "accept")
            elif state == "ipv6":
                need(o, 40); push("IPv6", o)
                p = pkt[o + 6]; o += 40; state = V6_NEXT.get(p, "accept")
            elif state == "gre":
                need(o, 4)
                flags = pkt[o]
                c, k, s = flags >> 7 & 1, flags >> 5 & 1, flags >> 4 & 1
                proto = be16(o + 2)
                push("GRE", o)
                opts, q = [], o + 4
                for present, name in ((c, "GREChksumOffset"), (k, "GREKey"), (s, "GRESequenceNum")):
                    if present:
                        need(q, 4)
                        if len(hdrs) + len(opts) >= MAX_HDRS:
                            raise _Stop("DEPTH_LIMIT")
                        opts.append((name, q)); q += 4
                hdrs.extend(reversed(opts))  # Q2: list order GRE, Seq, Key, Chksum
                o = q; state = GRE_NEXT.get(proto, "accept")
            elif state == "erspan2":
                need(o, 8); push("ERSPAN2", o); o += 8; state = "ether"
            elif state == "erspan3":
                need(o, 12); push("ERSPAN3", o)
                ob = pkt[o + 11] & 1; o += 12
                if ob:
                    need(o, 8); push("ERSPANPLATFORM", o); o += 8
                state = "ether"
            elif state in ("arp", "icmp", "tcp"):
                name = {"arp": "ARP", "icmp": "ICMP", "tcp": "TCP"}[state]
                need(o, SIZES[name]); push(name, o); o += SIZES[name]; state = "accept"
            elif state == "udp":
                need(o, 8); push("UDP", o)
                dst = be16(o + 2); o += 8; state = "vxlan" if dst == 4789 else "accept"
            elif state == "vxlan":
                need(o, 8); push("Vxlan", o); o += 8; state = "ether"
            elif state == "accept":
                return "OK", hdrs, o, n - o
            else:
                raise ValueError(state)
    except _Stop as e:
        return e.status, [], 0, 0


def bit_range_py(b, start, end):
    """make_header! getter semantics with arbitrary-precision ints (reference widths <= 64)."""
    v = 0
    for i in range(start, end + 1):
        v = (v << 1) | ((b[i // 8] >> (7 - i % 8)) & 1)
    return v
