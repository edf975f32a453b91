"""Output schema of the batched parser — the Python mirror of include/pktgpu.h.

Everything here is metadata: header ids/names (reference src/headers.rs:529-827), the
parser entry points (src/parser/fast.rs), and the struct-of-arrays column layout of
`pkt_out_t`.  The order of OUT_COLUMNS is the field order of `pkt_out_t` and must not
change without bumping PKTGPU_ABI_VERSION.
"""
import numpy as np

MAX_HDRS = 16
ABI_VERSION = 5

# pkt_status_t
OK, TRUNCATED, DEPTH_LIMIT = 0, 1, 2
STATUS_NAMES = ["OK", "TRUNCATED", "DEPTH_LIMIT"]

# pkt_hdr_type_t -> Header::name() of the reference (headers.rs:529-827)
HDR_NAMES = [
    "", "Ether", "Vlan", "IPv4", "IPv6", "ICMP", "TCP", "UDP", "ARP", "Vxlan", "Dot3",
    "LLC", "SNAP", "GRE", "GREChksumOffset", "GRESequenceNum", "GREKey", "ERSPAN2",
    "ERSPAN3", "ERSPANPLATFORM", "STP", "MPLS",
]
HDR_ID = {n: i for i, n in enumerate(HDR_NAMES) if n}
HDR_SIZES = [0, 14, 4, 20, 40, 4, 20, 8, 28, 8, 14, 3, 5, 4, 4, 4, 4, 8, 12, 8, 35, 4]

# pkt_entry_t: one per pub fn of parser::fast (fast.rs)
ENTRIES = [
    "parse", "parse_dot3", "parse_llc", "parse_snap", "parse_ethernet", "parse_vlan",
    "parse_mpls", "parse_mpls_bos", "parse_ipv4", "parse_ipv6", "parse_gre",
    "parse_erspan2", "parse_erspan3", "parse_arp", "parse_icmp", "parse_tcp", "parse_udp",
    "parse_vxlan",
]
ENTRY_ID = {n: i for i, n in enumerate(ENTRIES)}

# (column, dtype, per-packet shape, group).  Shape "slots" = slot-major [MAX_HDRS][n].
OUT_COLUMNS = [
    ("status", np.uint8, (), "chain"),
    ("n_hdrs", np.uint8, (), "chain"),
    ("hdr_type", np.uint8, "slots", "chain"),
    ("hdr_off", np.uint16, "slots", "chain"),
    ("payload_off", np.uint16, (), "chain"),
    ("payload_len", np.uint16, (), "chain"),
    ("hdr_mask", np.uint32, (), "chain"),
    ("eth_dst", np.uint64, (), "ether"),
    ("eth_src", np.uint64, (), "ether"),
    ("eth_etype", np.uint16, (), "ether"),
    ("vlan_pcp", np.uint8, (), "vlan"),
    ("vlan_cfi", np.uint8, (), "vlan"),
    ("vlan_vid", np.uint16, (), "vlan"),
    ("vlan_etype", np.uint16, (), "vlan"),
    ("ipv4_version", np.uint8, (), "ipv4"),
    ("ipv4_ihl", np.uint8, (), "ipv4"),
    ("ipv4_diffserv", np.uint8, (), "ipv4"),
    ("ipv4_total_len", np.uint16, (), "ipv4"),
    ("ipv4_identification", np.uint16, (), "ipv4"),
    ("ipv4_flags", np.uint8, (), "ipv4"),
    ("ipv4_frag_startset", np.uint16, (), "ipv4"),
    ("ipv4_ttl", np.uint8, (), "ipv4"),
    ("ipv4_protocol", np.uint8, (), "ipv4"),
    ("ipv4_header_checksum", np.uint16, (), "ipv4"),
    ("ipv4_src", np.uint32, (), "ipv4"),
    ("ipv4_dst", np.uint32, (), "ipv4"),
    ("ipv4_csum_calc", np.uint16, (), "ipv4"),
    ("ipv6_version", np.uint8, (), "ipv6"),
    ("ipv6_traffic_class", np.uint8, (), "ipv6"),
    ("ipv6_flow_label", np.uint32, (), "ipv6"),
    ("ipv6_payload_len", np.uint16, (), "ipv6"),
    ("ipv6_next_hdr", np.uint8, (), "ipv6"),
    ("ipv6_hop_limit", np.uint8, (), "ipv6"),
    ("ipv6_src", np.uint8, (16,), "ipv6"),
    ("ipv6_dst", np.uint8, (16,), "ipv6"),
    ("tcp_src", np.uint16, (), "tcp"),
    ("tcp_dst", np.uint16, (), "tcp"),
    ("tcp_seq_no", np.uint32, (), "tcp"),
    ("tcp_ack_no", np.uint32, (), "tcp"),
    ("tcp_data_startset", np.uint8, (), "tcp"),
    ("tcp_res", np.uint8, (), "tcp"),
    ("tcp_flags", np.uint8, (), "tcp"),
    ("tcp_window", np.uint16, (), "tcp"),
    ("tcp_checksum", np.uint16, (), "tcp"),
    ("tcp_urgent_ptr", np.uint16, (), "tcp"),
    ("udp_src", np.uint16, (), "udp"),
    ("udp_dst", np.uint16, (), "udp"),
    ("udp_length", np.uint16, (), "udp"),
    ("udp_checksum", np.uint16, (), "udp"),
]
COLUMN_NAMES = [c[0] for c in OUT_COLUMNS]
GROUPS = ["chain", "ether", "vlan", "ipv4", "ipv6", "tcp", "udp"]


def columns_of(groups):
    """Column names of the given groups (e.g. ["chain", "ether", "ipv4", "udp"])."""
    groups = set(groups)
    bad = groups - set(GROUPS)
    if bad:
        raise ValueError(f"unknown column groups {sorted(bad)}")
    return [c[0] for c in OUT_COLUMNS if c[3] in groups]


def column_shape(name, n):
    """numpy shape of column `name` for a batch of n packets."""
    for c, dt, shp, _ in OUT_COLUMNS:
        if c == name:
            if shp == "slots":
                return (MAX_HDRS, n)
            return (n,) + tuple(shp)
    raise KeyError(name)


def column_dtype(name):
    for c, dt, _, _ in OUT_COLUMNS:
        if c == name:
            return np.dtype(dt)
    raise KeyError(name)


def column_mask(columns):
    """pkt_out_t column mask (bit k = k-th member) of a set of column names."""
    cols = set(columns)
    return sum(1 << k for k, c in enumerate(COLUMN_NAMES) if c in cols)


def bytes_per_packet(columns, n_slots=MAX_HDRS):
    """Bytes written per packet for a column set; slot columns count `n_slots` slots."""
    total = 0
    for c, dt, shp, _ in OUT_COLUMNS:
        if c not in columns:
            continue
        isz = np.dtype(dt).itemsize
        if shp == "slots":
            total += isz * n_slots
        else:
            total += isz * int(np.prod(shp)) if shp else isz
    return total
