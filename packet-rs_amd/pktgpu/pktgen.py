"""Batched packet generation on the GPU (§8(f) rank 4: the reference's pktgen workload).

The reference builds packets one at a time (`utils::create_*_packet`, src/utils.rs:7-876) and its
perf test times new / clone / update+clone loops (tests/lib.rs:756-788).  Here the builder runs
once on the host to produce a template, and the device does the per-packet work:

  clone        pkt_broadcast            n copies of the template at a fixed stride
  chain        pkt_parse_batch          fast::parse of the copies (chain columns only)
  update       pkt_set_fields           `<Hdr>::set_<field>(v)` with per-packet values
  re-checksum  pkt_ipv4_update_checksum `set_header_checksum(Packet::ipv4_checksum(..))`
"""
import numpy as np

from . import gen, schema

H = schema.HDR_ID

# (hdr, occurrence, start, end) of the fields gen_udp varies (headers.rs:530-634)
UDP_FIELDS = {
    "eth_dst": (H["Ether"], 0, 0, 47), "eth_src": (H["Ether"], 0, 48, 95),
    "ipv4_diffserv": (H["IPv4"], 0, 8, 15), "ipv4_identification": (H["IPv4"], 0, 32, 47),
    "ipv4_ttl": (H["IPv4"], 0, 64, 71), "ipv4_src": (H["IPv4"], 0, 96, 127),
    "ipv4_dst": (H["IPv4"], 0, 128, 159), "udp_src": (H["UDP"], 0, 0, 15),
    "udp_dst": (H["UDP"], 0, 16, 31),
}


def udp_template(payload_len=22):
    """create_udp_packet with the SURVEY §8(c) arguments: 14 + 20 + 8 header bytes + payload."""
    return gen.create_udp_packet("00:01:02:03:04:05", "00:06:07:08:09:0a", False, 10, 3, 5,
                                 "192.168.0.199", "192.168.0.1", 0, 64, 0, 0x4000, [], 1234, 9090,
                                 False, bytes(range(payload_len))).to_vec()


def gen_udp(parser, n, fields, stride=64, template=None, stream=None):
    """n Ether/IPv4/UDP packets on the device: the template cloned n times, then every field in
    `fields` ({name in UDP_FIELDS: uint64 device tensor [n]}) set per packet and the IPv4
    checksum recomputed.  Returns the flat uint8 device slab."""
    import torch
    tpl = template if template is not None else udp_template()
    src = torch.from_numpy(np.frombuffer(tpl, np.uint8).copy()).to(parser.torch_device)
    slab = parser.broadcast(src, n, stride, stream=stream)
    chain = parser.parse(slab, stride=stride, n=n, columns=["n_hdrs", "hdr_type", "hdr_off"],
                         stream=stream)
    names = [k for k in fields]
    if names:
        parser.set_fields(slab, chain, [UDP_FIELDS[k] for k in names], [fields[k] for k in names],
                          stride=stride, n=n, stream=stream)
    parser.ipv4_update_checksum(slab, chain, 0, stride=stride, n=n, stream=stream)
    return slab
