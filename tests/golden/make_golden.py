"""Regenerate the committed golden fixtures in tests/golden/.

  python tests/golden/make_golden.py

Outputs
  ref22.pcap            the 22 packets of the reference's create_packet_test
                        (tests/lib.rs:220-671) in the tests/pcap.rs:7-37 format, built by the
                        builder restatement in packet-rs_amd/pktgpu/gen.py (timestamps 0).
  ref22_expected.json   per packet: the header list (Header::name(), wire offset) and the
                        payload bounds that fast::parse returns, produced by the C oracle and
                        cross-checked here against the independent Python walk (tests/pyref.py);
                        the script refuses to write when the two disagree.
  kat_reference.json    known-answer values transcribed from the reference's own tests
                        (headers.rs:856-881, tests/lib.rs:58-218, 818-837) and the SURVEY §8(c)
                        worked example.

The reference (Rust) cannot run in this container, so no fixture here is a reference
output; the KATs are the values its test files assert.
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(REPO, "packet-rs_amd"), os.path.join(REPO, "oracle"),
                os.path.join(REPO, "tests")]

from pktgpu import gen, schema  # noqa: E402
import oracle  # noqa: E402
import pyref  # noqa: E402

KAT = {
    "tester": {  # headers.rs:829-881
        "bytes": [0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0x20, 0x01, 0x0d, 0xb8, 0x85, 0xa3, 0xf0,
                  0xe0, 0xd0, 0xc0, 0x8a, 0x2e, 0x03, 0x70, 0x73, 0x34, 0x45, 0x67, 0x20, 0x01,
                  0x0d, 0xb8, 0x85, 0xa3, 0x00, 0x00, 0x00, 0x00, 0x8a, 0x2e, 0x03, 0x70, 0x73,
                  0x35],
        "fields": {"bit1": [0, 0, 1], "bit2": [1, 2, 3], "bit3": [3, 5, 7], "bit4": [6, 9, 15],
                   "bit5": [10, 14, 31], "bit6": [15, 20, 63], "bit7": [21, 27, 127],
                   "bit8": [28, 35, 255], "bit9": [36, 44, 511], "bit10": [45, 47, 7],
                   "byte1": [48, 55, 0x20], "byte2": [56, 71, 0x010d], "byte3": [72, 95, 0xb885a3],
                   "byte8": [128, 191, 0x8a2e037073344567]},
        "byte4_as_u32": [66, 127, 0xf0e0d0c0],
        "byte16_bytes": [192, 319, [0x20, 0x01, 0x0d, 0xb8, 0x85, 0xa3, 0x00, 0x00, 0x00, 0x00,
                                    0x8a, 0x2e, 0x03, 0x70, 0x73, 0x35]],
    },
    "ether_default": {"bytes": [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 8, 0],  # headers.rs:537-539
                      "dst": 0x102030405, "src": 0x60708090a0b, "etype": 0x800},  # lib.rs:63-73
    "ether_from": {"bytes": [0xaa] * 6 + [0xbb] * 6 + [0x86, 0xdd],  # lib.rs:77-86
                   "dst": 0xaaaaaaaaaaaa, "src": 0xbbbbbbbbbbbb, "etype": 0x86dd},
    "vlan_default": {"bytes": [0x0, 0xa, 0x08, 0x00], "pcp": 0, "cfi": 0, "vid": 0xa},  # lib.rs:94-104
    "vlan_from": {"bytes": [0x7f, 0xff, 0x08, 0x00], "vid": 4095, "pcp": 3, "cfi": 1},  # lib.rs:108-115
    "arp_default": {"bytes": [0x0, 0x1, 0x8, 0x0, 0x6, 0x4, 0x0, 0x1, 0x00, 0x01, 0x02, 0x03,
                              0x04, 0x05, 0xa, 0x0, 0x0, 0x1, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00,
                              0x0, 0x0, 0x0, 0x0],  # headers.rs:650-652, lib.rs:206-218
                    "hwtype": 1, "proto_type": 0x800, "hwlen": 6, "proto_len": 4, "opcode": 1,
                    "sender_hw_addr": 0x000102030405, "sender_proto_addr": 0xa000001,
                    "target_hw_addr": 0, "target_proto_addr": 0},
    "vxlan_default": {"bytes": [0x8, 0x0, 0x0, 0x0, 0x0, 0x07, 0xd0, 0x0],  # lib.rs:139-149
                      "flags": 8, "vni": 2000},
    "ipv4_builder": {"args": [5, 10, 4, 64, 0xdd, 6, "10.10.10.1", "11.11.11.1", 86],  # lib.rs:130-131
                     "verify": 0},
    "payload_test": {"payload": list(range(10))},  # lib.rs:818-837
    "worked_example": {
        "bytes_hex": ("00 01 02 03 04 05 00 06 07 08 09 0a 08 00 45 00 00 32 00 00 40 00 40 11 "
                      "b8 a2 c0 a8 00 c7 c0 a8 00 01 23 82 04 d2 00 1e 00 00").replace(" ", "")
                     + bytes(range(22)).hex(),
        "ipv4_csum": 0xb8a2, "udp_src": 9090, "udp_dst": 1234, "udp_len": 30,
        "hdr_offsets": [0, 14, 34], "payload_off": 42, "payload_len": 22},
}


def main():
    pkts = [p.to_vec() for p in gen.reference_22_packets()]
    with open(os.path.join(HERE, "ref22.pcap"), "wb") as f:
        f.write(gen.pcap_bytes(pkts))
    import numpy as np
    offs, lens = gen.pcap_index_py(gen.pcap_bytes(pkts))
    slab = np.frombuffer(gen.pcap_bytes(pkts), np.uint8)
    res = oracle.parse_batch(slab, len(pkts), offsets=offs, lens=lens)
    exp = []
    for i, (name, p) in enumerate(zip(gen.REFERENCE_22_NAMES, pkts)):
        nh = int(res["n_hdrs"][i])
        hdrs = [(schema.HDR_NAMES[res["hdr_type"][j, i]], int(res["hdr_off"][j, i])) for j in range(nh)]
        st = schema.STATUS_NAMES[res["status"][i]]
        py = pyref.parse(p)
        if (st, hdrs, int(res["payload_off"][i]), int(res["payload_len"][i])) != \
                (py[0], [tuple(h) for h in py[1]], py[2], py[3]):
            raise SystemExit(f"oracle and pyref disagree on {name}: {hdrs} vs {py}")
        exp.append({"name": name, "len": len(p), "status": st, "hdrs": hdrs,
                    "payload_off": int(res["payload_off"][i]),
                    "payload_len": int(res["payload_len"][i])})
    with open(os.path.join(HERE, "ref22_expected.json"), "w") as f:
        json.dump(exp, f, indent=1)
    with open(os.path.join(HERE, "kat_reference.json"), "w") as f:
        json.dump(KAT, f, indent=1)
    print("wrote", len(exp), "packets")


if __name__ == "__main__":
    main()
