"""make_header! field tables (src/headers.rs:529-827) as exported by libpktgpu's
pkt_hdr_field(); generated, do not edit.  {hdr_type: {field: (start, end)}}"""
FIELDS = {
    1: {"dst": (0, 47), "src": (48, 95), "etype": (96, 111)},  # Ether
    2: {"pcp": (0, 2), "cfi": (3, 3), "vid": (4, 15), "etype": (16, 31)},  # Vlan
    3: {"version": (0, 3), "ihl": (4, 7), "diffserv": (8, 15), "total_len": (16, 31), "identification": (32, 47), "flags": (48, 50), "frag_startset": (51, 63), "ttl": (64, 71), "protocol": (72, 79), "header_checksum": (80, 95), "src": (96, 127), "dst": (128, 159)},  # IPv4
    4: {"version": (0, 3), "traffic_class": (4, 11), "flow_label": (12, 31), "payload_len": (32, 47), "next_hdr": (48, 55), "hop_limit": (56, 63), "src": (64, 191), "dst": (192, 319)},  # IPv6
    5: {"icmp_type": (0, 7), "icmp_code": (8, 15), "chksum": (16, 31)},  # ICMP
    6: {"src": (0, 15), "dst": (16, 31), "seq_no": (32, 63), "ack_no": (64, 95), "data_startset": (96, 99), "res": (100, 103), "flags": (104, 111), "window": (112, 127), "checksum": (128, 143), "urgent_ptr": (144, 159)},  # TCP
    7: {"src": (0, 15), "dst": (16, 31), "length": (32, 47), "checksum": (48, 63)},  # UDP
    8: {"hwtype": (0, 15), "proto_type": (16, 31), "hwlen": (32, 39), "proto_len": (40, 47), "opcode": (48, 63), "sender_hw_addr": (64, 111), "sender_proto_addr": (112, 143), "target_hw_addr": (144, 191), "target_proto_addr": (192, 223)},  # ARP
    9: {"flags": (0, 7), "reserved": (8, 31), "vni": (32, 55), "reserved2": (56, 63)},  # Vxlan
    10: {"dst": (0, 47), "src": (48, 95), "length": (96, 111)},  # Dot3
    11: {"dsap": (0, 7), "ssap": (8, 15), "ctrl": (16, 23)},  # LLC
    12: {"oui": (0, 23), "code": (24, 39)},  # SNAP
    13: {"chksum_present": (0, 0), "routing_present": (1, 1), "key_present": (2, 2), "seqnum_present": (3, 3), "strict_route_src": (4, 4), "recurse": (5, 7), "flags": (8, 12), "version": (13, 15), "proto": (16, 31)},  # GRE
    14: {"chksum": (0, 15), "offset": (16, 31)},  # GREChksumOffset
    15: {"seqnum": (0, 31)},  # GRESequenceNum
    16: {"key": (0, 31)},  # GREKey
    17: {"version": (0, 3), "vlan": (4, 15), "cos": (16, 18), "en": (19, 20), "t": (21, 21), "session_id": (22, 31), "reserved": (32, 43), "index": (44, 63)},  # ERSPAN2
    18: {"version": (0, 3), "vlan": (4, 15), "cos": (16, 18), "bos": (19, 20), "t": (21, 21), "session_id": (22, 31), "timestamp": (32, 63), "sgt": (64, 79), "p": (80, 80), "ft": (81, 85), "hw_id": (86, 91), "d": (92, 92), "gra": (93, 94), "o": (95, 95)},  # ERSPAN3
    19: {"id": (0, 5), "info": (6, 63)},  # ERSPANPLATFORM
    20: {"proto": (0, 15), "version": (16, 23), "bpdu_type": (24, 31), "flags": (32, 39), "root_id": (40, 55), "root_mac": (56, 103), "root_path_cost": (104, 135), "bridge_id": (136, 151), "bridge_mac": (152, 199), "port_id": (200, 215), "message_age": (216, 231), "max_age": (232, 247), "hello_time": (248, 263), "fwd_delay": (264, 279)},  # STP
    21: {"label": (0, 19), "exp": (20, 22), "bos": (23, 23), "ttl": (24, 31)},  # MPLS
}
