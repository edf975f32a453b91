// pktgpu_host.cpp — host-side part of the C ABI: metadata tables, the pcap indexer and the
// host checksum.  No device code.
#include <cstring>

#include "../../include/pktgpu.h"

namespace {

struct FieldDef {
    const char* name;
    uint16_t start, end;
};
struct HdrDef {
    const char* name;
    int size;
    int nfields;
    FieldDef f[16];
};

// make_header! invocations of the reference (src/headers.rs:529-827).
const HdrDef kHdrs[PKT_HDR_COUNT] = {
    {"", 0, 0, {}},
    {"Ether", 14, 3, {{"dst", 0, 47}, {"src", 48, 95}, {"etype", 96, 111}}},
    {"Vlan", 4, 4, {{"pcp", 0, 2}, {"cfi", 3, 3}, {"vid", 4, 15}, {"etype", 16, 31}}},
    {"IPv4", 20, 12,
     {{"version", 0, 3}, {"ihl", 4, 7}, {"diffserv", 8, 15}, {"total_len", 16, 31},
      {"identification", 32, 47}, {"flags", 48, 50}, {"frag_startset", 51, 63}, {"ttl", 64, 71},
      {"protocol", 72, 79}, {"header_checksum", 80, 95}, {"src", 96, 127}, {"dst", 128, 159}}},
    {"IPv6", 40, 8,
     {{"version", 0, 3}, {"traffic_class", 4, 11}, {"flow_label", 12, 31}, {"payload_len", 32, 47},
      {"next_hdr", 48, 55}, {"hop_limit", 56, 63}, {"src", 64, 191}, {"dst", 192, 319}}},
    {"ICMP", 4, 3, {{"icmp_type", 0, 7}, {"icmp_code", 8, 15}, {"chksum", 16, 31}}},
    {"TCP", 20, 10,
     {{"src", 0, 15}, {"dst", 16, 31}, {"seq_no", 32, 63}, {"ack_no", 64, 95},
      {"data_startset", 96, 99}, {"res", 100, 103}, {"flags", 104, 111}, {"window", 112, 127},
      {"checksum", 128, 143}, {"urgent_ptr", 144, 159}}},
    {"UDP", 8, 4, {{"src", 0, 15}, {"dst", 16, 31}, {"length", 32, 47}, {"checksum", 48, 63}}},
    {"ARP", 28, 9,
     {{"hwtype", 0, 15}, {"proto_type", 16, 31}, {"hwlen", 32, 39}, {"proto_len", 40, 47},
      {"opcode", 48, 63}, {"sender_hw_addr", 64, 111}, {"sender_proto_addr", 112, 143},
      {"target_hw_addr", 144, 191}, {"target_proto_addr", 192, 223}}},
    {"Vxlan", 8, 4, {{"flags", 0, 7}, {"reserved", 8, 31}, {"vni", 32, 55}, {"reserved2", 56, 63}}},
    {"Dot3", 14, 3, {{"dst", 0, 47}, {"src", 48, 95}, {"length", 96, 111}}},
    {"LLC", 3, 3, {{"dsap", 0, 7}, {"ssap", 8, 15}, {"ctrl", 16, 23}}},
    {"SNAP", 5, 2, {{"oui", 0, 23}, {"code", 24, 39}}},
    {"GRE", 4, 9,
     {{"chksum_present", 0, 0}, {"routing_present", 1, 1}, {"key_present", 2, 2},
      {"seqnum_present", 3, 3}, {"strict_route_src", 4, 4}, {"recurse", 5, 7}, {"flags", 8, 12},
      {"version", 13, 15}, {"proto", 16, 31}}},
    {"GREChksumOffset", 4, 2, {{"chksum", 0, 15}, {"offset", 16, 31}}},
    {"GRESequenceNum", 4, 1, {{"seqnum", 0, 31}}},
    {"GREKey", 4, 1, {{"key", 0, 31}}},
    {"ERSPAN2", 8, 8,
     {{"version", 0, 3}, {"vlan", 4, 15}, {"cos", 16, 18}, {"en", 19, 20}, {"t", 21, 21},
      {"session_id", 22, 31}, {"reserved", 32, 43}, {"index", 44, 63}}},
    {"ERSPAN3", 12, 14,
     {{"version", 0, 3}, {"vlan", 4, 15}, {"cos", 16, 18}, {"bos", 19, 20}, {"t", 21, 21},
      {"session_id", 22, 31}, {"timestamp", 32, 63}, {"sgt", 64, 79}, {"p", 80, 80}, {"ft", 81, 85},
      {"hw_id", 86, 91}, {"d", 92, 92}, {"gra", 93, 94}, {"o", 95, 95}}},
    {"ERSPANPLATFORM", 8, 2, {{"id", 0, 5}, {"info", 6, 63}}},
    {"STP", 35, 14,
     {{"proto", 0, 15}, {"version", 16, 23}, {"bpdu_type", 24, 31}, {"flags", 32, 39},
      {"root_id", 40, 55}, {"root_mac", 56, 103}, {"root_path_cost", 104, 135},
      {"bridge_id", 136, 151}, {"bridge_mac", 152, 199}, {"port_id", 200, 215},
      {"message_age", 216, 231}, {"max_age", 232, 247}, {"hello_time", 248, 263},
      {"fwd_delay", 264, 279}}},
    {"MPLS", 4, 4, {{"label", 0, 19}, {"exp", 20, 22}, {"bos", 23, 23}, {"ttl", 24, 31}}},
};

const char* kEntryNames[PKT_ENTRY_COUNT] = {
    "parse", "parse_dot3", "parse_llc", "parse_snap", "parse_ethernet", "parse_vlan",
    "parse_mpls", "parse_mpls_bos", "parse_ipv4", "parse_ipv6", "parse_gre", "parse_erspan2",
    "parse_erspan3", "parse_arp", "parse_icmp", "parse_tcp", "parse_udp", "parse_vxlan"};

const char* kStatusNames[3] = {"OK", "TRUNCATED", "DEPTH_LIMIT"};

inline uint32_t rd_le32(const uint8_t* p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

}  // namespace

extern "C" {

int pkt_abi_version(void) { return PKTGPU_ABI_VERSION; }
size_t pkt_sizeof_batch(void) { return sizeof(pkt_batch_t); }
size_t pkt_sizeof_out(void) { return sizeof(pkt_out_t); }
size_t pkt_sizeof_field_spec(void) { return sizeof(pkt_field_spec_t); }

const char* pkt_hdr_name(int t) { return (t > 0 && t < PKT_HDR_COUNT) ? kHdrs[t].name : nullptr; }
int pkt_hdr_size(int t) { return (t > 0 && t < PKT_HDR_COUNT) ? kHdrs[t].size : 0; }
int pkt_hdr_field_count(int t) { return (t > 0 && t < PKT_HDR_COUNT) ? kHdrs[t].nfields : 0; }

int pkt_hdr_field(int t, int idx, const char** name, uint16_t* start, uint16_t* end) {
    if (t <= 0 || t >= PKT_HDR_COUNT || idx < 0 || idx >= kHdrs[t].nfields) return PKT_ERR_INVALID_ARG;
    if (name) *name = kHdrs[t].f[idx].name;
    if (start) *start = kHdrs[t].f[idx].start;
    if (end) *end = kHdrs[t].f[idx].end;
    return PKT_SUCCESS;
}

const char* pkt_status_name(int s) { return (s >= 0 && s < 3) ? kStatusNames[s] : nullptr; }
const char* pkt_entry_name(int e) { return (e >= 0 && e < PKT_ENTRY_COUNT) ? kEntryNames[e] : nullptr; }

// tests/pcap.rs:7-37: 24-byte global header (LE magic d4 c3 b2 a1), then per record a 16-byte
// header {ts_sec, ts_usec, incl_len, orig_len} followed by incl_len bytes.
int pkt_pcap_index(const uint8_t* buf, uint64_t len, uint64_t* offsets, uint32_t* lens, uint64_t cap,
                   uint64_t* n_out) {
    if (!buf || !n_out || (cap && (!offsets || !lens))) return PKT_ERR_INVALID_ARG;
    *n_out = 0;
    if (len < 24 || buf[0] != 0xD4 || buf[1] != 0xC3 || buf[2] != 0xB2 || buf[3] != 0xA1)
        return PKT_ERR_INVALID_ARG;
    uint64_t off = 24, n = 0;
    while (off + 16 <= len) {
        uint32_t incl = rd_le32(buf + off + 8);
        if (off + 16 + (uint64_t)incl > len) return PKT_ERR_INVALID_ARG;
        if (n < cap) {
            offsets[n] = off + 16;
            lens[n] = incl;
        }
        n++;
        off += 16 + (uint64_t)incl;
    }
    *n_out = n;
    return PKT_SUCCESS;
}

// The PacketSlice of packet i from host chain columns (lib.rs:136-140: hdrs in `insert` order,
// packet.rs:724-731: insert / set_payload).
int pkt_view(const pkt_out_t* out, uint64_t n, uint64_t i, uint8_t types[PKT_MAX_HDRS], uint16_t offs[PKT_MAX_HDRS],
             uint32_t* n_hdrs, uint16_t* payload_off, uint16_t* payload_len) {
    if (!out || !types || !offs || !n_hdrs || !payload_off || !payload_len || i >= n) return PKT_ERR_INVALID_ARG;
    if (!out->status || !out->n_hdrs || !out->hdr_type || !out->hdr_off || !out->payload_off || !out->payload_len)
        return PKT_ERR_INVALID_ARG;
    *n_hdrs = 0;
    *payload_off = *payload_len = 0;
    const int st = out->status[i];
    if (st != PKT_OK) return st;
    const uint32_t nh = out->n_hdrs[i];
    if (nh > PKT_MAX_HDRS) return PKT_ERR_INVALID_ARG;
    for (uint32_t k = 0; k < nh; k++) {
        types[k] = out->hdr_type[(uint64_t)k * n + i];
        offs[k] = out->hdr_off[(uint64_t)k * n + i];
    }
    *n_hdrs = nh;
    *payload_off = out->payload_off[i];
    *payload_len = out->payload_len[i];
    return st;
}

// Packet::ipv4_checksum (src/packet.rs:93-107), Q1 fold included.
uint16_t pkt_ipv4_checksum_host(const uint8_t* v, size_t len) {
    uint32_t s = 0;
    for (size_t i = 0; i + 1 < len; i += 2) {
        if (i == 10) continue;
        s += ((uint32_t)v[i] << 8) | v[i + 1];
    }
    while (s >> 16) s = ((s >> 16) + s) & 0xFFFFu;
    return (uint16_t)~s;
}

}  // extern "C"
