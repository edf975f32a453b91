/*
 * pkt_oracle.c — CPU ORACLE (test infrastructure only).
 *
 * A literal C restatement of packet_rs 0.4.0's decode path, used as the parity checker for
 * the HIP kernels and as the `cpu_baseline` leg of bench.py.  Only tests/, smoke() and
 * bench.py's cpu_baseline may load it.  The product (packet-rs_amd/) never links it.
 *
 * The Rust reference cannot be built here (no cargo/rustc, crates not vendored — see
 * DESIGN.md), so this restatement follows the sources line by line:
 *   - the recursive walk of src/parser/fast.rs:5-227, including each `&arr[a..b]` /
 *     `arr[k]` bounds panic (-> PKT_TRUNCATED), the per-header Box allocation and the
 *     `Vec::insert(0, ..)` prepend of PacketSlice::insert (packet.rs:724-726);
 *   - bit_range, one loop iteration per bit (headers.rs:252-263), with the release-build
 *     shift semantics for fields wider than 64 bits (Q8);
 *   - Packet::ipv4_checksum with its `((s>>16)+s)&0xFFFF` fold (packet.rs:93-107, Q1);
 *   - slow::parse + Packet::to_vec for the config-1 round trip (slow.rs, packet.rs:385-392).
 * Parity pinning: tests/test_oracle.py checks this file against every known-answer test
 * the reference holds for the path (headers.rs:856-881, tests/lib.rs:58-218, 220-680,
 * 818-837).  Header order/offsets after a parse are pinned by no reference test; they
 * are cross-checked against an independent pure-Python restatement (tests/pyref.py).
 */
#include "pkt_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ header tables */
/* make_header! invocations, headers.rs:529-827: name, size, (field, start, end)... */
typedef struct { const char *name; uint16_t start, end; } orc_field_t;
typedef struct { const char *name; int size; int nfields; orc_field_t f[16]; } orc_hdr_def_t;

static const orc_hdr_def_t ORC_HDRS[PKT_HDR_COUNT] = {
    [PKT_HDR_NONE] = {"", 0, 0, {{0}}},
    [PKT_HDR_ETHER] = {"Ether", 14, 3, {{"dst", 0, 47}, {"src", 48, 95}, {"etype", 96, 111}}},
    [PKT_HDR_VLAN] = {"Vlan", 4, 4, {{"pcp", 0, 2}, {"cfi", 3, 3}, {"vid", 4, 15}, {"etype", 16, 31}}},
    [PKT_HDR_IPV4] = {"IPv4", 20, 12,
                      {{"version", 0, 3}, {"ihl", 4, 7}, {"diffserv", 8, 15}, {"total_len", 16, 31},
                       {"identification", 32, 47}, {"flags", 48, 50}, {"frag_startset", 51, 63},
                       {"ttl", 64, 71}, {"protocol", 72, 79}, {"header_checksum", 80, 95},
                       {"src", 96, 127}, {"dst", 128, 159}}},
    [PKT_HDR_IPV6] = {"IPv6", 40, 8,
                      {{"version", 0, 3}, {"traffic_class", 4, 11}, {"flow_label", 12, 31},
                       {"payload_len", 32, 47}, {"next_hdr", 48, 55}, {"hop_limit", 56, 63},
                       {"src", 64, 191}, {"dst", 192, 319}}},
    [PKT_HDR_ICMP] = {"ICMP", 4, 3, {{"icmp_type", 0, 7}, {"icmp_code", 8, 15}, {"chksum", 16, 31}}},
    [PKT_HDR_TCP] = {"TCP", 20, 10,
                     {{"src", 0, 15}, {"dst", 16, 31}, {"seq_no", 32, 63}, {"ack_no", 64, 95},
                      {"data_startset", 96, 99}, {"res", 100, 103}, {"flags", 104, 111},
                      {"window", 112, 127}, {"checksum", 128, 143}, {"urgent_ptr", 144, 159}}},
    [PKT_HDR_UDP] = {"UDP", 8, 4, {{"src", 0, 15}, {"dst", 16, 31}, {"length", 32, 47}, {"checksum", 48, 63}}},
    [PKT_HDR_ARP] = {"ARP", 28, 9,
                     {{"hwtype", 0, 15}, {"proto_type", 16, 31}, {"hwlen", 32, 39}, {"proto_len", 40, 47},
                      {"opcode", 48, 63}, {"sender_hw_addr", 64, 111}, {"sender_proto_addr", 112, 143},
                      {"target_hw_addr", 144, 191}, {"target_proto_addr", 192, 223}}},
    [PKT_HDR_VXLAN] = {"Vxlan", 8, 4, {{"flags", 0, 7}, {"reserved", 8, 31}, {"vni", 32, 55}, {"reserved2", 56, 63}}},
    [PKT_HDR_DOT3] = {"Dot3", 14, 3, {{"dst", 0, 47}, {"src", 48, 95}, {"length", 96, 111}}},
    [PKT_HDR_LLC] = {"LLC", 3, 3, {{"dsap", 0, 7}, {"ssap", 8, 15}, {"ctrl", 16, 23}}},
    [PKT_HDR_SNAP] = {"SNAP", 5, 2, {{"oui", 0, 23}, {"code", 24, 39}}},
    [PKT_HDR_GRE] = {"GRE", 4, 9,
                     {{"chksum_present", 0, 0}, {"routing_present", 1, 1}, {"key_present", 2, 2},
                      {"seqnum_present", 3, 3}, {"strict_route_src", 4, 4}, {"recurse", 5, 7},
                      {"flags", 8, 12}, {"version", 13, 15}, {"proto", 16, 31}}},
    [PKT_HDR_GRE_CHKSUM_OFFSET] = {"GREChksumOffset", 4, 2, {{"chksum", 0, 15}, {"offset", 16, 31}}},
    [PKT_HDR_GRE_SEQUENCE_NUM] = {"GRESequenceNum", 4, 1, {{"seqnum", 0, 31}}},
    [PKT_HDR_GRE_KEY] = {"GREKey", 4, 1, {{"key", 0, 31}}},
    [PKT_HDR_ERSPAN2] = {"ERSPAN2", 8, 8,
                         {{"version", 0, 3}, {"vlan", 4, 15}, {"cos", 16, 18}, {"en", 19, 20}, {"t", 21, 21},
                          {"session_id", 22, 31}, {"reserved", 32, 43}, {"index", 44, 63}}},
    [PKT_HDR_ERSPAN3] = {"ERSPAN3", 12, 14,
                         {{"version", 0, 3}, {"vlan", 4, 15}, {"cos", 16, 18}, {"bos", 19, 20}, {"t", 21, 21},
                          {"session_id", 22, 31}, {"timestamp", 32, 63}, {"sgt", 64, 79}, {"p", 80, 80},
                          {"ft", 81, 85}, {"hw_id", 86, 91}, {"d", 92, 92}, {"gra", 93, 94}, {"o", 95, 95}}},
    [PKT_HDR_ERSPAN_PLATFORM] = {"ERSPANPLATFORM", 8, 2, {{"id", 0, 5}, {"info", 6, 63}}},
    [PKT_HDR_STP] = {"STP", 35, 14,
                     {{"proto", 0, 15}, {"version", 16, 23}, {"bpdu_type", 24, 31}, {"flags", 32, 39},
                      {"root_id", 40, 55}, {"root_mac", 56, 103}, {"root_path_cost", 104, 135},
                      {"bridge_id", 136, 151}, {"bridge_mac", 152, 199}, {"port_id", 200, 215},
                      {"message_age", 216, 231}, {"max_age", 232, 247}, {"hello_time", 248, 263},
                      {"fwd_delay", 264, 279}}},
    [PKT_HDR_MPLS] = {"MPLS", 4, 4, {{"label", 0, 19}, {"exp", 20, 22}, {"bos", 23, 23}, {"ttl", 24, 31}}},
};

const char *orc_hdr_name(int t) { return (t > 0 && t < PKT_HDR_COUNT) ? ORC_HDRS[t].name : NULL; }
int orc_hdr_size(int t) { return (t > 0 && t < PKT_HDR_COUNT) ? ORC_HDRS[t].size : 0; }
int orc_hdr_field_count(int t) { return (t > 0 && t < PKT_HDR_COUNT) ? ORC_HDRS[t].nfields : 0; }
int orc_hdr_field(int t, int i, const char **name, uint16_t *start, uint16_t *end) {
    if (t <= 0 || t >= PKT_HDR_COUNT || i < 0 || i >= ORC_HDRS[t].nfields) return -1;
    *name = ORC_HDRS[t].f[i].name;
    *start = ORC_HDRS[t].f[i].start;
    *end = ORC_HDRS[t].f[i].end;
    return 0;
}

/* ------------------------------------------------------------------ bit_range */
/* headers.rs:253-263.  `map` is the header slice; msb/lsb are bit numbers counted MSB-first
 * from map[0].  Rust release semantics for the final shifts: the shift amount
 * (64 - width) wraps as usize and is masked to 6 bits by the shl/shr instructions. */
uint64_t orc_bit_range(const uint8_t *map, size_t msb, size_t lsb) {
    const size_t bit_len = 8, value_bit_len = 64;
    uint64_t value = 0;
    for (size_t i = lsb; i <= msb; i++) {
        value <<= 1;
        value |= (uint64_t)((map[i / bit_len] >> (bit_len - i % bit_len - 1)) & 1);
    }
    size_t sh = (value_bit_len - (msb - lsb + 1)) & 63; /* Q8: wrapping usize, masked shift */
    return value << sh >> sh;
}

/* headers.rs:202-211 — bytes(msb, lsb), one bit_range per byte. */
void orc_bytes(const uint8_t *map, size_t msb, size_t lsb, uint8_t *out) {
    size_t k = 0;
    for (size_t i = lsb; i <= msb; i += 8) out[k++] = (uint8_t)orc_bit_range(map, i + 7, i);
}

/* ------------------------------------------------------------------ ipv4_checksum */
/* packet.rs:93-107, including `(chksum >> 16) + chksum & 0xFFFF`, which Rust parses as
 * `((chksum >> 16) + chksum) & 0xFFFF` (Q1: the end-around carry of hi+lo is dropped). */
uint16_t orc_ipv4_checksum(const uint8_t *v, size_t len) {
    uint32_t chksum = 0;
    for (size_t i = 0; i < len; i += 2) {
        if (i == 10) continue;
        uint16_t msb = (uint16_t)((uint16_t)v[i] << 8);
        chksum += (uint32_t)msb | (uint32_t)v[i + 1];
    }
    while ((chksum >> 16) != 0) chksum = ((chksum >> 16) + chksum) & 0xFFFF;
    return (uint16_t)~(uint16_t)chksum;
}

/* ------------------------------------------------------------------ PacketSlice */
/* One `Box<dyn Header>` = a heap node holding the slice (type + position). */
typedef struct { int type; size_t off; } orc_hdr_box_t;

typedef struct {
    orc_hdr_box_t **hdrs; /* Vec<Box<dyn Header>> */
    size_t n, cap;
    size_t payload_off, payload_len;
} orc_pslice_t;

/* PacketSlice::insert (packet.rs:724-726): Vec::insert(0, Box::new(hdr)). */
static int ps_insert(orc_pslice_t *ps, int type, size_t off) {
    orc_hdr_box_t *b = (orc_hdr_box_t *)malloc(sizeof(*b));
    if (!b) return -1;
    b->type = type;
    b->off = off;
    if (ps->n == ps->cap) {
        size_t nc = ps->cap ? ps->cap * 2 : 4;
        orc_hdr_box_t **nh = (orc_hdr_box_t **)realloc(ps->hdrs, nc * sizeof(*nh));
        if (!nh) { free(b); return -1; }
        ps->hdrs = nh;
        ps->cap = nc;
    }
    memmove(ps->hdrs + 1, ps->hdrs, ps->n * sizeof(*ps->hdrs));
    ps->hdrs[0] = b;
    ps->n++;
    return 0;
}

static void ps_free(orc_pslice_t *ps) {
    for (size_t i = 0; i < ps->n; i++) free(ps->hdrs[i]);
    free(ps->hdrs);
    ps->hdrs = NULL;
    ps->n = ps->cap = 0;
}

/* The walk.  `p`/`plen` is the whole packet; each function sees arr = p + off with
 * arr.len() = plen - off, exactly like the reference's re-sliced `&arr[X::size()..]`.
 * Return codes: 0 ok, PKT_TRUNCATED where Rust would panic, PKT_DEPTH_LIMIT when the
 * number of headers entered (in forward order) would exceed PKT_MAX_HDRS. */
typedef struct {
    const uint8_t *p;
    size_t plen;
    int entered;
} walk_t;

#define ARR_LEN(w, off) ((w)->plen - (off))
/* `&arr[0..k]` / `&arr[k..]` / `arr[k-1]`: panic unless k <= arr.len() */
#define NEED(w, off, k)                          \
    do {                                         \
        if ((size_t)(k) > ARR_LEN(w, off)) return PKT_TRUNCATED; \
    } while (0)
#define ENTER(w)                                         \
    do {                                                 \
        if ((w)->entered >= PKT_MAX_HDRS) return PKT_DEPTH_LIMIT; \
        (w)->entered++;                                  \
    } while (0)
#define TRY(x)                  \
    do {                        \
        int rc_ = (x);          \
        if (rc_) return rc_;    \
    } while (0)
#define INSERT(ps, t, off) TRY(ps_insert((ps), (t), (off)) ? PKT_TRUNCATED : 0)

static int w_parse(walk_t *w, size_t off, orc_pslice_t *ps);
static int w_dot3(walk_t *w, size_t off, orc_pslice_t *ps);
static int w_llc(walk_t *w, size_t off, orc_pslice_t *ps);
static int w_snap(walk_t *w, size_t off, orc_pslice_t *ps);
static int w_ethernet(walk_t *w, size_t off, orc_pslice_t *ps);
static int w_vlan(walk_t *w, size_t off, orc_pslice_t *ps);
static int w_mpls(walk_t *w, size_t off, orc_pslice_t *ps);
static int w_mpls_bos(walk_t *w, size_t off, orc_pslice_t *ps);
static int w_ipv4(walk_t *w, size_t off, orc_pslice_t *ps);
static int w_ipv6(walk_t *w, size_t off, orc_pslice_t *ps);
static int w_gre(walk_t *w, size_t off, orc_pslice_t *ps);
static int w_erspan2(walk_t *w, size_t off, orc_pslice_t *ps);
static int w_erspan3(walk_t *w, size_t off, orc_pslice_t *ps);
static int w_arp(walk_t *w, size_t off, orc_pslice_t *ps);
static int w_icmp(walk_t *w, size_t off, orc_pslice_t *ps);
static int w_tcp(walk_t *w, size_t off, orc_pslice_t *ps);
static int w_udp(walk_t *w, size_t off, orc_pslice_t *ps);
static int w_vxlan(walk_t *w, size_t off, orc_pslice_t *ps);

/* fast.rs:223-227 */
static int w_accept(walk_t *w, size_t off, orc_pslice_t *ps) {
    ps->payload_off = off;
    ps->payload_len = ARR_LEN(w, off);
    return 0;
}

/* Getter on a header slice: `<Hdr>Slice::<field>()` = bit_range(end, start). */
static uint64_t getf(walk_t *w, size_t off, int t, int field_idx) {
    const orc_field_t *f = &ORC_HDRS[t].f[field_idx];
    return orc_bit_range(w->p + off, f->end, f->start);
}

/* fast.rs:5-12 */
static int w_parse(walk_t *w, size_t off, orc_pslice_t *ps) {
    NEED(w, off, 14); /* arr[12], arr[13] */
    uint16_t length = (uint16_t)(((uint16_t)w->p[off + 12] << 8) | w->p[off + 13]);
    if (length < 1500) return w_dot3(w, off, ps);
    return w_ethernet(w, off, ps);
}
/* fast.rs:13-18 */
static int w_dot3(walk_t *w, size_t off, orc_pslice_t *ps) {
    NEED(w, off, 14);
    ENTER(w);
    TRY(w_llc(w, off + 14, ps));
    INSERT(ps, PKT_HDR_DOT3, off);
    return 0;
}
/* fast.rs:19-28 */
static int w_llc(walk_t *w, size_t off, orc_pslice_t *ps) {
    NEED(w, off, 3);
    ENTER(w);
    const uint8_t *a = w->p + off;
    if (a[0] == 0xAA && a[1] == 0xAA && a[2] == 0x03)
        TRY(w_snap(w, off + 3, ps));
    else
        TRY(w_accept(w, off + 3, ps));
    INSERT(ps, PKT_HDR_LLC, off);
    return 0;
}
/* fast.rs:29-34 */
static int w_snap(walk_t *w, size_t off, orc_pslice_t *ps) {
    NEED(w, off, 5);
    ENTER(w);
    TRY(w_accept(w, off + 5, ps));
    INSERT(ps, PKT_HDR_SNAP, off);
    return 0;
}
/* EtherType dispatch shared by fast.rs:37-45 and 51-59 (types.rs:51-75). */
static int w_etype_next(walk_t *w, size_t off, uint16_t etype, orc_pslice_t *ps) {
    switch (etype) {
    case 0x8100: return w_vlan(w, off, ps);
    case 0x0806: return w_arp(w, off, ps);
    case 0x0800: return w_ipv4(w, off, ps);
    case 0x86DD: return w_ipv6(w, off, ps);
    case 0x8847: return w_mpls(w, off, ps);
    default: return w_accept(w, off, ps); /* incl. ERSPANII/III and unknown values */
    }
}
/* fast.rs:35-48 */
static int w_ethernet(walk_t *w, size_t off, orc_pslice_t *ps) {
    NEED(w, off, 14);
    ENTER(w);
    uint16_t etype = (uint16_t)getf(w, off, PKT_HDR_ETHER, 2);
    TRY(w_etype_next(w, off + 14, etype, ps));
    INSERT(ps, PKT_HDR_ETHER, off);
    return 0;
}
/* fast.rs:49-62 */
static int w_vlan(walk_t *w, size_t off, orc_pslice_t *ps) {
    NEED(w, off, 4);
    ENTER(w);
    uint16_t etype = (uint16_t)getf(w, off, PKT_HDR_VLAN, 3);
    TRY(w_etype_next(w, off + 4, etype, ps));
    INSERT(ps, PKT_HDR_VLAN, off);
    return 0;
}
/* fast.rs:63-73 */
static int w_mpls(walk_t *w, size_t off, orc_pslice_t *ps) {
    NEED(w, off, 4);
    ENTER(w);
    uint64_t bos = getf(w, off, PKT_HDR_MPLS, 2);
    if (bos == 1)
        TRY(w_mpls_bos(w, off + 4, ps));
    else
        TRY(w_mpls(w, off + 4, ps));
    INSERT(ps, PKT_HDR_MPLS, off);
    return 0;
}
/* fast.rs:74-83: the 4 bytes after a bos label are another MPLS header (Q3), then the
 * high nibble of arr[4] picks IPv4 / IPv6 / Ethernet (types.rs:9-23). */
static int w_mpls_bos(walk_t *w, size_t off, orc_pslice_t *ps) {
    NEED(w, off, 4);
    ENTER(w);
    NEED(w, off, 5); /* arr[MPLS::size()] */
    uint8_t nib = (uint8_t)((w->p[off + 4] >> 4) & 0xf);
    if (nib == 4)
        TRY(w_ipv4(w, off + 4, ps));
    else if (nib == 6)
        TRY(w_ipv6(w, off + 4, ps));
    else
        TRY(w_ethernet(w, off + 4, ps));
    INSERT(ps, PKT_HDR_MPLS, off);
    return 0;
}
/* fast.rs:84-98 (Q4: ihl ignored; Q6: proto 58 -> payload) */
static int w_ipv4(walk_t *w, size_t off, orc_pslice_t *ps) {
    NEED(w, off, 20);
    ENTER(w);
    uint8_t proto = (uint8_t)getf(w, off, PKT_HDR_IPV4, 8);
    size_t n = off + 20;
    switch (proto) {
    case 1: TRY(w_icmp(w, n, ps)); break;
    case 4: TRY(w_ipv4(w, n, ps)); break;
    case 6: TRY(w_tcp(w, n, ps)); break;
    case 17: TRY(w_udp(w, n, ps)); break;
    case 41: TRY(w_ipv6(w, n, ps)); break;
    case 47: TRY(w_gre(w, n, ps)); break;
    default: TRY(w_accept(w, n, ps)); break;
    }
    INSERT(ps, PKT_HDR_IPV4, off);
    return 0;
}
/* fast.rs:99-113 (Q6: next_hdr 1 -> payload, 58 -> ICMP) */
static int w_ipv6(walk_t *w, size_t off, orc_pslice_t *ps) {
    NEED(w, off, 40);
    ENTER(w);
    uint8_t nh = (uint8_t)getf(w, off, PKT_HDR_IPV6, 4);
    size_t n = off + 40;
    switch (nh) {
    case 58: TRY(w_icmp(w, n, ps)); break;
    case 4: TRY(w_ipv4(w, n, ps)); break;
    case 6: TRY(w_tcp(w, n, ps)); break;
    case 17: TRY(w_udp(w, n, ps)); break;
    case 41: TRY(w_ipv6(w, n, ps)); break;
    case 47: TRY(w_gre(w, n, ps)); break;
    default: TRY(w_accept(w, n, ps)); break;
    }
    INSERT(ps, PKT_HDR_IPV6, off);
    return 0;
}
/* fast.rs:114-165.  Options are sliced in wire order C, K, S, then inserted C, K, S, GRE,
 * so the list reads GRE, SeqNum, Key, ChksumOffset (Q2). */
static int w_gre(walk_t *w, size_t off, orc_pslice_t *ps) {
    NEED(w, off, 4);
    ENTER(w);
    uint16_t proto = (uint16_t)getf(w, off, PKT_HDR_GRE, 8);
    uint64_t c = getf(w, off, PKT_HDR_GRE, 0);
    uint64_t s = getf(w, off, PKT_HDR_GRE, 3);
    uint64_t k = getf(w, off, PKT_HDR_GRE, 2);
    size_t o = 4;
    long gco = -1, gk = -1, gsn = -1;
    if (c == 1) { NEED(w, off, o + 4); ENTER(w); gco = (long)(off + o); o += 4; }
    if (k == 1) { NEED(w, off, o + 4); ENTER(w); gk = (long)(off + o); o += 4; }
    if (s == 1) { NEED(w, off, o + 4); ENTER(w); gsn = (long)(off + o); o += 4; }
    size_t n = off + o;
    switch (proto) {
    case 0x0800: TRY(w_ipv4(w, n, ps)); break;
    case 0x86DD: TRY(w_ipv6(w, n, ps)); break;
    case 0x88be: TRY(w_erspan2(w, n, ps)); break;
    case 0x22eb: TRY(w_erspan3(w, n, ps)); break;
    default: TRY(w_accept(w, n, ps)); break;
    }
    if (gco >= 0) INSERT(ps, PKT_HDR_GRE_CHKSUM_OFFSET, (size_t)gco);
    if (gk >= 0) INSERT(ps, PKT_HDR_GRE_KEY, (size_t)gk);
    if (gsn >= 0) INSERT(ps, PKT_HDR_GRE_SEQUENCE_NUM, (size_t)gsn);
    INSERT(ps, PKT_HDR_GRE, off);
    return 0;
}
/* fast.rs:166-171 */
static int w_erspan2(walk_t *w, size_t off, orc_pslice_t *ps) {
    NEED(w, off, 8);
    ENTER(w);
    TRY(w_ethernet(w, off + 8, ps));
    INSERT(ps, PKT_HDR_ERSPAN2, off);
    return 0;
}
/* fast.rs:172-192 */
static int w_erspan3(walk_t *w, size_t off, orc_pslice_t *ps) {
    NEED(w, off, 12);
    ENTER(w);
    uint64_t o = getf(w, off, PKT_HDR_ERSPAN3, 13);
    size_t k = 12;
    long plat = -1;
    if (o == 1) { NEED(w, off, k + 8); ENTER(w); plat = (long)(off + k); k += 8; }
    TRY(w_ethernet(w, off + k, ps));
    if (plat >= 0) INSERT(ps, PKT_HDR_ERSPAN_PLATFORM, (size_t)plat);
    INSERT(ps, PKT_HDR_ERSPAN3, off);
    return 0;
}
/* fast.rs:193-197 */
static int w_arp(walk_t *w, size_t off, orc_pslice_t *ps) {
    NEED(w, off, 28);
    ENTER(w);
    TRY(w_accept(w, off + 28, ps));
    INSERT(ps, PKT_HDR_ARP, off);
    return 0;
}
/* fast.rs:198-202 (ICMP::size() = 4, Q13) */
static int w_icmp(walk_t *w, size_t off, orc_pslice_t *ps) {
    NEED(w, off, 4);
    ENTER(w);
    TRY(w_accept(w, off + 4, ps));
    INSERT(ps, PKT_HDR_ICMP, off);
    return 0;
}
/* fast.rs:203-207 (Q4: data offset ignored) */
static int w_tcp(walk_t *w, size_t off, orc_pslice_t *ps) {
    NEED(w, off, 20);
    ENTER(w);
    TRY(w_accept(w, off + 20, ps));
    INSERT(ps, PKT_HDR_TCP, off);
    return 0;
}
/* fast.rs:208-217 (types.rs:7 UDP_PORT_VXLAN = 4789, on the DESTINATION port) */
static int w_udp(walk_t *w, size_t off, orc_pslice_t *ps) {
    NEED(w, off, 8);
    ENTER(w);
    uint16_t dst = (uint16_t)getf(w, off, PKT_HDR_UDP, 1);
    if (dst == 4789)
        TRY(w_vxlan(w, off + 8, ps));
    else
        TRY(w_accept(w, off + 8, ps));
    INSERT(ps, PKT_HDR_UDP, off);
    return 0;
}
/* fast.rs:218-222 */
static int w_vxlan(walk_t *w, size_t off, orc_pslice_t *ps) {
    NEED(w, off, 8);
    ENTER(w);
    TRY(w_ethernet(w, off + 8, ps));
    INSERT(ps, PKT_HDR_VXLAN, off);
    return 0;
}

typedef int (*walk_fn)(walk_t *, size_t, orc_pslice_t *);
static const walk_fn ENTRY_FNS[PKT_ENTRY_COUNT] = {
    w_parse, w_dot3, w_llc, w_snap, w_ethernet, w_vlan, w_mpls, w_mpls_bos, w_ipv4,
    w_ipv6, w_gre, w_erspan2, w_erspan3, w_arp, w_icmp, w_tcp, w_udp, w_vxlan,
};

/* ------------------------------------------------------------------ batch driver */
#define PUT(col, i, v) do { if (out->col) out->col[i] = (v); } while (0)

static void zero_fields(const pkt_out_t *o, uint64_t i) {
    const pkt_out_t *out = o;
    PUT(eth_dst, i, 0); PUT(eth_src, i, 0); PUT(eth_etype, i, 0);
    PUT(vlan_pcp, i, 0); PUT(vlan_cfi, i, 0); PUT(vlan_vid, i, 0); PUT(vlan_etype, i, 0);
    PUT(ipv4_version, i, 0); PUT(ipv4_ihl, i, 0); PUT(ipv4_diffserv, i, 0);
    PUT(ipv4_total_len, i, 0); PUT(ipv4_identification, i, 0); PUT(ipv4_flags, i, 0);
    PUT(ipv4_frag_startset, i, 0); PUT(ipv4_ttl, i, 0); PUT(ipv4_protocol, i, 0);
    PUT(ipv4_header_checksum, i, 0); PUT(ipv4_src, i, 0); PUT(ipv4_dst, i, 0);
    PUT(ipv4_csum_calc, i, 0);
    PUT(ipv6_version, i, 0); PUT(ipv6_traffic_class, i, 0); PUT(ipv6_flow_label, i, 0);
    PUT(ipv6_payload_len, i, 0); PUT(ipv6_next_hdr, i, 0); PUT(ipv6_hop_limit, i, 0);
    if (out->ipv6_src) memset(out->ipv6_src + i * 16, 0, 16);
    if (out->ipv6_dst) memset(out->ipv6_dst + i * 16, 0, 16);
    PUT(tcp_src, i, 0); PUT(tcp_dst, i, 0); PUT(tcp_seq_no, i, 0); PUT(tcp_ack_no, i, 0);
    PUT(tcp_data_startset, i, 0); PUT(tcp_res, i, 0); PUT(tcp_flags, i, 0);
    PUT(tcp_window, i, 0); PUT(tcp_checksum, i, 0); PUT(tcp_urgent_ptr, i, 0);
    PUT(udp_src, i, 0); PUT(udp_dst, i, 0); PUT(udp_length, i, 0); PUT(udp_checksum, i, 0);
}

/* The getters of the FIRST header of each type (Packet's Index<&str>, packet.rs:64-66). */
static void fill_fields(const pkt_out_t *out, uint64_t i, const uint8_t *p, const orc_pslice_t *ps) {
    long first[PKT_HDR_COUNT];
    for (int t = 0; t < PKT_HDR_COUNT; t++) first[t] = -1;
    for (size_t j = 0; j < ps->n; j++)
        if (first[ps->hdrs[j]->type] < 0) first[ps->hdrs[j]->type] = (long)ps->hdrs[j]->off;
    zero_fields(out, i);
#define G(t, k) orc_bit_range(h, ORC_HDRS[t].f[k].end, ORC_HDRS[t].f[k].start)
    const uint8_t *h;
    if (first[PKT_HDR_ETHER] >= 0) {
        h = p + first[PKT_HDR_ETHER];
        PUT(eth_dst, i, G(PKT_HDR_ETHER, 0));
        PUT(eth_src, i, G(PKT_HDR_ETHER, 1));
        PUT(eth_etype, i, (uint16_t)G(PKT_HDR_ETHER, 2));
    }
    if (first[PKT_HDR_VLAN] >= 0) {
        h = p + first[PKT_HDR_VLAN];
        PUT(vlan_pcp, i, (uint8_t)G(PKT_HDR_VLAN, 0));
        PUT(vlan_cfi, i, (uint8_t)G(PKT_HDR_VLAN, 1));
        PUT(vlan_vid, i, (uint16_t)G(PKT_HDR_VLAN, 2));
        PUT(vlan_etype, i, (uint16_t)G(PKT_HDR_VLAN, 3));
    }
    if (first[PKT_HDR_IPV4] >= 0) {
        h = p + first[PKT_HDR_IPV4];
        PUT(ipv4_version, i, (uint8_t)G(PKT_HDR_IPV4, 0));
        PUT(ipv4_ihl, i, (uint8_t)G(PKT_HDR_IPV4, 1));
        PUT(ipv4_diffserv, i, (uint8_t)G(PKT_HDR_IPV4, 2));
        PUT(ipv4_total_len, i, (uint16_t)G(PKT_HDR_IPV4, 3));
        PUT(ipv4_identification, i, (uint16_t)G(PKT_HDR_IPV4, 4));
        PUT(ipv4_flags, i, (uint8_t)G(PKT_HDR_IPV4, 5));
        PUT(ipv4_frag_startset, i, (uint16_t)G(PKT_HDR_IPV4, 6));
        PUT(ipv4_ttl, i, (uint8_t)G(PKT_HDR_IPV4, 7));
        PUT(ipv4_protocol, i, (uint8_t)G(PKT_HDR_IPV4, 8));
        PUT(ipv4_header_checksum, i, (uint16_t)G(PKT_HDR_IPV4, 9));
        PUT(ipv4_src, i, (uint32_t)G(PKT_HDR_IPV4, 10));
        PUT(ipv4_dst, i, (uint32_t)G(PKT_HDR_IPV4, 11));
        PUT(ipv4_csum_calc, i, orc_ipv4_checksum(h, 20));
    }
    if (first[PKT_HDR_IPV6] >= 0) {
        h = p + first[PKT_HDR_IPV6];
        PUT(ipv6_version, i, (uint8_t)G(PKT_HDR_IPV6, 0));
        PUT(ipv6_traffic_class, i, (uint8_t)G(PKT_HDR_IPV6, 1));
        PUT(ipv6_flow_label, i, (uint32_t)G(PKT_HDR_IPV6, 2));
        PUT(ipv6_payload_len, i, (uint16_t)G(PKT_HDR_IPV6, 3));
        PUT(ipv6_next_hdr, i, (uint8_t)G(PKT_HDR_IPV6, 4));
        PUT(ipv6_hop_limit, i, (uint8_t)G(PKT_HDR_IPV6, 5));
        if (out->ipv6_src) orc_bytes(h, 191, 64, out->ipv6_src + i * 16);
        if (out->ipv6_dst) orc_bytes(h, 319, 192, out->ipv6_dst + i * 16);
    }
    if (first[PKT_HDR_TCP] >= 0) {
        h = p + first[PKT_HDR_TCP];
        PUT(tcp_src, i, (uint16_t)G(PKT_HDR_TCP, 0));
        PUT(tcp_dst, i, (uint16_t)G(PKT_HDR_TCP, 1));
        PUT(tcp_seq_no, i, (uint32_t)G(PKT_HDR_TCP, 2));
        PUT(tcp_ack_no, i, (uint32_t)G(PKT_HDR_TCP, 3));
        PUT(tcp_data_startset, i, (uint8_t)G(PKT_HDR_TCP, 4));
        PUT(tcp_res, i, (uint8_t)G(PKT_HDR_TCP, 5));
        PUT(tcp_flags, i, (uint8_t)G(PKT_HDR_TCP, 6));
        PUT(tcp_window, i, (uint16_t)G(PKT_HDR_TCP, 7));
        PUT(tcp_checksum, i, (uint16_t)G(PKT_HDR_TCP, 8));
        PUT(tcp_urgent_ptr, i, (uint16_t)G(PKT_HDR_TCP, 9));
    }
    if (first[PKT_HDR_UDP] >= 0) {
        h = p + first[PKT_HDR_UDP];
        PUT(udp_src, i, (uint16_t)G(PKT_HDR_UDP, 0));
        PUT(udp_dst, i, (uint16_t)G(PKT_HDR_UDP, 1));
        PUT(udp_length, i, (uint16_t)G(PKT_HDR_UDP, 2));
        PUT(udp_checksum, i, (uint16_t)G(PKT_HDR_UDP, 3));
    }
#undef G
}

/* Packet i of a batch (include/pktgpu.h, pkt_batch_t): its range clamped to the slab end and to
 * 65535 bytes.  This is the batch ABI's framing, not part of the reference's algorithm. */
static void packet_bounds(const pkt_batch_t *b, uint64_t i, const uint8_t **p, size_t *len) {
    uint64_t off, l;
    if (b->offsets) {
        off = b->offsets[i];
        l = b->lens[i];
    } else {
        off = i * (uint64_t)b->stride;
        l = b->lens ? b->lens[i] : b->stride;
    }
    uint64_t room = off < b->slab_len ? b->slab_len - off : 0;
    if (l > room) l = room;
    if (l > 0xFFFF) l = 0xFFFF;
    *p = b->slab + (off < b->slab_len ? off : 0);
    *len = (size_t)l;
}

int orc_parse_one(const uint8_t *p, size_t len, int entry, const pkt_out_t *out, uint64_t i, uint64_t n) {
    orc_pslice_t ps = {0};
    walk_t w = {p, len, 0};
    int st = ENTRY_FNS[entry](&w, 0, &ps);
    PUT(status, i, (uint8_t)st);
    if (st != PKT_OK) {
        PUT(n_hdrs, i, 0);
        PUT(payload_off, i, 0);
        PUT(payload_len, i, 0);
        PUT(hdr_mask, i, 0);
        zero_fields(out, i);
        ps_free(&ps);
        return st;
    }
    uint32_t mask = 0;
    for (size_t j = 0; j < ps.n; j++) {
        if (out->hdr_type) out->hdr_type[j * n + i] = (uint8_t)ps.hdrs[j]->type;
        if (out->hdr_off) out->hdr_off[j * n + i] = (uint16_t)ps.hdrs[j]->off;
        mask |= 1u << ps.hdrs[j]->type;
    }
    PUT(n_hdrs, i, (uint8_t)ps.n);
    PUT(payload_off, i, (uint16_t)ps.payload_off);
    PUT(payload_len, i, (uint16_t)ps.payload_len);
    PUT(hdr_mask, i, mask);
    fill_fields(out, i, p, &ps);
    ps_free(&ps);
    return st;
}

typedef struct {
    const pkt_batch_t *b;
    int entry;
    const pkt_out_t *out;
    uint64_t lo, hi;
} job_t;

static void *run_job(void *arg) {
    job_t *j = (job_t *)arg;
    for (uint64_t i = j->lo; i < j->hi; i++) {
        const uint8_t *p;
        size_t len;
        packet_bounds(j->b, i, &p, &len);
        orc_parse_one(p, len, j->entry, j->out, i, j->b->n);
    }
    return NULL;
}

int orc_parse_batch(const pkt_batch_t *b, int entry, const pkt_out_t *out, int nthreads) {
    if (!b || !out || entry < 0 || entry >= PKT_ENTRY_COUNT) return -1;
    if (b->n && !b->slab) return -1;
    if (b->offsets && !b->lens) return -1;
    if (nthreads < 1) nthreads = 1;
    if ((uint64_t)nthreads > b->n) nthreads = b->n ? (int)b->n : 1;
    if (nthreads == 1) {
        job_t j = {b, entry, out, 0, b->n};
        run_job(&j);
        return 0;
    }
    pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
    job_t *jobs = (job_t *)calloc((size_t)nthreads, sizeof(job_t));
    if (!th || !jobs) { free(th); free(jobs); return -1; }
    for (int t = 0; t < nthreads; t++) {
        jobs[t] = (job_t){b, entry, out, b->n * (uint64_t)t / (uint64_t)nthreads,
                          b->n * (uint64_t)(t + 1) / (uint64_t)nthreads};
        pthread_create(&th[t], NULL, run_job, &jobs[t]);
    }
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    free(th);
    free(jobs);
    return 0;
}

/* ------------------------------------------------------------------ field getters */
/* `<Hdr>Slice::<field>()` on the occurrence-th header of a type in the chain. */
int orc_extract_fields(const pkt_batch_t *b, const pkt_chain_t *chain, const pkt_field_spec_t *specs,
                       uint32_t nspec, uint64_t *const *values, uint8_t *const *found) {
    for (uint64_t i = 0; i < b->n; i++) {
        const uint8_t *p;
        size_t len;
        packet_bounds(b, i, &p, &len);
        for (uint32_t s = 0; s < nspec; s++) {
            int occ = 0, hit = -1;
            for (int j = 0; j < chain->n_hdrs[i]; j++) {
                if (chain->hdr_type[(uint64_t)j * b->n + i] == specs[s].hdr_type) {
                    if (occ == specs[s].occurrence) { hit = j; break; }
                    occ++;
                }
            }
            uint64_t v = 0;
            if (hit >= 0) v = orc_bit_range(p + chain->hdr_off[(uint64_t)hit * b->n + i], specs[s].end, specs[s].start);
            values[s][i] = v;
            if (found && found[s]) found[s][i] = hit >= 0;
        }
    }
    return 0;
}

/* ------------------------------------------------------------------ slow::parse round trip */
/* Config 1: slow::parse (slow.rs) builds the same list from owned copies
 * (`arr[..].to_vec()`), and Packet::to_vec (packet.rs:385-392) concatenates each header's
 * bytes in list order, then the payload.  Returns the serialised length, or -status. */
long orc_slow_parse_to_vec(const uint8_t *p, size_t len, int entry, uint8_t *out, size_t cap) {
    orc_pslice_t ps = {0};
    walk_t w = {p, len, 0};
    int st = ENTRY_FNS[entry](&w, 0, &ps);
    if (st != PKT_OK) { ps_free(&ps); return -st; }
    size_t k = 0;
    for (size_t j = 0; j < ps.n; j++) {
        int sz = ORC_HDRS[ps.hdrs[j]->type].size;
        uint8_t *owned = (uint8_t *)malloc((size_t)sz); /* X::from(arr[..].to_vec()) */
        memcpy(owned, p + ps.hdrs[j]->off, (size_t)sz);
        if (k + (size_t)sz <= cap) memcpy(out + k, owned, (size_t)sz);
        k += (size_t)sz;
        free(owned);
    }
    if (k + ps.payload_len <= cap) memcpy(out + k, p + ps.payload_off, ps.payload_len);
    k += ps.payload_len;
    ps_free(&ps);
    return (long)k;
}

/* PacketSlice::to_vec (packet.rs:733-740) after fast::parse: the header slices in list order,
 * then the payload — no owned copies (tests/lib.rs:804-817 parse_slice_test). */
static long fast_parse_to_vec(const uint8_t *p, size_t len, int entry, uint8_t *out, size_t cap) {
    orc_pslice_t ps = {0};
    walk_t w = {p, len, 0};
    int st = ENTRY_FNS[entry](&w, 0, &ps);
    if (st != PKT_OK) { ps_free(&ps); return -st; }
    size_t k = 0;
    for (size_t j = 0; j < ps.n; j++) {
        size_t sz = (size_t)ORC_HDRS[ps.hdrs[j]->type].size;
        if (k + sz <= cap) memcpy(out + k, p + ps.hdrs[j]->off, sz);
        k += sz;
    }
    if (k + ps.payload_len <= cap) memcpy(out + k, p + ps.payload_off, ps.payload_len);
    k += ps.payload_len;
    ps_free(&ps);
    return (long)k;
}

typedef struct {
    const pkt_batch_t *b;
    int entry, slow;
    uint8_t *dst;
    uint64_t dst_len;
    uint32_t *out_len;
    uint64_t lo, hi;
} rt_job_t;

static void *run_rt_job(void *arg) {
    rt_job_t *j = (rt_job_t *)arg;
    for (uint64_t i = j->lo; i < j->hi; i++) {
        const uint8_t *p;
        size_t len;
        packet_bounds(j->b, i, &p, &len);
        const uint64_t o = j->b->offsets ? j->b->offsets[i] : i * (uint64_t)j->b->stride;
        const size_t cap = o < j->dst_len ? (size_t)(j->dst_len - o) : 0;
        long k = j->slow ? orc_slow_parse_to_vec(p, len, j->entry, j->dst + o, cap)
                         : fast_parse_to_vec(p, len, j->entry, j->dst + o, cap);
        if (j->out_len) j->out_len[i] = k > 0 ? (uint32_t)k : 0;
    }
    return NULL;
}

/* Batched round trip, the CPU baseline of tests/lib.rs:790-817: for every packet,
 * slow::parse(..).to_vec() (slow = 1, parse_test) or fast::parse(..).to_vec() (slow = 0,
 * parse_slice_test), written at the packet's own position in dst (i*stride or offsets[i]).
 * out_len[i] = bytes written (0 when the reference would panic). */
int orc_round_trip_batch(const pkt_batch_t *b, int entry, int slow, uint8_t *dst, uint64_t dst_len,
                         uint32_t *out_len, int nthreads) {
    if (!b || !dst || entry < 0 || entry >= PKT_ENTRY_COUNT) return -1;
    if (b->n && !b->slab) return -1;
    if (b->offsets && !b->lens) return -1;
    if (nthreads < 1) nthreads = 1;
    if ((uint64_t)nthreads > b->n) nthreads = b->n ? (int)b->n : 1;
    pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
    rt_job_t *jobs = (rt_job_t *)calloc((size_t)nthreads, sizeof(rt_job_t));
    if (!th || !jobs) { free(th); free(jobs); return -1; }
    for (int t = 0; t < nthreads; t++) {
        jobs[t] = (rt_job_t){b, entry, slow, dst, dst_len, out_len, b->n * (uint64_t)t / (uint64_t)nthreads,
                             b->n * (uint64_t)(t + 1) / (uint64_t)nthreads};
        if (nthreads > 1) pthread_create(&th[t], NULL, run_rt_job, &jobs[t]);
    }
    if (nthreads == 1) run_rt_job(&jobs[0]);
    else for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    free(th);
    free(jobs);
    return 0;
}

/* ------------------------------------------------------------------ header rewrite */
/* headers.rs:315-324 — set_bit_range: for i in (lsb..=msb).rev(): bit i := value & 1;
 * value >>= 1 (one bit at a time, with the lock-free slice here). */
void orc_set_bit_range(uint8_t *map, size_t msb, size_t lsb, uint64_t value) {
    const size_t bit_len = 8;
    for (size_t i = msb + 1; i-- > lsb;) {
        map[i / bit_len] &= (uint8_t)~(1u << (bit_len - i % bit_len - 1));
        map[i / bit_len] |= (uint8_t)((value & 1) << (bit_len - i % bit_len - 1));
        value >>= 1;
    }
}

static int find_hdr(const pkt_chain_t *c, uint64_t n, uint64_t i, int type, int occurrence) {
    int occ = 0;
    for (int j = 0; j < c->n_hdrs[i]; j++)
        if (c->hdr_type[(uint64_t)j * n + i] == type) {
            if (occ == occurrence) return j;
            occ++;
        }
    return -1;
}

/* Batched setters in spec order, in place (slab is written through b->slab). */
int orc_set_fields(const pkt_batch_t *b, const pkt_chain_t *chain, const pkt_field_spec_t *specs,
                   uint32_t nspec, const uint64_t *const *values) {
    uint8_t *slab = (uint8_t *)b->slab;
    for (uint64_t i = 0; i < b->n; i++) {
        uint64_t off = b->offsets ? b->offsets[i] : i * (uint64_t)b->stride;
        for (uint32_t s = 0; s < nspec; s++) {
            int j = find_hdr(chain, b->n, i, specs[s].hdr_type, specs[s].occurrence);
            if (j < 0) continue;
            orc_set_bit_range(slab + off + chain->hdr_off[(uint64_t)j * b->n + i], specs[s].end,
                              specs[s].start, values[s][i]);
        }
    }
    return 0;
}

/* utils.rs:233-236: ipv4.set_header_checksum(Packet::ipv4_checksum(ipv4.to_vec())) */
int orc_ipv4_update_checksum(const pkt_batch_t *b, const pkt_chain_t *chain, uint32_t occurrence) {
    uint8_t *slab = (uint8_t *)b->slab;
    for (uint64_t i = 0; i < b->n; i++) {
        int j = find_hdr(chain, b->n, i, PKT_HDR_IPV4, (int)occurrence);
        if (j < 0) continue;
        uint64_t off = b->offsets ? b->offsets[i] : i * (uint64_t)b->stride;
        uint8_t *h = slab + off + chain->hdr_off[(uint64_t)j * b->n + i];
        orc_set_bit_range(h, 95, 80, orc_ipv4_checksum(h, 20));
    }
    return 0;
}

/* ------------------------------------------------------------------ pktgen loop (CPU baseline) */
/* tests/lib.rs:756-788 pktgen_perf_test on the owned Packet model: Packet { hdrs: Vec<Box<dyn
 * Header>>, payload: Vec<u8> } (lib.rs:129-134) with every header's bytes behind an
 * Arc<Mutex<Vec<u8>>> (headers.rs:297-302).
 *   clone   (mode 0): p = pkt.clone() (packet.rs:393-400: a Box per header, the Arc shared — Q13 —
 *                     and the payload Vec copied), then p.to_vec() (packet.rs:385-392: one Vec
 *                     grown header by header, each header's mutex locked to read it).
 *   update  (mode 1): pkt["Ether"].set_etype(i % 0xFFFF) first — set_bit_range locks the header's
 *                     mutex once per bit (headers.rs:315-324) — then the clone as above.
 * Packet i's bytes go to out + i*stride (so the GPU generator's output can be compared with it).
 * Each thread owns its own Packet (the reference loop is single-threaded). */
typedef struct {
    pthread_mutex_t mu;
    int refs;
    uint8_t *data;
    size_t size;
} orc_owned_hdr_t;

typedef struct {
    const uint8_t *tpl;
    size_t len, payload_off;
    const uint8_t *types;
    const uint16_t *offs;
    int nh, mode;
    uint8_t *out;
    size_t stride;
    uint64_t lo, hi;
} pg_job_t;

static void *run_pg_job(void *arg) {
    pg_job_t *j = (pg_job_t *)arg;
    orc_owned_hdr_t *h = (orc_owned_hdr_t *)calloc((size_t)j->nh, sizeof(orc_owned_hdr_t));
    int ether = -1;
    for (int k = 0; k < j->nh; k++) {
        pthread_mutex_init(&h[k].mu, NULL);
        h[k].refs = 1;
        h[k].size = (size_t)ORC_HDRS[j->types[k]].size;
        h[k].data = (uint8_t *)malloc(h[k].size);
        memcpy(h[k].data, j->tpl + j->offs[k], h[k].size);
        if (ether < 0 && j->types[k] == PKT_HDR_ETHER) ether = k;
    }
    const size_t plen = j->len - j->payload_off;
    for (uint64_t i = j->lo; i < j->hi; i++) {
        if (j->mode == 1 && ether >= 0) {  /* set_etype: bits 96..111, one lock per bit */
            uint64_t v = i % 0xFFFF;
            for (size_t b = 112; b-- > 96;) {
                pthread_mutex_lock(&h[ether].mu);
                h[ether].data[b / 8] &= (uint8_t)~(1u << (7 - b % 8));
                h[ether].data[b / 8] |= (uint8_t)((v & 1) << (7 - b % 8));
                pthread_mutex_unlock(&h[ether].mu);
                v >>= 1;
            }
        }
        /* clone: a Box per header sharing the Arc, the payload copied */
        orc_owned_hdr_t ***box = (orc_owned_hdr_t ***)malloc((size_t)j->nh * sizeof(*box));
        for (int k = 0; k < j->nh; k++) {
            box[k] = (orc_owned_hdr_t **)malloc(sizeof(**box));
            *box[k] = &h[k];
            __atomic_add_fetch(&h[k].refs, 1, __ATOMIC_RELAXED);
        }
        uint8_t *payload = (uint8_t *)malloc(plen ? plen : 1);
        memcpy(payload, j->tpl + j->payload_off, plen);
        /* to_vec: Vec::new() grown by extend_from_slice */
        size_t cap = 0, n = 0;
        uint8_t *vec = NULL;
        for (int k = 0; k <= j->nh; k++) {
            const uint8_t *src;
            size_t sz;
            orc_owned_hdr_t *hh = NULL;
            if (k < j->nh) {
                hh = *box[k];
                pthread_mutex_lock(&hh->mu);
                src = hh->data;
                sz = hh->size;
            } else {
                src = payload;
                sz = plen;
            }
            if (n + sz > cap) {
                size_t nc = cap ? 2 * cap : 8;
                while (nc < n + sz) nc *= 2;
                vec = (uint8_t *)realloc(vec, nc);
                cap = nc;
            }
            memcpy(vec + n, src, sz);
            n += sz;
            if (hh) pthread_mutex_unlock(&hh->mu);
        }
        memcpy(j->out + i * j->stride, vec, n);
        free(vec);
        free(payload);
        for (int k = 0; k < j->nh; k++) {
            __atomic_sub_fetch(&(*box[k])->refs, 1, __ATOMIC_RELAXED);
            free(box[k]);
        }
        free(box);
    }
    for (int k = 0; k < j->nh; k++) {
        pthread_mutex_destroy(&h[k].mu);
        free(h[k].data);
    }
    free(h);
    return NULL;
}

int orc_pktgen_loop(const uint8_t *tpl, size_t len, int entry, int mode, uint64_t first, uint64_t cnt,
                    uint8_t *out, size_t stride, int nthreads) {
    if (!tpl || !out || stride < len || mode < 0 || mode > 1 || entry < 0 || entry >= PKT_ENTRY_COUNT) return -1;
    orc_pslice_t ps = {0};
    walk_t w = {tpl, len, 0};
    if (ENTRY_FNS[entry](&w, 0, &ps) != PKT_OK) { ps_free(&ps); return -1; }
    uint8_t types[64];
    uint16_t offs[64];
    int nh = (int)(ps.n < 64 ? ps.n : 64);
    for (int k = 0; k < nh; k++) {
        types[k] = (uint8_t)ps.hdrs[k]->type;
        offs[k] = (uint16_t)ps.hdrs[k]->off;
    }
    const size_t poff = ps.payload_off;
    ps_free(&ps);
    if (nthreads < 1) nthreads = 1;
    pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
    pg_job_t *jobs = (pg_job_t *)calloc((size_t)nthreads, sizeof(pg_job_t));
    if (!th || !jobs) { free(th); free(jobs); return -1; }
    for (int t = 0; t < nthreads; t++) {
        jobs[t] = (pg_job_t){tpl, len, poff, types, offs, nh, mode, out - first * stride, stride,
                             first + cnt * (uint64_t)t / (uint64_t)nthreads,
                             first + cnt * (uint64_t)(t + 1) / (uint64_t)nthreads};
        if (nthreads > 1) pthread_create(&th[t], NULL, run_pg_job, &jobs[t]);
    }
    if (nthreads == 1) run_pg_job(&jobs[0]);
    else for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    free(th);
    free(jobs);
    return 0;
}
