// pktgpu.hip — kernels and the C ABI (include/pktgpu.h) of the MI355X batched parser.
//
// Kernels
//   parse_kernel<NCH>       fast::parse_<entry> over a batch: per-lane windows of NCH 16-byte
//                           chunks staged in LDS, the chain walk, and the fused field/checksum
//                           extraction of the first Ether/Vlan/IPv4/IPv6/TCP/UDP (Q11).
//   parse_span_kernel<NCH>  the same with wave spans staged by LDS-DMA (pkt_ctx_set_staging 2).
// (getters / to_vec / setters over a parsed batch: pktgpu_rewrite.hip; the device pcap indexer:
// pktgpu_pcap.hip; packet generation: pktgpu_gen.hip)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <type_traits>

#include "pktgpu_ctx.hpp"
#include "pktgpu_device.hpp"

using namespace pktgpu;

namespace {

// Output column groups.  A kernel is specialised on GM = the groups whose columns are ALL
// requested (no per-column checks at all), or GM = G_RUNTIME (each column checked for NULL).
enum : uint32_t {
    G_CHAIN = 1, G_ETHER = 2, G_VLAN = 4, G_IPV4 = 8, G_IPV6 = 16, G_TCP = 32, G_UDP = 64,
    G_ALL = 127, G_RUNTIME = 128,
    // flag: store the columns non-temporally.  Set for the indexed-batch (lockstep) kernels: C4
    // isolated 105 -> 98 us, pipelined 86 -> 82.5 us, line requests 2.39M -> 2.29M (the columns
    // no longer evict the records' lines from L2); fixed-stride C2 keeps plain stores (pipelined
    // +0.3 us with them), profiles/ab/r02ntst_nt_column_stores.txt
    G_NT = 256
};

template <uint32_t GM, uint32_t G>
__device__ __forceinline__ bool want(const void* p) {
    if constexpr ((GM & G_RUNTIME) != 0) return p != nullptr;
    else return (GM & G) != 0;
}

// Store at a 32-bit byte offset from a column base (global_store ... saddr: one VGPR offset).
template <bool NT, class T>
__device__ __forceinline__ void st(T* base, uint32_t boff, T v) {
    if constexpr (NT && std::is_integral<T>::value)
        __builtin_nontemporal_store(v, reinterpret_cast<T*>(reinterpret_cast<char*>(base) + boff));
    else
        *reinterpret_cast<T*>(reinterpret_cast<char*>(base) + boff) = v;
}

// Record (type, offset) in header slot `slot` of packet i (slot-major columns, row stride ns = the
// batch size): 32-bit byte offsets from the column bases while every slot row of the batch lies
// within 4 GiB of them (ns <= 2^27, a wave-uniform branch), the 64-bit products beyond.
template <uint32_t GM>
__device__ __forceinline__ void push_slot(const pkt_out_t& out, uint64_t ns, uint32_t slot, uint32_t i, uint32_t ty,
                                          uint32_t o) {
    if (ns <= (1ull << 27)) {
        const uint32_t e = slot * (uint32_t)ns + i;
        if (want<GM, G_CHAIN>(out.hdr_type)) st<false, uint8_t>(out.hdr_type, e, (uint8_t)ty);
        if (want<GM, G_CHAIN>(out.hdr_off)) st<false, uint16_t>(out.hdr_off, 2u * e, (uint16_t)o);
    } else {
        if (want<GM, G_CHAIN>(out.hdr_type)) out.hdr_type[(uint64_t)slot * ns + i] = (uint8_t)ty;
        if (want<GM, G_CHAIN>(out.hdr_off)) out.hdr_off[(uint64_t)slot * ns + i] = (uint16_t)o;
    }
}

// Fields of the first header of each group (Q11), from the walk's first offsets.
// `i` is the packet index within this launch (< kLaunchChunk = 2^26, so every per-packet byte
// offset, up to i * 16 for the IPv6 addresses, fits 32 bits).
template <uint32_t GM, class View>
__device__ __forceinline__ void emit_fields(const pkt_out_t& out, uint32_t i, const View& pv,
                                            const WalkResult& r, bool ok) {
    const uint32_t o1 = i, o2 = i * 2u, o4 = i * 4u, o8 = i * 8u, o16 = i * 16u;
    // Ether (headers.rs:530-540): dst 0-47, src 48-95, etype 96-111
    if (want<GM, G_ETHER>(out.eth_dst) || want<GM, G_ETHER>(out.eth_src) || want<GM, G_ETHER>(out.eth_etype)) {
        uint32_t d[4] = {0, 0, 0, 0};
        const bool h = ok && r.f_eth >= 0;
        if (h) pv.template hdr<4>((uint32_t)r.f_eth, 14, d);
        if (want<GM, G_ETHER>(out.eth_dst)) st<(GM & G_NT) != 0, uint64_t>(out.eth_dst, o8, ((uint64_t)d[0] << 16) | (d[1] >> 16));
        if (want<GM, G_ETHER>(out.eth_src)) st<(GM & G_NT) != 0, uint64_t>(out.eth_src, o8, ((uint64_t)(d[1] & 0xFFFFu) << 32) | d[2]);
        if (want<GM, G_ETHER>(out.eth_etype)) st<(GM & G_NT) != 0, uint16_t>(out.eth_etype, o2, (uint16_t)(d[3] >> 16));
    }
    // Vlan (headers.rs:543-552): pcp 0-2, cfi 3, vid 4-15, etype 16-31
    if (want<GM, G_VLAN>(out.vlan_pcp) || want<GM, G_VLAN>(out.vlan_cfi) || want<GM, G_VLAN>(out.vlan_vid) ||
        want<GM, G_VLAN>(out.vlan_etype)) {
        uint32_t d[1] = {0};
        if (ok && r.f_vlan >= 0) pv.template hdr<1>((uint32_t)r.f_vlan, 4, d);
        if (want<GM, G_VLAN>(out.vlan_pcp)) st<(GM & G_NT) != 0, uint8_t>(out.vlan_pcp, o1, (uint8_t)(d[0] >> 29));
        if (want<GM, G_VLAN>(out.vlan_cfi)) st<(GM & G_NT) != 0, uint8_t>(out.vlan_cfi, o1, (uint8_t)((d[0] >> 28) & 1u));
        if (want<GM, G_VLAN>(out.vlan_vid)) st<(GM & G_NT) != 0, uint16_t>(out.vlan_vid, o2, (uint16_t)((d[0] >> 16) & 0xFFFu));
        if (want<GM, G_VLAN>(out.vlan_etype)) st<(GM & G_NT) != 0, uint16_t>(out.vlan_etype, o2, (uint16_t)(d[0] & 0xFFFFu));
    }
    // IPv4 (headers.rs:555-574) + Packet::ipv4_checksum (packet.rs:93-107)
    if (want<GM, G_IPV4>(out.ipv4_version) || want<GM, G_IPV4>(out.ipv4_ihl) || want<GM, G_IPV4>(out.ipv4_diffserv) ||
        want<GM, G_IPV4>(out.ipv4_total_len) || want<GM, G_IPV4>(out.ipv4_identification) ||
        want<GM, G_IPV4>(out.ipv4_flags) || want<GM, G_IPV4>(out.ipv4_frag_startset) || want<GM, G_IPV4>(out.ipv4_ttl) ||
        want<GM, G_IPV4>(out.ipv4_protocol) || want<GM, G_IPV4>(out.ipv4_header_checksum) ||
        want<GM, G_IPV4>(out.ipv4_src) || want<GM, G_IPV4>(out.ipv4_dst) || want<GM, G_IPV4>(out.ipv4_csum_calc)) {
        uint32_t d[5] = {0, 0, 0, 0, 0};
        const bool h = ok && r.f_ipv4 >= 0;
        if (h) pv.template hdr<5>((uint32_t)r.f_ipv4, 20, d);
        if (want<GM, G_IPV4>(out.ipv4_version)) st<(GM & G_NT) != 0, uint8_t>(out.ipv4_version, o1, (uint8_t)(d[0] >> 28));
        if (want<GM, G_IPV4>(out.ipv4_ihl)) st<(GM & G_NT) != 0, uint8_t>(out.ipv4_ihl, o1, (uint8_t)((d[0] >> 24) & 0xFu));
        if (want<GM, G_IPV4>(out.ipv4_diffserv)) st<(GM & G_NT) != 0, uint8_t>(out.ipv4_diffserv, o1, (uint8_t)((d[0] >> 16) & 0xFFu));
        if (want<GM, G_IPV4>(out.ipv4_total_len)) st<(GM & G_NT) != 0, uint16_t>(out.ipv4_total_len, o2, (uint16_t)(d[0] & 0xFFFFu));
        if (want<GM, G_IPV4>(out.ipv4_identification)) st<(GM & G_NT) != 0, uint16_t>(out.ipv4_identification, o2, (uint16_t)(d[1] >> 16));
        if (want<GM, G_IPV4>(out.ipv4_flags)) st<(GM & G_NT) != 0, uint8_t>(out.ipv4_flags, o1, (uint8_t)((d[1] >> 13) & 7u));
        if (want<GM, G_IPV4>(out.ipv4_frag_startset)) st<(GM & G_NT) != 0, uint16_t>(out.ipv4_frag_startset, o2, (uint16_t)(d[1] & 0x1FFFu));
        if (want<GM, G_IPV4>(out.ipv4_ttl)) st<(GM & G_NT) != 0, uint8_t>(out.ipv4_ttl, o1, (uint8_t)(d[2] >> 24));
        if (want<GM, G_IPV4>(out.ipv4_protocol)) st<(GM & G_NT) != 0, uint8_t>(out.ipv4_protocol, o1, (uint8_t)((d[2] >> 16) & 0xFFu));
        if (want<GM, G_IPV4>(out.ipv4_header_checksum)) st<(GM & G_NT) != 0, uint16_t>(out.ipv4_header_checksum, o2, (uint16_t)(d[2] & 0xFFFFu));
        if (want<GM, G_IPV4>(out.ipv4_src)) st<(GM & G_NT) != 0, uint32_t>(out.ipv4_src, o4, d[3]);
        if (want<GM, G_IPV4>(out.ipv4_dst)) st<(GM & G_NT) != 0, uint32_t>(out.ipv4_dst, o4, d[4]);
        if (want<GM, G_IPV4>(out.ipv4_csum_calc)) {
            // nine BE words, word 5 (byte offset 10) skipped; fold ((s>>16)+s)&0xFFFF (Q1)
            uint32_t s = (d[0] >> 16) + (d[0] & 0xFFFFu) + (d[1] >> 16) + (d[1] & 0xFFFFu) +
                         (d[2] >> 16) + (d[3] >> 16) + (d[3] & 0xFFFFu) + (d[4] >> 16) + (d[4] & 0xFFFFu);
            s = ((s >> 16) + s) & 0xFFFFu;
            st<(GM & G_NT) != 0, uint16_t>(out.ipv4_csum_calc, o2, h ? (uint16_t)(~s) : (uint16_t)0);
        }
    }
    // IPv6 (headers.rs:577-592); src/dst as the raw 16 bytes of bytes(msb, lsb)
    if (want<GM, G_IPV6>(out.ipv6_version) || want<GM, G_IPV6>(out.ipv6_traffic_class) ||
        want<GM, G_IPV6>(out.ipv6_flow_label) || want<GM, G_IPV6>(out.ipv6_payload_len) ||
        want<GM, G_IPV6>(out.ipv6_next_hdr) || want<GM, G_IPV6>(out.ipv6_hop_limit) ||
        want<GM, G_IPV6>(out.ipv6_src) || want<GM, G_IPV6>(out.ipv6_dst)) {
        uint32_t d[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
        if (ok && r.f_ipv6 >= 0) pv.template hdr<10>((uint32_t)r.f_ipv6, 40, d);
        if (want<GM, G_IPV6>(out.ipv6_version)) st<(GM & G_NT) != 0, uint8_t>(out.ipv6_version, o1, (uint8_t)(d[0] >> 28));
        if (want<GM, G_IPV6>(out.ipv6_traffic_class)) st<(GM & G_NT) != 0, uint8_t>(out.ipv6_traffic_class, o1, (uint8_t)((d[0] >> 20) & 0xFFu));
        if (want<GM, G_IPV6>(out.ipv6_flow_label)) st<(GM & G_NT) != 0, uint32_t>(out.ipv6_flow_label, o4, d[0] & 0xFFFFFu);
        if (want<GM, G_IPV6>(out.ipv6_payload_len)) st<(GM & G_NT) != 0, uint16_t>(out.ipv6_payload_len, o2, (uint16_t)(d[1] >> 16));
        if (want<GM, G_IPV6>(out.ipv6_next_hdr)) st<(GM & G_NT) != 0, uint8_t>(out.ipv6_next_hdr, o1, (uint8_t)((d[1] >> 8) & 0xFFu));
        if (want<GM, G_IPV6>(out.ipv6_hop_limit)) st<(GM & G_NT) != 0, uint8_t>(out.ipv6_hop_limit, o1, (uint8_t)(d[1] & 0xFFu));
        if (want<GM, G_IPV6>(out.ipv6_src))
            st<(GM & G_NT) != 0, uint4>(reinterpret_cast<uint4*>(out.ipv6_src), o16,
                      make_uint4(bswap32(d[2]), bswap32(d[3]), bswap32(d[4]), bswap32(d[5])));
        if (want<GM, G_IPV6>(out.ipv6_dst))
            st<(GM & G_NT) != 0, uint4>(reinterpret_cast<uint4*>(out.ipv6_dst), o16,
                      make_uint4(bswap32(d[6]), bswap32(d[7]), bswap32(d[8]), bswap32(d[9])));
    }
    // TCP (headers.rs:606-622)
    if (want<GM, G_TCP>(out.tcp_src) || want<GM, G_TCP>(out.tcp_dst) || want<GM, G_TCP>(out.tcp_seq_no) ||
        want<GM, G_TCP>(out.tcp_ack_no) || want<GM, G_TCP>(out.tcp_data_startset) || want<GM, G_TCP>(out.tcp_res) ||
        want<GM, G_TCP>(out.tcp_flags) || want<GM, G_TCP>(out.tcp_window) || want<GM, G_TCP>(out.tcp_checksum) ||
        want<GM, G_TCP>(out.tcp_urgent_ptr)) {
        uint32_t d[5] = {0, 0, 0, 0, 0};
        if (ok && r.f_tcp >= 0) pv.template hdr<5>((uint32_t)r.f_tcp, 20, d);
        if (want<GM, G_TCP>(out.tcp_src)) st<(GM & G_NT) != 0, uint16_t>(out.tcp_src, o2, (uint16_t)(d[0] >> 16));
        if (want<GM, G_TCP>(out.tcp_dst)) st<(GM & G_NT) != 0, uint16_t>(out.tcp_dst, o2, (uint16_t)(d[0] & 0xFFFFu));
        if (want<GM, G_TCP>(out.tcp_seq_no)) st<(GM & G_NT) != 0, uint32_t>(out.tcp_seq_no, o4, d[1]);
        if (want<GM, G_TCP>(out.tcp_ack_no)) st<(GM & G_NT) != 0, uint32_t>(out.tcp_ack_no, o4, d[2]);
        if (want<GM, G_TCP>(out.tcp_data_startset)) st<(GM & G_NT) != 0, uint8_t>(out.tcp_data_startset, o1, (uint8_t)(d[3] >> 28));
        if (want<GM, G_TCP>(out.tcp_res)) st<(GM & G_NT) != 0, uint8_t>(out.tcp_res, o1, (uint8_t)((d[3] >> 24) & 0xFu));
        if (want<GM, G_TCP>(out.tcp_flags)) st<(GM & G_NT) != 0, uint8_t>(out.tcp_flags, o1, (uint8_t)((d[3] >> 16) & 0xFFu));
        if (want<GM, G_TCP>(out.tcp_window)) st<(GM & G_NT) != 0, uint16_t>(out.tcp_window, o2, (uint16_t)(d[3] & 0xFFFFu));
        if (want<GM, G_TCP>(out.tcp_checksum)) st<(GM & G_NT) != 0, uint16_t>(out.tcp_checksum, o2, (uint16_t)(d[4] >> 16));
        if (want<GM, G_TCP>(out.tcp_urgent_ptr)) st<(GM & G_NT) != 0, uint16_t>(out.tcp_urgent_ptr, o2, (uint16_t)(d[4] & 0xFFFFu));
    }
    // UDP (headers.rs:625-634)
    if (want<GM, G_UDP>(out.udp_src) || want<GM, G_UDP>(out.udp_dst) || want<GM, G_UDP>(out.udp_length) ||
        want<GM, G_UDP>(out.udp_checksum)) {
        uint32_t d[2] = {0, 0};
        if (ok && r.f_udp >= 0) pv.template hdr<2>((uint32_t)r.f_udp, 8, d);
        if (want<GM, G_UDP>(out.udp_src)) st<(GM & G_NT) != 0, uint16_t>(out.udp_src, o2, (uint16_t)(d[0] >> 16));
        if (want<GM, G_UDP>(out.udp_dst)) st<(GM & G_NT) != 0, uint16_t>(out.udp_dst, o2, (uint16_t)(d[0] & 0xFFFFu));
        if (want<GM, G_UDP>(out.udp_length)) st<(GM & G_NT) != 0, uint16_t>(out.udp_length, o2, (uint16_t)(d[1] >> 16));
        if (want<GM, G_UDP>(out.udp_checksum)) st<(GM & G_NT) != 0, uint16_t>(out.udp_checksum, o2, (uint16_t)(d[1] & 0xFFFFu));
    }
}

// Packet i's start (byte offset in the slab) and length, clamped to the slab so that no read
// can leave the caller's allocation whatever the batch description says.
__device__ __forceinline__ void packet_range(const KParams& p, uint32_t i, uint64_t& off,
                                             uint32_t& len) {
    if (p.offsets) {
        off = p.offsets[i] - p.off_bias;
        len = p.lens[i];
    } else {
        off = (p.i0 + i) * (uint64_t)p.stride;
        if (p.lens) len = p.lens[i];
        else len = p.stride;
    }
    uint64_t room = off < p.slab_len ? p.slab_len - off : 0;
    if ((uint64_t)len > room) len = (uint32_t)room;
    if (len > 0xFFFFu) len = 0xFFFFu;  // u16 offsets/lengths in the ABI
}

// Dynamic LDS of a parse block (base 16-byte aligned; nothing static in front of it): the packet
// windows, packet-major: packet q's window at q * lane_stride, lane_stride = 4*NCH+1 dwords (odd, so the
// per-lane dword reads of the walk hit 64 distinct banks); +16 B for the last lane's over-read.
// (A chunk-major layout with ds_write_b128 staging had 4-way conflicts on the walk's reads: C4
// 3 % slower, C2/C3 neutral, scripts/ab_bench.sh.)
__host__ __device__ constexpr uint32_t lane_stride(int nch) { return (uint32_t)(4 * nch + 1) * 4u; }
__host__ __device__ constexpr size_t window_lds(int nch) {
    return ((size_t)kBlock * lane_stride(nch) + 16 + 15) & ~(size_t)15;
}

__device__ __forceinline__ PacketView make_view(const KParams& p, uint8_t* lds, uint32_t q, uint64_t off,
                                                uint32_t len, int nch) {
    PacketView pv;
    pv.lw = lds + q * lane_stride(nch);
    pv.slab = p.slab;
    pv.off = off;
    pv.last4 = ((p.slab_len + 15) & ~(uint64_t)15) - 4;
    pv.shift = (uint32_t)(off & 15);
    pv.win_lo = 0;
    pv.win_end = (uint32_t)nch * 16u - pv.shift;
    pv.len = len;
    return pv;
}

template <uint32_t GM>
__device__ __forceinline__ void emit_chain(const pkt_out_t& out, uint32_t i, uint32_t len, const WalkResult& r) {
    const bool ok = r.status == PKT_OK;
    if (want<GM, G_CHAIN>(out.status)) st<(GM & G_NT) != 0, uint8_t>(out.status, i, (uint8_t)r.status);
    if (want<GM, G_CHAIN>(out.n_hdrs)) st<(GM & G_NT) != 0, uint8_t>(out.n_hdrs, i, ok ? (uint8_t)r.n : (uint8_t)0);
    if (want<GM, G_CHAIN>(out.payload_off)) st<(GM & G_NT) != 0, uint16_t>(out.payload_off, 2 * i, ok ? (uint16_t)r.payload_off : (uint16_t)0);
    if (want<GM, G_CHAIN>(out.payload_len)) st<(GM & G_NT) != 0, uint16_t>(out.payload_len, 2 * i, ok ? (uint16_t)(len - r.payload_off) : (uint16_t)0);
    if (want<GM, G_CHAIN>(out.hdr_mask)) st<(GM & G_NT) != 0, uint32_t>(out.hdr_mask, 4 * i, ok ? r.mask : 0u);
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#ifndef PKTGPU_LATE_COLS
#define PKTGPU_LATE_COLS 1  // parse_kernel loads its column bases after the walk (0: at the start)
#endif
#define KARG_AS __attribute__((address_space(4)))
// A generic pointer the caller knows to be global memory, re-marked as such (addrspacecast to global
// and back): loads and stores through it stay global_* instructions instead of flat_*.
template <class T>
__device__ __forceinline__ T* as_global(T* q) {
    return (T*)((__attribute__((address_space(1))) T*)q);
}

// Diagnostic build only (-DPKTGPU_STAMPS=1: scripts/build_variant.sh, read by scripts/stamps.py): s_memtime stamps per wave of the
// parse kernel — start, windows in LDS, walk done, emit issued, stores drained — plus the wave's
// hardware id, written by lane 0 to a debug buffer no other code reads (pkt_debug_stamps).  In the
// normal build no stamp executes.
#ifndef PKTGPU_STAMPS
#define PKTGPU_STAMPS 0
#endif
#if PKTGPU_STAMPS
__device__ uint64_t* g_pkt_stamps;
#define PKT_STAMP(k)                                                                          \
    do {                                                                                      \
        __builtin_amdgcn_sched_barrier(0);                                                    \
        uint64_t t_;                                                                          \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");            \
        __builtin_amdgcn_sched_barrier(0);                                                    \
        pkt_st[k] = t_;                                                                       \
    } while (0)
#else
#define PKT_STAMP(k) \
    do {             \
    } while (0)
#endif

// Lane t's packet range and its first NCH 16-byte chunks (from the 16-byte-aligned start) by
// per-lane dwordx4 loads (faster than the LDS-DMA gather, scripts/probe.py).  Chunks past the
// readable end of the slab (round_up(slab_len, 16)) are clamped to an in-bounds chunk; those
// bytes lie beyond every packet and are never interpreted.
template <int NCH>
__device__ __forceinline__ void load_packet(const KParams& p, uint32_t i, bool active, u32x4 (&chunk)[NCH],
                                            uint64_t& off, uint32_t& len) {
    off = 0;
    len = 0;
    if (active) packet_range(p, i, off, len);
    const uint64_t a0 = off & ~(uint64_t)15;
    const uint64_t last16 = ((p.slab_len + 15) & ~(uint64_t)15) - 16;
#pragma unroll
    for (int c = 0; c < NCH; c++) {
        uint64_t o = a0 + 16u * (uint32_t)c;
        o = o > last16 ? last16 : o;
        chunk[c] = *reinterpret_cast<const u32x4*>(p.slab + o);
    }
}

// Packet q's window: its chunks as dwords at q * lane_stride(NCH) (odd dword stride).
template <int NCH>
__device__ __forceinline__ void stage_window(uint8_t* lds, uint32_t q, const u32x4 (&chunk)[NCH]) {
#pragma unroll
    for (int c = 0; c < NCH; c++) {
        uint32_t* w = reinterpret_cast<uint32_t*>(lds + q * lane_stride(NCH)) + 4 * c;
        w[0] = chunk[c].x;
        w[1] = chunk[c].y;
        w[2] = chunk[c].z;
        w[3] = chunk[c].w;
    }
}

// ---- several batches in one launch (pkt_parse_batches) ----
// K batches of the same size and layout whose outputs lie at one common byte distance from batch
// 0's (e.g. one packed output buffer each): block j parses tile j % bpb of batch j / bpb.  Every
// per-batch value comes from the kernel arguments (a scalar load at a computed offset: no table
// read from memory before the block can start), and the launch's ramp and drain are paid once for
// the K batches instead of once per batch.
constexpr int kMaxMulti = 16;
struct MultiBatch {
    const uint8_t* slab;
    uint64_t slab_len;
    const uint64_t* offsets;
    const uint32_t* lens;
    int64_t out_delta;  // bytes from batch 0's column pointers to this batch's
};
struct MultiParams {
    KParams base;  // batch 0 (its slab, index, outputs), the shared n / stride / entry / knobs
    uint32_t bpb;  // blocks per batch
    uint32_t k;
    MultiBatch per[kMaxMulti];
};
static_assert(offsetof(MultiParams, base) == 0, "the late column loads read base.out at offsetof(KParams, out)");

// Where the emit's column bases come from (LATE): L_EARLY = the KParams the kernel holds since its
// start; L_SINGLE = loaded after the walk from the kernel arguments (parse_kernel: one KParams);
// L_MULTI = the same from a MultiParams (its base.out) plus batch `mb`'s out_delta, also loaded after
// the walk (parse_multi_kernel).
enum LateCols : int { L_EARLY = 0, L_SINGLE = 1, L_MULTI = 2 };

template <int NCH, uint32_t GM, int WK, bool STAGED = false, int LATE = L_EARLY>
__device__ __forceinline__ void parse_tile(const KParams& p, uint8_t* lds, uint32_t base,
                                           const u32x4 (&chunk)[NCH], uint64_t off_own, uint32_t len_own,
                                           bool active_own, uint64_t* pkt_st, const DispatchLds* T, uint32_t mb);

// Dynamic LDS of a lockstep launch: the windows (or spans), then the dispatch tables.
__host__ __device__ constexpr size_t with_tables(size_t bytes, int wk) {
    return wk == 1 ? ((bytes + 15) & ~(size_t)15) + sizeof(DispatchLds) : bytes;
}
template <int WK>
__device__ __forceinline__ const DispatchLds* tables(uint8_t* lds, size_t at, uint32_t t, uint32_t nt) {
    if constexpr (WK != 1) return nullptr;
    DispatchLds* T = reinterpret_cast<DispatchLds*>(lds + ((at + 15) & ~(size_t)15));
    dispatch_init(T, t, nt);
    __syncthreads();
    return T;
}

// One block = 256 packets, one lane per packet.  (A persistent grid of k blocks per CU striding
// over the tiles, each lane's loads of its next packet in flight while it parsed the current one,
// was measured no faster at k = 4 and slower at k = 1, 2: DESIGN.md §5.)
// Resident waves per SIMD the compiler may assume (VGPR budget 512 / waves): 8 for fixed-stride
// windows (<= 64 VGPRs); for indexed windows what their LDS allows anyway — 6 for the 96-byte
// windows (25.6 KB per block, 6 blocks per CU), 5 for the 112-byte ones (29.7 KB, 5 blocks), 4 for
// the 144-byte ones (37.9 KB, 4 blocks); wider windows unconstrained.
__host__ __device__ constexpr int waves_per_eu(int nch, int wk) {
    return nch > 9 ? 1 : (wk == 1 && nch >= 6 ? (nch == 9 ? 4 : nch == 7 ? 5 : 6) : 8);
}
// Tile `blk` (256 packets) of the batch `p` describes: load, stage, walk, emit.
template <int NCH, uint32_t GM, int WK, int LATE = L_EARLY>
__device__ __forceinline__ void parse_block(const KParams& p, uint32_t blk, uint8_t* lds, const DispatchLds* T,
                                            uint64_t* pkt_st, uint32_t mb = 0) {
    uint32_t base = blk * (uint32_t)kBlock;  // within this launch
    uint32_t n_eff = p.n;
    if (p.n_dev) {  // wave-uniform: the count the device produced (scalar load)
        const uint64_t nd = *p.n_dev;
        n_eff = nd < (uint64_t)n_eff ? (uint32_t)nd : n_eff;
        if (p.i0_dev) base += (uint32_t)*p.i0_dev;  // the launch starts at a device-produced index
        if (base >= n_eff) return;  // the whole block is past the count
    }
    const bool act = base + threadIdx.x < n_eff;
    u32x4 chunk[NCH];
    uint64_t off;
    uint32_t len;
    if constexpr (NCH >= 4) {
        // The wave loads its 64 windows cooperatively: the 64*NCH (packet, chunk) pairs, pair
        // 64k + lane in load k, so consecutive lanes fetch consecutive 16-byte chunks of one packet
        // and each window comes from one or two wave instructions — the per-lane shape (each lane
        // fetching its own chunks) is request-bound, 42 us for the 2^20 C4 windows alone
        // (scripts/probe_c4.py), and separate instructions to the same 128-B line re-request it from
        // memory (scripts/fetch_calib.py).  Each chunk goes straight into the owning lane's LDS
        // window.  C4 pipelined 78 vs 82 us/step, C2 23.9 vs 25.2, C3 43.3 vs 46.1 against per-lane
        // loads (profiles/ab/r02p_c4_coop_windows.txt, r02x_coop_fixed_stride.txt).
        // Lockstep (indexed) launches skip the chunks that start past their packet's end: a short
        // record (Dot3, ARP) fetches only its own lines.
        off = 0;
        len = 0;
        if (act) packet_range(p, base + threadIdx.x, off, len);
        const uint32_t wl = threadIdx.x & 63u, wave0 = threadIdx.x & ~63u;
        const uint64_t last16 = ((p.slab_len + 15) & ~(uint64_t)15) - 16;
#pragma unroll
        for (uint32_t k = 0; k < (uint32_t)NCH; k++) {
            const uint32_t pid = 64u * k + wl, r = pid / (uint32_t)NCH, c = pid % (uint32_t)NCH;
            const uint64_t offr = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(off >> 32), (int)r, 64) << 32) |
                                  (uint32_t)__shfl((int)(uint32_t)off, (int)r, 64);
            if constexpr (WK == 1) {
                const uint32_t lenr = (uint32_t)__shfl((int)len, (int)r, 64);
                if (16u * c >= (uint32_t)(offr & 15) + lenr) continue;  // chunk past the packet
            }
            uint64_t a = (offr & ~(uint64_t)15) + 16u * c;
            a = a > last16 ? last16 : a;
            const u32x4 v = *reinterpret_cast<const u32x4*>(p.slab + a);
            uint32_t* w = reinterpret_cast<uint32_t*>(lds + (wave0 + r) * lane_stride(NCH)) + 4 * c;
            w[0] = v.x;
            w[1] = v.y;
            w[2] = v.z;
            w[3] = v.w;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        PKT_STAMP(1);
        parse_tile<NCH, GM, WK, true, LATE>(p, lds, base, chunk, off, len, act, pkt_st, T, mb);
        return;
    }
    load_packet<NCH>(p, base + threadIdx.x, act, chunk, off, len);
    parse_tile<NCH, GM, WK, false, LATE>(p, lds, base, chunk, off, len, act, pkt_st, T, mb);
}

template <int NCH, uint32_t GM, int WK>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(waves_per_eu(NCH, WK))))
void parse_kernel(KParams p) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    uint64_t pkt_st[5] = {0, 0, 0, 0, 0};
    PKT_STAMP(0);
    const DispatchLds* T = tables<WK>(lds, window_lds(NCH), threadIdx.x, kBlock);
    parse_block<NCH, GM, WK, PKTGPU_LATE_COLS != 0 ? L_SINGLE : L_EARLY>(p, blockIdx.x, lds, T, pkt_st);
}

// Block j parses tile j % bpb of batch j / bpb.  Only the slot columns (hdr_type / hdr_off, which
// the walk writes) are moved to the batch at the kernel start; the other 47 column bases and the
// batch's out_delta are loaded after the walk (L_MULTI), as parse_kernel does: adding the delta to
// all 49 bases up front held them through the walk and spilled 36 (C2 columns) / 42 (C4, all
// columns) SGPRs to VGPR lanes (round-4 review).
template <int NCH, uint32_t GM, int WK>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(waves_per_eu(NCH, WK))))
void parse_multi_kernel(MultiParams mp) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    uint64_t pkt_st[5] = {0, 0, 0, 0, 0};
    const DispatchLds* T = tables<WK>(lds, window_lds(NCH), threadIdx.x, kBlock);
    const uint32_t b = blockIdx.x / mp.bpb;  // wave-uniform
    const MultiBatch& mb = mp.per[b];
    KParams p = mp.base;
    p.slab = mb.slab;
    p.slab_len = mb.slab_len;
    p.offsets = mb.offsets;
    p.lens = mb.lens;
    if (p.out.hdr_type) p.out.hdr_type += mb.out_delta;
    if (p.out.hdr_off) p.out.hdr_off = reinterpret_cast<uint16_t*>(reinterpret_cast<uint8_t*>(p.out.hdr_off) + mb.out_delta);
    parse_block<NCH, GM, WK, L_MULTI>(p, blockIdx.x - b * mp.bpb, lds, T, pkt_st, b);
}

// The emit of one column group with its bases loaded from the kernel arguments right here (LATE): columns
// [LO, HI) of pkt_out_t (group G), through an opaque copy of their address taken after a compiler memory
// barrier, so the loads come after the previous group's stores.  One group's bases live at a time (at most
// 13 pointers): the all-columns and C3 emits held every group's (~40 bases, 80 SGPRs) at once and spilled
// 32-74 SGPRs to VGPR lanes (round-5 review).
template <uint32_t GM, uint32_t G, int LO, int HI, int LATE, class View>
__device__ __forceinline__ void emit_group_late(uint64_t kseg, int64_t delta, uint32_t i, uint32_t len, const View& pv,
                                                const WalkResult& r) {
    constexpr bool rt = (GM & G_RUNTIME) != 0;
    if constexpr (rt || (GM & G) != 0) {
        uint64_t ka = kseg + offsetof(KParams, out) + sizeof(void*) * LO;
        asm volatile("" : "+s"(ka)::"memory");
        const void* const KARG_AS* kc = reinterpret_cast<const void* const KARG_AS*>(ka);
        pkt_out_t oc{};
        void** ocp = reinterpret_cast<void**>(&oc);
#pragma unroll
        for (int c = LO; c < HI; c++) {
            const void* q = kc[c - LO];
            if constexpr (LATE == L_MULTI) q = q ? reinterpret_cast<const uint8_t*>(q) + delta : q;
            ocp[c] = as_global(const_cast<void*>(q));
        }
        constexpr uint32_t GG = rt ? GM : (G | (GM & G_NT));
        if constexpr (G == G_CHAIN) emit_chain<GG>(oc, i, len, r);
        else emit_fields<GG>(oc, i, pv, r, r.status == PKT_OK);
    }
}

template <int NCH, uint32_t GM, int WK, bool STAGED, int LATE>
__device__ __forceinline__ void parse_tile(const KParams& p, uint8_t* lds, uint32_t base,
                                           const u32x4 (&chunk)[NCH], uint64_t off_own, uint32_t len_own,
                                           bool active_own, uint64_t* pkt_st, const DispatchLds* T, uint32_t mb) {
    (void)pkt_st;
    (void)mb;
    const uint32_t t = threadIdx.x;
    const uint32_t i_own = base + t;
    // Register fast path (pkt_ctx_set_fastpath): an aligned packet whose EtherType chain is
    // 0x0800, 0x8100 0x0800 or 0x8100 0x8100 0x0800 (bytes 12, 16, 20: v = 0..2 VLAN tags), whose
    // IPv4 protocol (byte 23 + 4v) is 17 with a UDP dst port (bytes 36 + 4v) != 4789 and
    // len >= 42 + 4v, or 6 with len >= 54 + 4v, takes exactly fast.rs's Ether -> Vlan{v} -> IPv4 ->
    // UDP|TCP -> accept path (no bound or depth check can fail on it), so a few compares on the
    // loaded registers decide its whole chain: it skips the walk.
    bool fast = false, fudp = false;
    uint32_t fv = 0;
    if constexpr (NCH >= 4) {
        if (p.fast && active_own && (off_own & 15) == 0) {
            // dwords 3..11 of the packet (little-endian), from the registers or, when the wave
            // loaded its windows cooperatively, from the lane's own LDS window
            uint32_t d3, d4, d5, d6, d7, d9, d10, d11;
            if constexpr (STAGED) {
                const uint32_t* w = reinterpret_cast<const uint32_t*>(lds + t * lane_stride(NCH));
                d3 = w[3], d4 = w[4], d5 = w[5], d6 = w[6], d7 = w[7], d9 = w[9], d10 = w[10], d11 = w[11];
            } else {
                d3 = chunk[0].w, d4 = chunk[1].x, d5 = chunk[1].y, d6 = chunk[1].z, d7 = chunk[1].w;
                d9 = chunk[2].y, d10 = chunk[2].z, d11 = chunk[2].w;
            }
            const uint32_t e0 = d3 & 0xFFFFu, e1 = d4 & 0xFFFFu, e2 = d5 & 0xFFFFu;
            const bool v0 = e0 == 0x0008u;                    // little-endian 0x0800
            const bool v1 = e0 == 0x0081u && e1 == 0x0008u;   // 0x8100, 0x0800
            const bool v2 = e0 == 0x0081u && e1 == 0x0081u && e2 == 0x0008u;
            fv = v1 ? 1u : (v2 ? 2u : 0u);
            const uint32_t proto = (v0 ? d5 : v1 ? d6 : d7) >> 24;
            const uint32_t dport = (v0 ? d9 : v1 ? d10 : d11) & 0xFFFFu;
            const uint32_t l4 = 34u + 4u * fv;
            fudp = proto == 17u;
            fast = (v0 || v1 || v2) && ((fudp && len_own >= l4 + 8u && dport != 0xB512u) ||
                                        (proto == 6u && len_own >= l4 + 20u));
        }
    }
    // Fast lanes skip the walk; all lanes stage their window and emit from LDS together (one
    // store per column per wave).  (Decoding all-fast waves from registers instead: shorter
    // isolated launches, slower pipelined steps)
    const pkt_out_t& out = p.out;
    const uint64_t ns = p.n_slot_stride;
    auto push = [&](uint32_t slot, uint32_t ty, uint32_t o) { push_slot<GM>(out, ns, slot, i_own, ty, o); };
    // fast.rs:5-12 (>= 1500) -> parse_ethernet 35-48 (0x8100 -> parse_vlan 49-62, repeated;
    // 0x0800) -> parse_ipv4 84-98 (17 / 6) -> parse_udp 208-217 (dst != 4789) | parse_tcp 203-207
    // -> accept 223-227
    auto fast_result = [&](WalkResult& r, uint32_t v) {
        const uint32_t l4 = 34u + 4u * v;
        r.status = PKT_OK;
        r.n = 3 + v;
        r.payload_off = l4 + (fudp ? 8u : 20u);
        r.mask = (1u << PKT_HDR_ETHER) | (1u << PKT_HDR_IPV4) | (fudp ? 1u << PKT_HDR_UDP : 1u << PKT_HDR_TCP) |
                 (v ? 1u << PKT_HDR_VLAN : 0u);
        r.f_eth = 0;
        r.f_vlan = v ? 14 : -1;
        r.f_ipv4 = (int32_t)(14u + 4u * v);
        r.f_ipv6 = -1;
        r.f_tcp = fudp ? -1 : (int32_t)l4;
        r.f_udp = fudp ? (int32_t)l4 : -1;
        push(0, PKT_HDR_ETHER, 0);
        if (v >= 1) push(1, PKT_HDR_VLAN, 14);
        if (v >= 2) push(2, PKT_HDR_VLAN, 18);
        push(1 + v, PKT_HDR_IPV4, 14u + 4u * v);
        push(2 + v, fudp ? PKT_HDR_UDP : PKT_HDR_TCP, l4);
    };
    if constexpr (!STAGED) stage_window<NCH>(lds, t, chunk);
    PacketView pv_own = make_view(p, lds, t, off_own, len_own, NCH);

    // each lane walks and emits its own packet (no barrier: own LDS only)
    __builtin_amdgcn_wave_barrier();
    WalkResult r;
    walk<WK>(pv_own, entry_state(p.entry), active_own && !fast, push, r, T);
    if constexpr (NCH >= 4) {
        if (fast) fast_result(r, fv);
    }
    PKT_STAMP(2);
    if (p.nh_max) {  // wave-uniform: the used slot rows of the batch, for a gather of its chain
        const uint32_t m = wave_max_u32((active_own && r.status == PKT_OK) ? r.n : 0u);
        if ((t & 63u) == 0 && m) atomicMax(p.nh_max + (blockIdx.x & (kMaxSpread - 1)), m);
    }
    if (active_own) {
        if constexpr (LATE != L_EARLY) {
            // The column bases are loaded here, after the walk, by scalar loads from the kernel
            // arguments (an opaque copy of their address keeps the loads from being hoisted to the
            // kernel start), and re-marked as global pointers so every store stays a global store.
            // Loaded at the start instead, the 49 bases of the all-columns kernel held 106 SGPRs
            // through the walk and spilled 48 to VGPR lanes (~96 lane instructions per wave); round
            // 3's late load through a generic pointer made every column access a flat access, 6x
            // slower (profiles/ab/r03j_late_column_pointers.txt).
            // (parse_kernel's only argument is the KParams, parse_multi_kernel's the MultiParams
            // whose first member is batch 0's KParams: either starts the kernarg segment)
            const uint64_t kseg = reinterpret_cast<uint64_t>(__builtin_amdgcn_kernarg_segment_ptr());
            uint64_t ka = kseg + offsetof(KParams, out);
            asm volatile("" : "+s"(ka));
            const void* const KARG_AS* kc = reinterpret_cast<const void* const KARG_AS*>(ka);
            int64_t delta = 0;
            if constexpr (LATE == L_MULTI) {
                // (mb is wave-uniform, but the integer division that made it leaves it in a VGPR)
                const uint32_t mbs = __builtin_amdgcn_readfirstlane(mb);
                uint64_t kd = kseg + offsetof(MultiParams, per) + (uint64_t)mbs * sizeof(MultiBatch) +
                              offsetof(MultiBatch, out_delta);
                asm volatile("" : "+s"(kd));
                delta = *reinterpret_cast<const int64_t KARG_AS*>(kd);
            }
            (void)kc;
            // column ranges of the groups in pkt_out_t order (group_masks)
            emit_group_late<GM, G_CHAIN, 0, 7, LATE>(kseg, delta, i_own, len_own, pv_own, r);
            emit_group_late<GM, G_ETHER, 7, 10, LATE>(kseg, delta, i_own, len_own, pv_own, r);
            emit_group_late<GM, G_VLAN, 10, 14, LATE>(kseg, delta, i_own, len_own, pv_own, r);
            emit_group_late<GM, G_IPV4, 14, 27, LATE>(kseg, delta, i_own, len_own, pv_own, r);
            emit_group_late<GM, G_IPV6, 27, 35, LATE>(kseg, delta, i_own, len_own, pv_own, r);
            emit_group_late<GM, G_TCP, 35, 45, LATE>(kseg, delta, i_own, len_own, pv_own, r);
            emit_group_late<GM, G_UDP, 45, 49, LATE>(kseg, delta, i_own, len_own, pv_own, r);
        } else {
            emit_chain<GM>(out, i_own, len_own, r);
            emit_fields<GM>(out, i_own, pv_own, r, r.status == PKT_OK);
        }
    }
#if PKTGPU_STAMPS
    PKT_STAMP(3);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    PKT_STAMP(4);
    if ((t & 63u) == 0 && g_pkt_stamps) {
        uint32_t hw, xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        uint64_t* d = g_pkt_stamps + ((uint64_t)blockIdx.x * kWavesPerBlock + (t >> 6)) * 8u;
        for (int k = 0; k < 5; k++) d[k] = pkt_st[k];
        d[5] = hw;
        d[6] = xcc & 15u;  // s_memtime counts per XCD: stamps compare within one XCD only
    }
#endif
}

// ---- span staging (indexed batches: the records of a pcap lie back to back) ----
// The 64 records of a wave usually occupy ONE contiguous byte range of the slab.  The wave copies
// that range [lo & ~15, hi) into its LDS region by LDS-DMA (global_load_lds_dwordx4: 1 KiB of
// consecutive bytes per wave-instruction, fully coalesced, no VGPRs) and every lane then walks its
// record entirely out of LDS: no per-lane window, no global-memory reads for deep tunnels, and
// each HBM line is fetched once.  A wave whose range exceeds the region (records far apart or
// long) stages per-lane windows into the same region instead (the parse_kernel staging).
#define LDS_AS __attribute__((address_space(3)))
#ifndef PKTGPU_SPAN_CAP
#define PKTGPU_SPAN_CAP 16384u  // bytes of range one wave stages (a multiple of 1024)
#endif
static_assert(PKTGPU_SPAN_CAP % 1024u == 0, "span cap: whole 1 KiB LDS-DMA pieces");
constexpr uint32_t kSpanBlock = 64;  // one wave per block: one LDS region per block
__host__ __device__ constexpr uint32_t span_region(int nch) {
    // the range, or the fallback's 64 packed windows; +16: the walk's dword over-read
    return ((PKTGPU_SPAN_CAP > 64u * lane_stride(nch) ? PKTGPU_SPAN_CAP : 64u * lane_stride(nch)) + 16u + 15u) & ~15u;
}

__device__ __forceinline__ uint64_t wave_uniform64(uint64_t v) {
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}

template <int NCH, uint32_t GM, int WK>
__global__ __launch_bounds__(kSpanBlock) void parse_span_kernel(KParams p) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const uint32_t lane = threadIdx.x;
    uint32_t n_eff = p.n, b0 = blockIdx.x * kSpanBlock;
    if (p.n_dev) {  // wave-uniform: the count the device produced (scalar load)
        const uint64_t nd = *p.n_dev;
        n_eff = nd < (uint64_t)n_eff ? (uint32_t)nd : n_eff;
        if (p.i0_dev) b0 += (uint32_t)*p.i0_dev;  // the launch starts at a device-produced index
        if (b0 >= n_eff) return;  // the whole wave (= block) is past the count
    }
    const DispatchLds* T = tables<WK>(lds, span_region(NCH), lane, kSpanBlock);
    const uint32_t i = b0 + lane;  // within this launch
    const bool active = i < n_eff;
    uint64_t off = 0;
    uint32_t len = 0;
    if (active) packet_range(p, i, off, len);
    // the wave's byte range [lo, hi) (butterfly min/max; lane 0 is active: blocks whose first packet
    // lies past the count have returned above)
    uint64_t lo = active ? off : ~(uint64_t)0, hi = active ? off + len : 0;
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) {
        const uint64_t l2 = __shfl_xor(lo, m, 64), h2 = __shfl_xor(hi, m, 64);
        lo = l2 < lo ? l2 : lo;
        hi = h2 > hi ? h2 : hi;
    }
    const uint64_t a0 = wave_uniform64(lo) & ~(uint64_t)15;
    const uint64_t hi_u = wave_uniform64(hi);
    const uint64_t bytes = hi_u > a0 ? hi_u - a0 : 0;
    const uint64_t last16 = ((p.slab_len + 15) & ~(uint64_t)15) - 16;
    PacketView pv;
    if (bytes <= PKTGPU_SPAN_CAP) {  // wave-uniform
        const uint32_t npiece = (uint32_t)((bytes + 1023) >> 10);
        for (uint32_t k = 0; k < npiece; k++) {
            uint64_t o = a0 + ((uint64_t)k << 10) + lane * 16u;
            o = o > last16 ? last16 : o;  // bytes past the slab end lie beyond every record
            __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(p.slab + o),
                                             (LDS_AS void*)(lds + (k << 10)), 16, 0, 0);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint32_t rel = active ? (uint32_t)(off - a0) : 0u;
        pv.lw = lds + (rel & ~3u);
        pv.slab = p.slab;
        pv.off = off;
        pv.last4 = ((p.slab_len + 15) & ~(uint64_t)15) - 4;
        pv.shift = rel & 3u;
        pv.win_lo = 0;
        pv.win_end = (npiece << 10) - rel;  // >= len: the whole record is in LDS
        pv.len = len;
    } else {
        u32x4 chunk[NCH];
        const uint64_t c0 = off & ~(uint64_t)15;
#pragma unroll
        for (int c = 0; c < NCH; c++) {
            uint64_t o = c0 + 16u * (uint32_t)c;
            o = o > last16 ? last16 : o;
            chunk[c] = *reinterpret_cast<const u32x4*>(p.slab + o);
        }
        stage_window<NCH>(lds, lane, chunk);
        pv = make_view(p, lds, lane, off, len, NCH);
    }
    const pkt_out_t& out = p.out;
    const uint64_t ns = p.n_slot_stride;
    auto push = [&](uint32_t slot, uint32_t ty, uint32_t o) { push_slot<GM>(out, ns, slot, i, ty, o); };
    WalkResult r;
    walk<WK>(pv, entry_state(p.entry), active, push, r, T);
    if (p.nh_max) {
        const uint32_t m = wave_max_u32((active && r.status == PKT_OK) ? r.n : 0u);
        if (lane == 0 && m) atomicMax(p.nh_max + (blockIdx.x & (kMaxSpread - 1)), m);
    }
    if (!active) return;
    // the column bases group by group, loaded after the walk (parse_kernel's late loads: the kernel's
    // only argument is the KParams, so the kernarg segment starts with it)
    const uint64_t kseg = reinterpret_cast<uint64_t>(__builtin_amdgcn_kernarg_segment_ptr());
    emit_group_late<GM, G_CHAIN, 0, 7, L_SINGLE>(kseg, 0, i, len, pv, r);
    emit_group_late<GM, G_ETHER, 7, 10, L_SINGLE>(kseg, 0, i, len, pv, r);
    emit_group_late<GM, G_VLAN, 10, 14, L_SINGLE>(kseg, 0, i, len, pv, r);
    emit_group_late<GM, G_IPV4, 14, 27, L_SINGLE>(kseg, 0, i, len, pv, r);
    emit_group_late<GM, G_IPV6, 27, 35, L_SINGLE>(kseg, 0, i, len, pv, r);
    emit_group_late<GM, G_TCP, 35, 45, L_SINGLE>(kseg, 0, i, len, pv, r);
    emit_group_late<GM, G_UDP, 45, 49, L_SINGLE>(kseg, 0, i, len, pv, r);
}


// How a launch stages packet bytes: per-lane windows (one tile per block) or wave spans.
// (Round 3's pipelined windows — persistent waves loading the next tile's windows into VGPRs while
// walking the current one — were slower on every measured batch, C4 96.7 vs 89.9 us isolated,
// profiles/ab/r03b_c4_staging3_pipelined_windows.txt, and correct only while every instantiation
// stayed spill-free; removed in round 4.)
enum LaunchMode { M_TILE = 0, M_SPAN = 2 };

template <int NCH, uint32_t GM, int WK>
hipError_t launch_mode(const KParams& kp, int mode, hipStream_t s, const MultiParams* mp, uint32_t gn) {
    if (mp) {  // several batches, one launch (windows only)
        hipLaunchKernelGGL((parse_multi_kernel<NCH, GM, WK>), dim3(mp->bpb * mp->k), dim3(kBlock),
                           with_tables(window_lds(NCH), WK), s, *mp);
        return hipGetLastError();
    }
    if (mode == M_SPAN) {
        hipLaunchKernelGGL((parse_span_kernel<NCH, GM, WK>), dim3((unsigned)((gn + kSpanBlock - 1) / kSpanBlock)),
                           dim3(kSpanBlock), with_tables(span_region(NCH), WK), s, kp);
    } else {
        const size_t lds = with_tables(window_lds(NCH), WK);
        hipLaunchKernelGGL((parse_kernel<NCH, GM, WK>), dim3((unsigned)((gn + kBlock - 1) / kBlock)), dim3(kBlock),
                           lds, s, kp);
    }
    return hipGetLastError();
}

// Kernels are compiled per fully-requested column-group set; the lockstep walk (mixed traffic)
// only for the chain-only, all-columns and per-column-check sets.
template <int NCH>
hipError_t launch_gm(const KParams& kp, uint32_t gm, int mode, int wk, hipStream_t s, const MultiParams* mp,
                     uint32_t gn) {
    // lockstep (indexed batches; non-temporal column stores): compiled for the windows of 6, 7, 9
    // and 17 chunks only (window requests of <= 80, 96, 128 and 256 B; parse_impl widens the rest)
    if constexpr (NCH >= 6) if (wk == 1) {
        switch (gm) {
            case G_CHAIN: return launch_mode<NCH, G_CHAIN | G_NT, 1>(kp, mode, s, mp, gn);
            case G_ALL: return launch_mode<NCH, G_ALL | G_NT, 1>(kp, mode, s, mp, gn);
            default: return launch_mode<NCH, G_RUNTIME | G_NT, 1>(kp, mode, s, mp, gn);
        }
    }
    switch (gm) {
        case G_CHAIN: return launch_mode<NCH, G_CHAIN, 0>(kp, mode, s, mp, gn);
        case G_CHAIN | G_ETHER | G_IPV4 | G_UDP: return launch_mode<NCH, G_CHAIN | G_ETHER | G_IPV4 | G_UDP, 0>(kp, mode, s, mp, gn);
        case G_CHAIN | G_ETHER | G_VLAN | G_IPV4 | G_TCP | G_UDP:
            return launch_mode<NCH, G_CHAIN | G_ETHER | G_VLAN | G_IPV4 | G_TCP | G_UDP, 0>(kp, mode, s, mp, gn);
        case G_ALL: return launch_mode<NCH, G_ALL, 0>(kp, mode, s, mp, gn);
        default: return launch_mode<NCH, G_RUNTIME, 0>(kp, mode, s, mp, gn);
    }
}

// Which groups are fully requested (all columns non-NULL) and which partly.
void group_masks(const pkt_out_t& o, uint32_t& full, uint32_t& any) {
    const void* const* cols = reinterpret_cast<const void* const*>(&o);
    // column ranges of each group in pkt_out_t order (see include/pktgpu.h)
    static const struct { uint32_t g; int lo, hi; } R[] = {
        {G_CHAIN, 0, 7}, {G_ETHER, 7, 10}, {G_VLAN, 10, 14}, {G_IPV4, 14, 27},
        {G_IPV6, 27, 35}, {G_TCP, 35, 45}, {G_UDP, 45, 49}};
    static_assert(sizeof(pkt_out_t) == 49 * sizeof(void*), "pkt_out_t layout");
    full = any = 0;
    for (const auto& g : R) {
        bool all = true, some = false;
        for (int c = g.lo; c < g.hi; c++) {
            all &= cols[c] != nullptr;
            some |= cols[c] != nullptr;
        }
        if (all) full |= g.g;
        if (some) any |= g.g;
    }
}

template <class T>
T* adv(T* p, uint64_t k) { return p ? p + k : p; }

// Is `p` pinned host memory the device can address?  On success `dev` = its device address.
template <class T>
bool host_mapped(const T* p, const T*& dev) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();  // pageable memory: not an error for the caller
        return false;
    }
    if (a.type != hipMemoryTypeHost || !a.devicePointer) return false;
    dev = reinterpret_cast<const T*>(a.devicePointer);
    return true;
}
template <class T>
bool host_mapped(T* p, T*& dev) {
    const T* d = nullptr;
    if (!host_mapped<T>(static_cast<const T*>(p), d)) return false;
    dev = const_cast<T*>(d);
    return true;
}

// Grow one device buffer of every pipeline slot to `need` bytes (all slots idle: the caller has
// synchronised the pipeline streams).
template <class T>
hipError_t grow(T* (&buf)[HostPipe::kSlots], uint64_t& cap, uint64_t need) {
    if (need <= cap) return hipSuccess;
    for (int k = 0; k < HostPipe::kSlots; k++) {
        if (buf[k]) (void)hipFree(buf[k]);
        buf[k] = nullptr;
        hipError_t e = hipMalloc(reinterpret_cast<void**>(&buf[k]), need);
        if (e != hipSuccess) { cap = 0; return e; }
    }
    cap = need;
    return hipSuccess;
}


// The largest n_hdrs of a batch: how many slot rows of hdr_type / hdr_off hold data.  16 bytes per
// thread (grid-strided), a wave max, one atomicMax per wave that saw a non-zero count.
__global__ __launch_bounds__(256) void max_hdrs_kernel(const uint8_t* nh, uint64_t n, uint32_t* out) {
    uint32_t m = 0;
    const uint64_t step = (uint64_t)gridDim.x * 256u * 16u;
    const bool al = ((uintptr_t)nh & 15) == 0;
    for (uint64_t i = ((uint64_t)blockIdx.x * 256u + threadIdx.x) * 16u; i < n; i += step) {
        if (al && i + 16 <= n) {
            const uint4 v = *reinterpret_cast<const uint4*>(nh + i);
            const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int k = 0; k < 4; k++)
                m = max(max(m, w[k] >> 24), max(max(w[k] & 0xFFu, (w[k] >> 8) & 0xFFu), (w[k] >> 16) & 0xFFu));
        } else {
            for (uint64_t k = i; k < i + 16 && k < n; k++) m = max(m, (uint32_t)nh[k]);
        }
    }
#pragma unroll
    for (int sft = 32; sft >= 1; sft >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, sft, 64));
    if ((threadIdx.x & 63) == 0 && m) atomicMax(out + (blockIdx.x & (kMaxSpread - 1)), m);
}

hipError_t ensure_max_scratch(pkt_ctx* ctx) {
    if (ctx->mx.dev) return hipSuccess;
    static_assert(MaxScratch::kSpread == (int)kMaxSpread, "one spread");
    constexpr size_t bytes = MaxScratch::kGroups * MaxScratch::kSpread * sizeof(uint32_t);
    hipError_t e = hipMalloc(reinterpret_cast<void**>(&ctx->mx.dev), bytes);
    if (e == hipSuccess)
        e = hipHostMalloc(reinterpret_cast<void**>(&ctx->mx.host), bytes,
                          hipHostMallocDefault);
    if (e != hipSuccess) {
        (void)hipFree(ctx->mx.dev);
        ctx->mx.dev = nullptr;
        ctx->mx.host = nullptr;
    }
    return e;
}

// Queue the reduction of n_hdrs[0, n) into scratch word `w` and its copy to the host mirror on `s`.
hipError_t max_hdrs_async(pkt_ctx* ctx, const uint8_t* nh, uint64_t n, int w, hipStream_t s) {
    hipError_t e = hipMemsetAsync(ctx->mx.dgroup(w), 0, MaxScratch::kSpread * sizeof(uint32_t), s);
    if (e != hipSuccess) return e;
    if (n) {
        const unsigned grid = (unsigned)std::min<uint64_t>((n + 4095) / 4096, 1024);
        hipLaunchKernelGGL(max_hdrs_kernel, dim3(grid), dim3(256), 0, s, nh, n, ctx->mx.dgroup(w));
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    return hipMemcpyAsync(ctx->mx.hgroup(w), ctx->mx.dgroup(w), MaxScratch::kSpread * sizeof(uint32_t),
                          hipMemcpyDeviceToHost, s);
}

}  // namespace

extern "C" {

#if PKTGPU_STAMPS
// Diagnostic build only: where the parse kernel writes its per-wave stamps (8 u64 per wave:
// 5 s_memtime stamps, HW_ID, batch size).  NULL = none.
int pkt_debug_stamps(void* dev_buf) {
    return hipMemcpyToSymbol(HIP_SYMBOL(g_pkt_stamps), &dev_buf, sizeof(dev_buf)) == hipSuccess ? PKT_SUCCESS
                                                                                           : PKT_ERR_HIP;
}
#endif

int pkt_chain_max_hdrs(pkt_ctx_t* ctx, const uint8_t* n_hdrs, uint64_t n, uint32_t* max_out, void* stream) {
    if (!ctx || !max_out || (n && !n_hdrs)) return fail(ctx, PKT_ERR_INVALID_ARG, "null argument");
    hipError_t e = hipSetDevice(ctx->device);
    if (e == hipSuccess) e = ensure_max_scratch(ctx);
    if (e != hipSuccess) return hip_fail(ctx, e, "pkt_chain_max_hdrs scratch");
    const int w = MaxScratch::kGroups - 1;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if ((e = max_hdrs_async(ctx, n_hdrs, n, w, s)) != hipSuccess) return hip_fail(ctx, e, "max_hdrs_kernel");
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return hip_fail(ctx, e, "hipStreamSynchronize");
    *max_out = std::min<uint32_t>(ctx->mx.host_max(w), PKT_MAX_HDRS);
    return PKT_SUCCESS;
}

int pkt_ctx_create(int device, pkt_ctx_t** out) {
    if (!out) return PKT_ERR_INVALID_ARG;
    *out = nullptr;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count == 0) return PKT_ERR_NO_DEVICE;
    if (device < 0 || device >= count) return PKT_ERR_INVALID_ARG;
    pkt_ctx* c = new pkt_ctx();
    c->device = device;
    c->window = 0;
    c->fast = 1;
    c->staging = 0;
    c->walk = 0;
    *out = c;
    return PKT_SUCCESS;
}

int pkt_ctx_destroy(pkt_ctx_t* ctx) {
    if (ctx && ctx->tv_flag) {
        (void)hipSetDevice(ctx->device);
        (void)hipDeviceSynchronize();
        (void)hipFree(ctx->tv_flag);
        for (hipEvent_t ev : ctx->tv_ev)
            if (ev) (void)hipEventDestroy(ev);
    }
    if (ctx && (ctx->tv_win || ctx->tv_win_ev)) {
        (void)hipSetDevice(ctx->device);
        (void)hipDeviceSynchronize();
        if (ctx->tv_win) (void)hipFree(ctx->tv_win);
        if (ctx->tv_win_ev) (void)hipEventDestroy(ctx->tv_win_ev);
    }
    if (ctx && ctx->mx.dev) {
        (void)hipSetDevice(ctx->device);
        (void)hipDeviceSynchronize();
        (void)hipFree(ctx->mx.dev);
        (void)hipHostFree(ctx->mx.host);
    }
    if (ctx && (ctx->pc.buf || ctx->pc.ctl)) {
        (void)hipSetDevice(ctx->device);
        (void)hipDeviceSynchronize();
        (void)hipFree(ctx->pc.buf);
        (void)hipHostFree(ctx->pc.ctl);
    }
    if (ctx && ctx->hp.init) {
        (void)hipSetDevice(ctx->device);
        for (int k = 0; k < HostPipe::kSlots; k++) {
            (void)hipStreamSynchronize(ctx->hp.s[k]);
            (void)hipStreamDestroy(ctx->hp.s[k]);
            if (ctx->hp.ev[k]) (void)hipEventDestroy(ctx->hp.ev[k]);
            (void)hipFree(ctx->hp.slab[k]);
            (void)hipFree(ctx->hp.offs[k]);
            (void)hipFree(ctx->hp.lens[k]);
            (void)hipFree(ctx->hp.out[k]);
        }
        (void)hipFree(ctx->hp.file);
        (void)hipFree(ctx->hp.ioffs);
        (void)hipFree(ctx->hp.ilens);
        (void)hipFree(ctx->hp.pcarry);
        (void)hipFree(ctx->hp.pnh);
        (void)hipFree(ctx->hp.dcol);
        for (hipEvent_t x : ctx->hp.ev_copy)
            if (x) (void)hipEventDestroy(x);
        if (ctx->hp.ev_parsed) (void)hipEventDestroy(ctx->hp.ev_parsed);
        for (hipEvent_t x : ctx->hp.ev_xdone)
            if (x) (void)hipEventDestroy(x);
    }
    delete ctx;
    return PKT_SUCCESS;
}

const char* pkt_ctx_last_error(const pkt_ctx_t* ctx) { return ctx ? ctx->err.c_str() : "null ctx"; }

int pkt_ctx_set_window(pkt_ctx_t* ctx, uint32_t w) {
    if (!ctx) return PKT_ERR_INVALID_ARG;
    ctx->window = w;
    return PKT_SUCCESS;
}

int pkt_ctx_set_fastpath(pkt_ctx_t* ctx, int enable) {
    if (!ctx || enable < 0 || enable > 1) return PKT_ERR_INVALID_ARG;
    ctx->fast = enable;
    return PKT_SUCCESS;
}

int pkt_ctx_set_staging(pkt_ctx_t* ctx, int mode) {
    if (!ctx || mode < 0 || mode > 2) return PKT_ERR_INVALID_ARG;
    ctx->staging = mode;
    return PKT_SUCCESS;
}

int pkt_ctx_set_walk(pkt_ctx_t* ctx, int mode) {
    if (!ctx || mode < 0 || mode > 2) return PKT_ERR_INVALID_ARG;
    ctx->walk = mode;
    return PKT_SUCCESS;
}

int pkt_ctx_set_host_piece(pkt_ctx_t* ctx, uint64_t bytes) {
    if (!ctx || (bytes != 0 && bytes < 4096)) return PKT_ERR_INVALID_ARG;
    ctx->host_piece = bytes;
    return PKT_SUCCESS;
}

int pkt_ctx_set_pcap_scan64(pkt_ctx_t* ctx, int enable) {
    if (!ctx || enable < 0 || enable > 1) return PKT_ERR_INVALID_ARG;
    ctx->pc.scan64 = enable != 0;
    return PKT_SUCCESS;
}

static int parse_impl(pkt_ctx_t* ctx, const pkt_batch_t* b, int entry, const pkt_out_t* out,
                      void* stream, uint64_t off_bias, int staging, uint32_t* nh_max = nullptr,
                      uint64_t slot_stride = 0, MultiParams* mp = nullptr, const uint64_t* n_dev = nullptr,
                      const uint64_t* i0_dev = nullptr, uint64_t grid_n = 0);

int pkt_parse_batch(pkt_ctx_t* ctx, const pkt_batch_t* b, int entry, const pkt_out_t* out,
                    void* stream) {
    // the kernel reads whole 16-byte chunks, clamped to the last one of the slab
    if (b && b->n && b->slab_len < 16) return fail(ctx, PKT_ERR_INVALID_ARG, "slab_len < 16");
    return parse_impl(ctx, b, entry, out, stream, 0, ctx ? ctx->staging : 0);
}

int pkt_parse_batches(pkt_ctx_t* ctx, const pkt_batch_t* batches, uint32_t nbatch, int entry, const pkt_out_t* outs,
                      void* stream) {
    if (!ctx || (nbatch && (!batches || !outs))) return fail(ctx, PKT_ERR_INVALID_ARG, "null argument");
    // One launch when the batches share size and layout and their outputs sit at one common byte
    // distance from batch 0's (per column); otherwise one pkt_parse_batch each (same results).
    bool one = nbatch >= 2 && nbatch <= (uint32_t)kMaxMulti && ctx->staging != 2;
    const pkt_batch_t& b0 = batches[0];
    const void* const* c0 = nbatch ? reinterpret_cast<const void* const*>(&outs[0]) : nullptr;
    MultiParams mp;
    for (uint32_t k = 0; k < nbatch && one; k++) {
        const pkt_batch_t& b = batches[k];
        one = b.n == b0.n && b.n > 0 && b.n <= kLaunchChunk && b.stride == b0.stride &&
              (b.offsets == nullptr) == (b0.offsets == nullptr) && (b.lens == nullptr) == (b0.lens == nullptr) &&
              b.slab && ((uintptr_t)b.slab & 15) == 0 && b.slab_len >= 16;
        const void* const* ck = reinterpret_cast<const void* const*>(&outs[k]);
        int64_t delta = 0;
        bool have = false;
        for (int c = 0; c < 49 && one; c++) {
            if ((ck[c] == nullptr) != (c0[c] == nullptr)) one = false;
            if (!ck[c]) continue;
            const int64_t d = (int64_t)((uintptr_t)ck[c] - (uintptr_t)c0[c]);
            if (have && d != delta) one = false;
            delta = d;
            have = true;
        }
        // batch k's IPv6 address columns are batch 0's + delta: the 16-byte alignment parse_impl
        // checks for batch 0 holds for every batch only if delta keeps it (else one call per batch,
        // each validated)
        if ((c0[kColIpv6Src] || c0[kColIpv6Dst]) && (delta & 15) != 0) one = false;
        if (one) mp.per[k] = MultiBatch{b.slab, b.slab_len, b.offsets, b.lens, delta};
    }
    if (!one) {
        for (uint32_t k = 0; k < nbatch; k++) {
            const int rc = pkt_parse_batch(ctx, &batches[k], entry, &outs[k], stream);
            if (rc != PKT_SUCCESS) return rc;
        }
        return PKT_SUCCESS;
    }
    mp.k = nbatch;
    mp.bpb = (uint32_t)((b0.n + kBlock - 1) / kBlock);
    return parse_impl(ctx, &b0, entry, &outs[0], stream, 0, ctx->staging, nullptr, 0, &mp);
}

}  // extern "C"

// (internal, pktgpu_ctx.hpp) pkt_parse_batch with the count from the device.
int pktgpu_parse_counted(pkt_ctx_t* ctx, const pkt_batch_t* b, int entry, const pkt_out_t* out, void* stream,
                         const uint64_t* count_dev, uint64_t slot_stride) {
    if (b && b->n && b->slab_len < 16) return fail(ctx, PKT_ERR_INVALID_ARG, "slab_len < 16");
    if (count_dev && b && b->n > kLaunchChunk) return fail(ctx, PKT_ERR_INVALID_ARG, "device count over 2^26 packets");
    return parse_impl(ctx, b, entry, out, stream, 0, ctx ? ctx->staging : 0, nullptr, slot_stride, nullptr, count_dev);
}

// (internal, pktgpu_ctx.hpp) pkt_parse_batch whose kernel also reduces the batch's largest n_hdrs
// (a wave max + one atomicMax per wave, fused into the parse) into a ctx word, copied to the ctx's
// pinned mirror on `stream`: *rows_host holds it once the stream has passed this call.
int pktgpu_parse_rows_async(pkt_ctx_t* ctx, const pkt_batch_t* b, int entry, const pkt_out_t* out, void* stream,
                            const uint32_t** rows_host) {
    if (!ctx || !rows_host) return fail(ctx, PKT_ERR_INVALID_ARG, "null argument");
    if (b && b->n && b->slab_len < 16) return fail(ctx, PKT_ERR_INVALID_ARG, "slab_len < 16");
    hipError_t e = hipSetDevice(ctx->device);
    if (e == hipSuccess) e = ensure_max_scratch(ctx);
    if (e != hipSuccess) return hip_fail(ctx, e, "parse rows scratch");
    const int w = MaxScratch::kGroups - 1;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if ((e = hipMemsetAsync(ctx->mx.dgroup(w), 0, MaxScratch::kSpread * sizeof(uint32_t), s)) != hipSuccess)
        return hip_fail(ctx, e, "hipMemsetAsync");
    const int rc = parse_impl(ctx, b, entry, out, stream, 0, ctx->staging, ctx->mx.dgroup(w));
    if (rc != PKT_SUCCESS) return rc;
    if ((e = hipMemcpyAsync(ctx->mx.hgroup(w), ctx->mx.dgroup(w), MaxScratch::kSpread * sizeof(uint32_t),
                            hipMemcpyDeviceToHost, s)) != hipSuccess)
        return hip_fail(ctx, e, "hipMemcpyAsync (rows)");
    *rows_host = ctx->mx.hgroup(w);
    return PKT_SUCCESS;
}

extern "C" {

// `staging` = the ctx's knob, or the host path's override (wave spans over the link).
// i0_dev / grid_n (with n_dev, one launch): the launch parses packets [*i0_dev (or 0), min(b->n, *n_dev))
// with a grid for grid_n packets (the most the device-produced range can hold; 0 = b->n).
static int parse_impl(pkt_ctx_t* ctx, const pkt_batch_t* b, int entry, const pkt_out_t* out,
                      void* stream, uint64_t off_bias, int staging, uint32_t* nh_max, uint64_t slot_stride,
                      MultiParams* mp, const uint64_t* n_dev, const uint64_t* i0_dev, uint64_t grid_n) {
    if (!ctx || !b || !out) return fail(ctx, PKT_ERR_INVALID_ARG, "null argument");
    if (entry < 0 || entry >= PKT_ENTRY_COUNT) return fail(ctx, PKT_ERR_INVALID_ARG, "bad entry");
    if (b->n == 0) return PKT_SUCCESS;
    if (!b->slab) return fail(ctx, PKT_ERR_INVALID_ARG, "null slab");
    if (((uintptr_t)b->slab & 15) != 0) return fail(ctx, PKT_ERR_INVALID_ARG, "slab not 16-byte aligned");
    if (b->offsets && !b->lens) return fail(ctx, PKT_ERR_INVALID_ARG, "offsets without lens");
    if (!b->offsets && b->stride == 0) return fail(ctx, PKT_ERR_INVALID_ARG, "stride 0");
    if (out->ipv6_src && ((uintptr_t)out->ipv6_src & 15)) return fail(ctx, PKT_ERR_INVALID_ARG, "ipv6_src not 16-byte aligned");
    if (out->ipv6_dst && ((uintptr_t)out->ipv6_dst & 15)) return fail(ctx, PKT_ERR_INVALID_ARG, "ipv6_dst not 16-byte aligned");
    if (b->slab_len == 0) return fail(ctx, PKT_ERR_INVALID_ARG, "slab_len 0");
    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) return hip_fail(ctx, e, "hipSetDevice");

    // Window: bytes of each packet staged in LDS.  Fixed stride: the slot (up to 128 B);
    // indexed: 128 B.  Unaligned packet starts need one more chunk.
    uint32_t w = ctx->window;
    // Auto window: the stride up to 64 bytes for fixed-stride slabs (Ether[/Vlan x2]/IPv4/TCP ends at
    // byte 62); 80 bytes for indexed batches (96 from the record's 16-byte-aligned start: every
    // header of 16 of the 22 reference templates, the rest read past it through L2).  C4 per 2^20
    // records, same box, 2 streams: 80 B 46.6 (chain) / 68.1 us (all columns), 64 B 49.4 / 75.8,
    // 96 B 49.6 / 69.1, 128 B 59.7 / 77.4 — wider windows read fewer lines twice but hold fewer
    // waves per CU (LDS), round 3.  (Round 4: windows packed from the record's first
    // byte — 80 or 96 packet bytes in 84 or 100 B of LDS per record, 7 or 6 blocks per CU — were
    // slower than this layout in every combination: C4 all columns 72.6-74.1 vs 69.9 us, chain
    // 52.6-57.7 vs 50.4 us per 2-stream step; the unaligned LDS stores of the staging cost more than
    // the occupancy or the lines they save, profiles/ab/r04c_c4_packed_windows.txt.)
    if (w == 0) w = b->offsets ? 80u : std::min<uint32_t>(std::max<uint32_t>(b->stride, 16u), 64u);
    w = std::min<uint32_t>(std::max<uint32_t>((w + 15) & ~15u, 16u), 256u);
    bool aligned = !b->offsets && (b->stride % 16 == 0);
    int nch = (int)(w / 16) + (aligned ? 0 : 1);

    uint32_t full, any;
    group_masks(*out, full, any);
    const uint32_t gm = (full == any) ? full : G_RUNTIME;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    // Staging: wave spans when asked; per-lane windows otherwise (auto: spans measured slower on
    // device-resident C3 and C4).
    const int mode = staging == 2 ? M_SPAN : M_TILE;
    // Walk: lockstep for indexed batches (pcap replays mix chains within a wave), waterfall for
    // fixed-stride slabs (one layout per wave), unless the ctx says otherwise.
    const int wk = ctx->walk == 2 ? 1 : ctx->walk == 1 ? 0 : (b->offsets ? 1 : 0);
    if (wk == 1 && nch < 6) nch = 6;  // the narrowest lockstep build
    for (uint64_t i0 = 0; i0 < b->n && e == hipSuccess; i0 += kLaunchChunk) {
        const uint64_t cnt = std::min<uint64_t>(kLaunchChunk, b->n - i0);
        KParams kp;
        kp.slab = b->slab;
        kp.slab_len = b->slab_len;
        kp.offsets = adv(b->offsets, i0);
        kp.lens = adv(b->lens, i0);
        kp.off_bias = off_bias;
        kp.i0 = i0;
        kp.n_slot_stride = slot_stride ? slot_stride : b->n;  // the slot columns' row stride
        kp.stride = b->stride;
        kp.n = (uint32_t)cnt;
        kp.entry = entry;
        kp.fast = ctx->fast && (entry == PKT_ENTRY_PARSE || entry == PKT_ENTRY_ETHERNET);
        kp.nh_max = nh_max;
        kp.n_dev = n_dev;  // (one launch: n_dev is only passed for batches of n <= kLaunchChunk)
        kp.i0_dev = n_dev ? i0_dev : nullptr;
        pkt_out_t o = *out;
        uint8_t** oc = reinterpret_cast<uint8_t**>(&o);
        for (int c = 0; c < 49; c++)
            if (oc[c]) oc[c] += i0 * kColSize[c];
        kp.out = o;
        if (mp) mp->base = kp;  // batch 0 of a multi-batch launch (n <= kLaunchChunk: one chunk)
        // the launch's grid: kp.n packets, or grid_n when the range starts at a device-produced index
        const uint32_t gn = (kp.n_dev && grid_n) ? (uint32_t)std::min<uint64_t>(grid_n, cnt) : kp.n;
        const int md = mp ? M_TILE : mode;
        // compiled window widths (chunks): a request between two is served by the wider one
        if (nch <= 2) e = launch_gm<2>(kp, gm, md, wk, s, mp, gn);
        else if (nch <= 4) e = launch_gm<4>(kp, gm, md, wk, s, mp, gn);
        else if (nch <= 5) e = launch_gm<5>(kp, gm, md, wk, s, mp, gn);
        else if (nch <= 6) e = launch_gm<6>(kp, gm, md, wk, s, mp, gn);
        else if (nch <= 7 && wk == 1) e = launch_gm<7>(kp, gm, md, wk, s, mp, gn);
        else if (nch <= 9) e = launch_gm<9>(kp, gm, md, wk, s, mp, gn);
        else e = launch_gm<17>(kp, gm, md, wk, s, mp, gn);
    }
    if (e != hipSuccess) return hip_fail(ctx, e, "parse_kernel launch");
    return PKT_SUCCESS;
}

int pkt_host_alloc(pkt_ctx_t* ctx, uint64_t bytes, void** p) {
    if (!ctx || !p) return fail(ctx, PKT_ERR_INVALID_ARG, "null argument");
    *p = nullptr;
    hipError_t e = hipSetDevice(ctx->device);
    if (e == hipSuccess) e = hipHostMalloc(p, bytes ? bytes : 1, hipHostMallocDefault);
    return e == hipSuccess ? PKT_SUCCESS : hip_fail(ctx, e, "hipHostMalloc");
}

int pkt_host_free(pkt_ctx_t* ctx, void* p) {
    if (!p) return PKT_SUCCESS;
    hipError_t e = hipHostFree(p);
    return e == hipSuccess ? PKT_SUCCESS : hip_fail(ctx, e, "hipHostFree");
}

// The staged host pipeline: the batch cut into chunks of `cn` packets over the ctx's three streams,
// each chunk parsed into a device output slot and its columns copied to the host rows (the slot rows
// once the chunk's n_hdrs maximum, reduced inside its parse, is known — one chunk later, so the host
// never waits on the chunk it has just queued).  dev_in = false: `b` is host memory and each chunk's
// bytes (+ offsets / lens) are copied in first; dev_in = true: `b` is already in device memory.
// hout (non-NULL: every requested host column is pinned, these are their device-mapped addresses): each
// chunk's columns leave by one export_kernel launch writing 16-byte chunks over the link (pktgpu_gather.hip)
// instead of one DMA copy per column — ~30 small copies per chunk, each with its own setup.
static int staged_parse(pkt_ctx_t* ctx, const pkt_batch_t* b, int entry, const pkt_out_t* out, uint64_t chunk,
                        bool dev_in, uint64_t slot_stride = 0, const pkt_out_t* hout = nullptr) {
    HostPipe& hp = ctx->hp;
    hipError_t e = hipSuccess;
    const uint64_t n = b->n, hstride = slot_stride ? slot_stride : n;  // host slot rows: [16][hstride]
    const uint64_t cn = std::min<uint64_t>(chunk ? chunk : (hout ? (1ull << 17) : (1ull << 18)), n);
    const uint64_t nchunks = (n + cn - 1) / cn;

    // bytes of input each chunk needs on the device (indexed: the span its records cover,
    // from the 16-byte-aligned start of the first)
    auto span = [&](uint64_t lo, uint64_t hi, uint64_t& base, uint64_t& bytes) {
        uint64_t a = UINT64_MAX, z = 0;
        if (b->offsets) {
            for (uint64_t i = lo; i < hi; i++) {
                a = std::min(a, b->offsets[i]);
                z = std::max(z, b->offsets[i] + b->lens[i]);
            }
        } else {
            a = lo * (uint64_t)b->stride;
            z = hi * (uint64_t)b->stride;
        }
        a = std::min(a, b->slab_len);
        if (b->offsets) a &= ~(uint64_t)15;  // fixed stride: the chunk starts at its first packet
        z = std::min(z, b->slab_len);
        base = a;
        bytes = z > a ? z - a : 0;
    };
    uint64_t slab_need = 16;
    if (!dev_in)
        for (uint64_t k = 0; k < nchunks; k++) {
            uint64_t base, bytes;
            span(k * cn, std::min(n, (k + 1) * cn), base, bytes);
            slab_need = std::max(slab_need, bytes);
        }
    // device output layout of one chunk: the requested columns, packed, 256-byte aligned
    const uint8_t* const* hcol = reinterpret_cast<const uint8_t* const*>(out);
    uint64_t col_off[49], out_need = 0;
    for (int c = 0; c < 49; c++) {
        col_off[c] = out_need;
        if (!hcol[c]) continue;
        const uint64_t rows = (c == kColHdrType || c == kColHdrOff) ? PKT_MAX_HDRS : 1;
        out_need += (rows * cn * kColSize[c] + 255) & ~(uint64_t)255;
    }
    for (int k = 0; k < HostPipe::kSlots; k++) (void)hipStreamSynchronize(hp.s[k]);
    if ((!dev_in && (e = grow(hp.slab, hp.slab_cap, (slab_need + 15) & ~(uint64_t)15)) != hipSuccess) ||
        (e = grow(hp.out, hp.out_cap, std::max<uint64_t>(out_need, 256))) != hipSuccess)
        return hip_fail(ctx, e, "hipMalloc (host pipeline)");
    if (!dev_in && (b->offsets || b->lens)) {
        uint64_t cap8 = hp.pkt_cap, cap4 = hp.pkt_cap;
        if ((e = grow(hp.offs, cap8, cn * 8)) != hipSuccess || (e = grow(hp.lens, cap4, cn * 8)) != hipSuccess)
            return hip_fail(ctx, e, "hipMalloc (host pipeline)");
        hp.pkt_cap = std::min(cap8, cap4);
    }

    // Slot rows move only as far as each chunk's largest n_hdrs (when n_hdrs is requested)
    const bool slot_rows = (hcol[kColHdrType] || hcol[kColHdrOff]) && hcol[1] != nullptr;
    if (slot_rows && (e = ensure_max_scratch(ctx)) != hipSuccess) return hip_fail(ctx, e, "max scratch");
    auto copy_slots = [&](uint64_t kk) -> hipError_t {  // chunk kk's slot rows [0, R) to the host
        const int q = (int)(kk % HostPipe::kSlots);
        const uint64_t lo = kk * cn, m = std::min(n, lo + cn) - lo;
        uint32_t rows = PKT_MAX_HDRS;
        if (slot_rows) {
            hipError_t es = hipEventSynchronize(hp.ev[q]);
            if (es != hipSuccess) return es;
            rows = std::min<uint32_t>(ctx->mx.host_max(q), PKT_MAX_HDRS);
        }
        for (int c : {kColHdrType, kColHdrOff}) {
            if (!hcol[c] || !rows) continue;
            const uint64_t sz = kColSize[c];
            hipError_t es = hipMemcpy2DAsync(const_cast<uint8_t*>(hcol[c]) + lo * sz, hstride * sz, hp.out[q] + col_off[c],
                                             m * sz, m * sz, rows, hipMemcpyDeviceToHost, hp.s[q]);
            if (es != hipSuccess) return es;
        }
        return hipSuccess;
    };
    int rc = PKT_SUCCESS;
    for (uint64_t k = 0; k < nchunks && rc == PKT_SUCCESS; k++) {
        const int q = (int)(k % HostPipe::kSlots);
        hipStream_t s = hp.s[q];
        const uint64_t lo = k * cn, hi = std::min(n, lo + cn), m = hi - lo;
        pkt_batch_t db;
        uint64_t bias = 0;
        if (dev_in) {
            db = *b;
            if (b->offsets) {
                db.offsets = b->offsets + lo;
                db.lens = b->lens + lo;
            } else {
                const uint64_t a = std::min<uint64_t>(lo * (uint64_t)b->stride, b->slab_len);
                db.slab = b->slab + a;  // 16-byte aligned: stride % 16 == 0 is checked by the caller
                db.slab_len = std::max<uint64_t>(b->slab_len - a, 16);
                if (b->lens) db.lens = b->lens + lo;
            }
            db.n = m;
        } else {
            uint64_t base, bytes;
            span(lo, hi, base, bytes);
            // in: the chunk's bytes (+ offsets / lens)
            if (bytes) e = hipMemcpyAsync(hp.slab[q], b->slab + base, bytes, hipMemcpyHostToDevice, s);
            if (e == hipSuccess && b->offsets)
                e = hipMemcpyAsync(hp.offs[q], b->offsets + lo, m * 8, hipMemcpyHostToDevice, s);
            if (e == hipSuccess && b->lens)
                e = hipMemcpyAsync(hp.lens[q], b->lens + lo, m * 4, hipMemcpyHostToDevice, s);
            if (e != hipSuccess) { rc = hip_fail(ctx, e, "hipMemcpyAsync H2D"); break; }
            // a chunk whose records cover no byte still parses (all TRUNCATED) against a 1-byte view;
            // fixed-stride chunks index from the chunk's first packet
            db.slab = hp.slab[q];
            db.slab_len = std::max<uint64_t>(bytes, 1);
            db.offsets = b->offsets ? hp.offs[q] : nullptr;
            db.lens = b->lens ? hp.lens[q] : nullptr;
            db.stride = b->stride;
            db.reserved = 0;
            db.n = m;
            bias = b->offsets ? base : 0;
        }
        pkt_out_t dout;
        uint8_t** dcol = reinterpret_cast<uint8_t**>(&dout);
        for (int c = 0; c < 49; c++) dcol[c] = hcol[c] ? hp.out[q] + col_off[c] : nullptr;
        // (the device buffer always has >= 16 readable bytes, so a view shorter than 16 is safe)
        if (slot_rows && (e = hipMemsetAsync(ctx->mx.dgroup(q), 0, MaxScratch::kSpread * sizeof(uint32_t), s)) != hipSuccess) {
            rc = hip_fail(ctx, e, "hipMemsetAsync");
            break;
        }
        rc = parse_impl(ctx, &db, entry, &dout, s, bias, ctx->staging, slot_rows ? ctx->mx.dgroup(q) : nullptr);
        if (rc != PKT_SUCCESS) break;
        if (hout) {  // every column of the chunk by one export launch (slot rows up to the chunk's n_hdrs max)
            ExportArgs xa;
            xa.ncol = 0;
            xa.lo_dev = xa.hi_dev = nullptr;
            xa.lo_h = 0;
            xa.hi_h = m;
            xa.cap = m;
            xa.nhw = slot_rows ? ctx->mx.dgroup(q) : nullptr;
            const uint8_t* const* hm = reinterpret_cast<const uint8_t* const*>(hout);
            for (int c = 0; c < 49; c++) {
                if (!hcol[c]) continue;
                const bool slot = c == kColHdrType || c == kColHdrOff;
                const uint64_t sz = kColSize[c];
                for (uint32_t r = 0; r < (slot ? (uint32_t)PKT_MAX_HDRS : 1u); r++)
                    xa.col[xa.ncol++] = ExportCol{reinterpret_cast<uint64_t>(dcol[c]) + (uint64_t)r * m * sz,
                                                  reinterpret_cast<uint64_t>(hm[c]) + ((uint64_t)r * hstride + lo) * sz,
                                                  (uint32_t)sz, slot ? r : kExportNoRow};
            }
            if ((e = pktgpu_export_launch(xa, s)) != hipSuccess) {
                rc = hip_fail(ctx, e, "export_kernel");
                break;
            }
            continue;
        }
        // out: every requested per-packet column into its host rows [lo, hi); the slot rows of this
        // chunk once its count is known (after the next chunk is queued)
        for (int c = 0; c < 49 && e == hipSuccess; c++) {
            if (!hcol[c] || c == kColHdrType || c == kColHdrOff) continue;
            const uint64_t sz = kColSize[c];
            e = hipMemcpyAsync(const_cast<uint8_t*>(hcol[c]) + lo * sz, dcol[c], m * sz, hipMemcpyDeviceToHost, s);
        }
        if (e == hipSuccess && slot_rows) {
            e = hipMemcpyAsync(ctx->mx.hgroup(q), ctx->mx.dgroup(q), MaxScratch::kSpread * sizeof(uint32_t),
                               hipMemcpyDeviceToHost, s);
            if (e == hipSuccess) e = hipEventRecord(hp.ev[q], s);
        }
        if (e == hipSuccess && k > 0) e = copy_slots(k - 1);
        if (e != hipSuccess) rc = hip_fail(ctx, e, "hipMemcpyAsync D2H");
    }
    if (rc == PKT_SUCCESS && nchunks > 0 && !hout) {
        e = copy_slots(nchunks - 1);
        if (e != hipSuccess) rc = hip_fail(ctx, e, "hipMemcpyAsync D2H");
    }
    for (int k = 0; k < HostPipe::kSlots; k++) {
        hipError_t es = hipStreamSynchronize(hp.s[k]);
        if (es != hipSuccess && rc == PKT_SUCCESS) rc = hip_fail(ctx, es, "hipStreamSynchronize");
    }
    return rc;
}

static int host_pipe_init(pkt_ctx_t* ctx) {
    HostPipe& hp = ctx->hp;
    if (hp.init) return PKT_SUCCESS;
    for (int k = 0; k < HostPipe::kSlots; k++) {
        hipError_t e = hipStreamCreateWithFlags(&hp.s[k], hipStreamNonBlocking);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&hp.ev[k], hipEventDisableTiming);
        if (e != hipSuccess) return hip_fail(ctx, e, "hipStreamCreate");
    }
    hp.init = true;
    return PKT_SUCCESS;
}

// Are the requested columns of `out` all pinned host memory mapped into the device?  `dout` = the
// same columns by their device addresses.
static bool out_mapped(const pkt_out_t* out, pkt_out_t& dout) {
    dout = *out;
    uint8_t** dc = reinterpret_cast<uint8_t**>(&dout);
    bool mapped = true;
    for (int c = 0; c < 49 && mapped; c++)
        if (dc[c]) mapped = host_mapped(dc[c], dc[c]);
    return mapped;
}

int pkt_parse_host(pkt_ctx_t* ctx, const pkt_batch_t* b, int entry, const pkt_out_t* out, uint64_t chunk) {
    if (!ctx || !b || !out) return fail(ctx, PKT_ERR_INVALID_ARG, "null argument");
    if (entry < 0 || entry >= PKT_ENTRY_COUNT) return fail(ctx, PKT_ERR_INVALID_ARG, "bad entry");
    if (b->n == 0) return PKT_SUCCESS;
    if (!b->slab || b->slab_len == 0) return fail(ctx, PKT_ERR_INVALID_ARG, "null or empty slab");
    if (b->offsets && !b->lens) return fail(ctx, PKT_ERR_INVALID_ARG, "offsets without lens");
    if (!b->offsets && b->stride == 0) return fail(ctx, PKT_ERR_INVALID_ARG, "stride 0");
    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) return hip_fail(ctx, e, "hipSetDevice");
    int rc = host_pipe_init(ctx);
    if (rc != PKT_SUCCESS) return rc;
    HostPipe& hp = ctx->hp;
    // Zero copy: when the slab, the index arrays and every requested column are pinned host memory
    // mapped into the device (pkt_host_alloc), the kernel reads and writes them over PCIe directly —
    // one launch, no staging copies, both link directions busy at once.  (Chunks copied
    // in by DMA, parsed on the device and their columns exported by a kernel writing 16-byte chunks —
    // the route the piecewise capture takes — measured slower here: C2 2.10 vs 1.86 ms, C4 6.63 vs
    // 6.28 ms per 2^20 packets, profiles/host/r05e_host_export_vs_zero_copy.jsonl; it serves pinned
    // columns of a pageable slab instead of one DMA copy per column.)
    {
        pkt_batch_t db = *b;
        pkt_out_t dout;
        const bool omap = out_mapped(out, dout);
        const bool mapped = omap && host_mapped(b->slab, db.slab) && (!b->offsets || host_mapped(b->offsets, db.offsets)) &&
                            (!b->lens || host_mapped(b->lens, db.lens));
        if (omap && !(mapped && ((uintptr_t)db.slab & 15) == 0 && b->slab_len >= 16))
            return staged_parse(ctx, b, entry, out, chunk, false, 0, &dout);
        if (mapped && ((uintptr_t)db.slab & 15) == 0 && b->slab_len >= 16) {
            // wave spans read the link in 1-KiB contiguous pieces and never go back to host memory
            // for a deep header (per-lane windows would, one dependent PCIe read each)
            rc = parse_impl(ctx, &db, entry, &dout, hp.s[0], 0, ctx->staging == 0 ? 2 : ctx->staging);
            if (rc != PKT_SUCCESS) return rc;
            e = hipStreamSynchronize(hp.s[0]);
            return e == hipSuccess ? PKT_SUCCESS : hip_fail(ctx, e, "hipStreamSynchronize");
        }
    }
    return staged_parse(ctx, b, entry, out, chunk, false);
}

}  // extern "C"

// The host pipeline's streams and the capture's device buffers (file + index, grown on demand; +16:
// the kernels' readable tail), after the ctx's earlier host-path work has finished.
static int pcap_host_buffers(pkt_ctx_t* ctx, uint64_t len, uint64_t cap) {
    if (ctx->pc.pending)
        return fail(ctx, PKT_ERR_INVALID_ARG, "a queued capture's outcome has not been taken on this ctx (pkt_parse_pcap_result)");
    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) return hip_fail(ctx, e, "hipSetDevice");
    int rc = host_pipe_init(ctx);
    if (rc != PKT_SUCCESS) return rc;
    HostPipe& hp = ctx->hp;
    for (int k = 0; k < HostPipe::kSlots; k++) (void)hipStreamSynchronize(hp.s[k]);
    const uint64_t fbytes = ((len + 15) & ~(uint64_t)15) + 16;
    if (fbytes > hp.file_cap) {
        (void)hipFree(hp.file);
        hp.file = nullptr;
        hp.file_cap = 0;
        if ((e = hipMalloc(reinterpret_cast<void**>(&hp.file), fbytes + fbytes / 4)) != hipSuccess)
            return hip_fail(ctx, e, "hipMalloc (pcap file)");
        hp.file_cap = fbytes + fbytes / 4;
    }
    if (cap > hp.idx_cap) {
        (void)hipFree(hp.ioffs);
        (void)hipFree(hp.ilens);
        hp.ioffs = nullptr;
        hp.ilens = nullptr;
        hp.idx_cap = 0;
        const uint64_t c2 = cap + cap / 4;
        e = hipMalloc(reinterpret_cast<void**>(&hp.ioffs), c2 * 8);
        if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&hp.ilens), c2 * 4);
        if (e != hipSuccess) return hip_fail(ctx, e, "hipMalloc (pcap index)");
        hp.idx_cap = c2;
    }
    return PKT_SUCCESS;
}

// A capture indexed and parsed as its bytes arrive (pkt_parse_pcap_host's pieces, pkt_pcap_stream_*), on
// the ctx's three host streams: hp.s[1] copies bytes in; hp.s[0] runs one STEP per batch of new bytes —
// the device indexer over the new regions only (segment mode: it starts from the previous step's carry,
// the first record start that step did not count and its record count, kept in device words, so the
// whole capture is indexed once, O(file), however many steps) and the parse of the records the step
// added into the device columns; hp.s[2] exports those records' column ranges to the caller's pinned
// columns in 16-byte chunks while the next bytes copy in (the link is full duplex).  The parse kernel
// writing the host columns itself (its 1-8 B per-lane stores over the link) moved them at ~21 GB/s
// against ~57 GB/s for wide chunks (profiles/host/r05b_pcap_host_pieces.jsonl).  The records a step adds
// all end in (its start, its end] and are disjoint (>= 16 B each): at most (end - start) / 16 + 1 of
// them, which sizes the step's parse grid.  Nothing on the host waits for the device between steps.
struct Ingest {
    pkt_ctx_t* ctx = nullptr;
    int entry = 0;
    uint64_t cap = 0;      // records the columns hold (slot rows strided by cap)
    pkt_out_t dcols{};     // the parse's output: the caller's device columns or the ctx's hp.dcol
    bool exporting = false;
    ExportArgs xa{};       // exporting: hp.dcol -> the caller's pinned columns
    uint64_t hi = 0;       // bytes copied to the device (hp.file[0, hi)), queued
    uint64_t indexed = 0;  // the prefix the last step indexed
    uint64_t steps = 0;
    uint64_t copies = 0;   // copies queued; copy c ends the capture's first copy_end[c % kCopyRing] bytes
    uint64_t copy_end[HostPipe::kCopyRing] = {};
    int rc = PKT_SUCCESS;  // the first failure (every later call returns it)
};
constexpr uint64_t kHostPiece = 16ull << 20;  // pkt_parse_pcap_host: default bytes per copied piece
static int pcap_host_pieces(pkt_ctx_t* ctx, const uint8_t* buf, uint64_t len, int entry, const pkt_out_t* out,
                            const pkt_out_t& hout, uint64_t* offsets, uint32_t* lens, uint64_t cap,
                            uint64_t* n_out, uint64_t piece, bool blocking);

extern "C" {

int pkt_parse_pcap_host_async(pkt_ctx_t* ctx, const uint8_t* buf, uint64_t len, int entry, const pkt_out_t* out,
                              uint64_t cap) {
    if (!ctx || !buf || !out || !cap) return fail(ctx, PKT_ERR_INVALID_ARG, "null argument");
    if (entry < 0 || entry >= PKT_ENTRY_COUNT) return fail(ctx, PKT_ERR_INVALID_ARG, "bad entry");
    if (cap > kLaunchChunk) return fail(ctx, PKT_ERR_INVALID_ARG, "pkt_parse_pcap_host_async: cap > 2^26 records");
    pkt_out_t dout;
    if (!out_mapped(out, dout))
        return fail(ctx, PKT_ERR_INVALID_ARG, "pkt_parse_pcap_host_async: the columns must be pinned (pkt_host_alloc)");
    int rc = pcap_host_buffers(ctx, len, cap);
    if (rc != PKT_SUCCESS) return rc;
    if (len < 24) return fail(ctx, PKT_ERR_INVALID_ARG, "pcap shorter than its global header");
    uint64_t n_unused = 0;
    // the blocking call's pieces, queued on the ctx's three streams (pkt_parse_pcap_host_result waits)
    return pcap_host_pieces(ctx, buf, len, entry, out, dout, nullptr, nullptr, cap, &n_unused,
                            ctx->host_piece ? ctx->host_piece : kHostPiece, false);
}

int pkt_parse_pcap_host_result(pkt_ctx_t* ctx, uint64_t* n_out) {
    if (!ctx || !n_out) return fail(ctx, PKT_ERR_INVALID_ARG, "null argument");
    *n_out = 0;
    if (ctx->pc.pending && ctx->hp.init) {  // the copy and export streams of the queued capture
        (void)hipSetDevice(ctx->device);
        const hipError_t e1 = hipStreamSynchronize(ctx->hp.s[1]), e2 = hipStreamSynchronize(ctx->hp.s[2]);
        if (e1 != hipSuccess || e2 != hipSuccess) {
            uint64_t ignored = 0;
            (void)pktgpu_pcap_take(ctx, &ignored);
            return hip_fail(ctx, e1 != hipSuccess ? e1 : e2, "pkt_parse_pcap_host_result");
        }
    }
    return pktgpu_pcap_take(ctx, n_out);
}

}  // extern "C"

static int ingest_fail(Ingest& ig, int code) {  // nothing left in flight that reads the caller's bytes
    HostPipe& hp = ig.ctx->hp;
    for (int k = 0; k < HostPipe::kSlots; k++) (void)hipStreamSynchronize(hp.s[k]);
    if (ig.rc == PKT_SUCCESS) ig.rc = code;
    return code;
}

// The buffers, ring and events of a capture of up to len_cap bytes and cap records into `out`: pinned host
// columns (hout = their device addresses: the parse writes hp.dcol, exported after each step) or the
// caller's device columns (hout NULL: the parse writes them).  Waits for the ctx's earlier host-path work.
static int ingest_begin(Ingest& ig, pkt_ctx_t* ctx, uint64_t len_cap, uint64_t cap, int entry, const pkt_out_t* out,
                        const pkt_out_t* hout) {
    ig.ctx = ctx;
    ig.entry = entry;
    ig.cap = cap;
    ig.hi = ig.indexed = ig.steps = ig.copies = 0;
    ig.rc = PKT_SUCCESS;
    int rc = pcap_host_buffers(ctx, len_cap, cap);
    if (rc != PKT_SUCCESS) return rc;
    HostPipe& hp = ctx->hp;
    hipError_t e = hipSuccess;
    if (!hp.pcarry) e = hipMalloc(reinterpret_cast<void**>(&hp.pcarry), HostPipe::kRing * kPcapCarryWords * 8);
    if (e == hipSuccess && !hp.pnh) e = hipMalloc(reinterpret_cast<void**>(&hp.pnh), HostPipe::kRing * kMaxSpread * 4);
    for (int j = 0; j < HostPipe::kCopyRing && e == hipSuccess; j++)
        if (!hp.ev_copy[j]) e = hipEventCreateWithFlags(&hp.ev_copy[j], hipEventDisableTiming);
    if (e == hipSuccess && !hp.ev_parsed) e = hipEventCreateWithFlags(&hp.ev_parsed, hipEventDisableTiming);
    for (int j = 0; j < HostPipe::kRing && e == hipSuccess; j++)
        if (!hp.ev_xdone[j]) e = hipEventCreateWithFlags(&hp.ev_xdone[j], hipEventDisableTiming);
    if (e != hipSuccess) return hip_fail(ctx, e, "capture ring");
    ig.exporting = hout != nullptr;
    if (!ig.exporting) {
        ig.dcols = *out;
    } else {
        // the device columns: the requested ones, each at a 256-byte boundary, the caller's shapes
        const uint8_t* const* hcol = reinterpret_cast<const uint8_t* const*>(out);
        uint64_t coff[49], need = 0;
        for (int c = 0; c < 49; c++) {
            coff[c] = need;
            if (hcol[c]) need += (col_bytes(c, cap) + 255) & ~(uint64_t)255;
        }
        if (need > hp.dcol_cap) {
            (void)hipFree(hp.dcol);
            hp.dcol = nullptr;
            hp.dcol_cap = 0;
            if ((e = hipMalloc(reinterpret_cast<void**>(&hp.dcol), need)) != hipSuccess)
                return hip_fail(ctx, e, "hipMalloc (capture columns)");
            hp.dcol_cap = need;
        }
        uint8_t** dc = reinterpret_cast<uint8_t**>(&ig.dcols);
        const uint8_t* const* hc = reinterpret_cast<const uint8_t* const*>(hout);  // device-mapped host columns
        ig.xa.ncol = 0;
        ig.xa.cap = cap;
        ig.xa.lo_h = ig.xa.hi_h = 0;
        for (int c = 0; c < 49; c++) {
            dc[c] = hcol[c] ? hp.dcol + coff[c] : nullptr;
            if (!hcol[c]) continue;
            const bool slot = c == kColHdrType || c == kColHdrOff;
            for (uint32_t r = 0; r < (slot ? (uint32_t)PKT_MAX_HDRS : 1u); r++)
                ig.xa.col[ig.xa.ncol++] = ExportCol{reinterpret_cast<uint64_t>(dc[c]) + (uint64_t)r * cap * kColSize[c],
                                                    reinterpret_cast<uint64_t>(hc[c]) + (uint64_t)r * cap * kColSize[c],
                                                    kColSize[c], slot ? r : kExportNoRow};
        }
    }
    return pktgpu_pcap_reserve(ctx, len_cap, hp.s[0]);  // the whole capture's scratch: no growth between steps
}

// Copy the next n bytes of the capture in (hp.s[1], asynchronous: `src` must stay valid until the copy has
// landed, ingest_copied).
static int ingest_copy(Ingest& ig, const uint8_t* src, uint64_t n) {
    if (ig.rc != PKT_SUCCESS) return ig.rc;
    HostPipe& hp = ig.ctx->hp;
    const uint32_t c = (uint32_t)(ig.copies % HostPipe::kCopyRing);
    hipError_t e = hipMemcpyAsync(hp.file + ig.hi, src, n, hipMemcpyHostToDevice, hp.s[1]);
    if (e == hipSuccess) e = hipEventRecord(hp.ev_copy[c], hp.s[1]);
    if (e != hipSuccess) return ingest_fail(ig, hip_fail(ig.ctx, e, "hipMemcpyAsync H2D (capture bytes)"));
    ig.hi += n;
    ig.copy_end[c] = ig.hi;
    ig.copies++;
    return PKT_SUCCESS;
}

// The event of the queued copy that ends the first `upto` bytes (one of the last kCopyRing copies).
static hipEvent_t ingest_copied(const Ingest& ig, uint64_t upto) {
    for (uint64_t c = ig.copies; c > 0 && c + HostPipe::kCopyRing > ig.copies; c--)
        if (ig.copy_end[(c - 1) % HostPipe::kCopyRing] == upto) return ig.ctx->hp.ev_copy[(c - 1) % HostPipe::kCopyRing];
    return nullptr;
}

// One step over the first `upto` bytes (0: every byte copied so far; `upto` ends a queued copy among the
// last kCopyRing) (last: the capture is complete — a record running past its end is the capture's error;
// otherwise such a record waits for the next step).  Needs upto >= 24.
static int ingest_step(Ingest& ig, bool last, uint64_t upto = 0) {
    if (ig.rc != PKT_SUCCESS) return ig.rc;
    pkt_ctx_t* ctx = ig.ctx;
    HostPipe& hp = ctx->hp;
    hipStream_t cs = hp.s[1], ps = hp.s[0], es = hp.s[2];
    (void)cs;
    constexpr uint32_t R = HostPipe::kRing;
    const uint64_t k = ig.steps;
    const uint32_t j = (uint32_t)(k % R), jp = (uint32_t)((k + R - 1) % R);
    const uint64_t hi = upto ? upto : ig.hi;
    const uint64_t region = pktgpu_pcap_region_bytes(), K = (hi + region - 1) / region;
    // the segment: from the region holding the previous step's end (its carry decides the exact entry),
    // at least the last region (a final step with no new bytes still decides the carried record)
    const uint32_t r0 = k ? (uint32_t)std::min<uint64_t>(ig.indexed / region, K - 1) : 0u;
    const hipEvent_t landed = ingest_copied(ig, hi);
    if (!landed || hi < ig.indexed) return ingest_fail(ig, fail(ctx, PKT_ERR_INVALID_ARG, "capture step past its copies"));
    hipError_t e = hipStreamWaitEvent(ps, landed, 0);
    // the ring slot this step writes was last read by step k - R + 1's export
    if (e == hipSuccess && ig.exporting && k + 1 >= R) e = hipStreamWaitEvent(ps, hp.ev_xdone[(k + 1) % R], 0);
    if (e != hipSuccess) return ingest_fail(ig, hip_fail(ctx, e, "hipStreamWaitEvent (capture step)"));
    uint64_t* carry = hp.pcarry + (uint64_t)j * kPcapCarryWords;
    const uint64_t* cin = k ? hp.pcarry + (uint64_t)jp * kPcapCarryWords : nullptr;
    const uint64_t* cnt = nullptr;
    int rc = pktgpu_pcap_launch(ctx, hp.file, hi, hp.ioffs, hp.ilens, ig.cap, ps, &cnt, !last, carry + 1, r0, cin, carry);
    if (rc != PKT_SUCCESS) return ingest_fail(ig, rc);
    pkt_batch_t db;
    db.slab = hp.file;
    db.slab_len = hi;  // the prefix: every record parsed here lies inside it
    db.offsets = hp.ioffs;
    db.lens = hp.ilens;
    db.stride = 0;
    db.reserved = 0;
    db.n = ig.cap;
    uint32_t* nh = ig.exporting ? hp.pnh + (uint64_t)j * kMaxSpread : nullptr;
    if (nh && (e = hipMemsetAsync(nh, 0, kMaxSpread * 4, ps)) != hipSuccess)
        return ingest_fail(ig, hip_fail(ctx, e, "hipMemsetAsync"));
    // the records this step added: [the previous step's count, this step's count)
    rc = parse_impl(ctx, &db, ig.entry, &ig.dcols, ps, 0, ctx->staging, nh, ig.cap, nullptr, cnt, cin ? cin + 1 : nullptr,
                    (hi - ig.indexed) / 16 + 1);
    if (rc != PKT_SUCCESS) return ingest_fail(ig, rc);
    if (ig.exporting) {
        if ((e = hipEventRecord(hp.ev_parsed, ps)) != hipSuccess || (e = hipStreamWaitEvent(es, hp.ev_parsed, 0)) != hipSuccess)
            return ingest_fail(ig, hip_fail(ctx, e, "hipEventRecord (step parsed)"));
        ig.xa.lo_dev = cin ? cin + 1 : nullptr;
        ig.xa.hi_dev = cnt;
        ig.xa.nhw = nh;
        if ((e = pktgpu_export_launch(ig.xa, es)) != hipSuccess || (e = hipEventRecord(hp.ev_xdone[j], es)) != hipSuccess)
            return ingest_fail(ig, hip_fail(ctx, e, "export_kernel"));
    }
    ig.indexed = hi;
    ig.steps++;
    return PKT_SUCCESS;
}

// Wait for every queued step: the capture's outcome (pcap_finish: count, magic, a record past the end),
// the index of the first min(count, cap) records copied to offsets / lens (host, may be NULL).
static int ingest_wait(Ingest& ig, uint64_t* n_out, uint64_t* offsets, uint32_t* lens) {
    if (ig.rc != PKT_SUCCESS) return ig.rc;
    pkt_ctx_t* ctx = ig.ctx;
    HostPipe& hp = ctx->hp;
    hipError_t e = hipStreamSynchronize(hp.s[0]);
    if (e != hipSuccess) return ingest_fail(ig, hip_fail(ctx, e, "hipStreamSynchronize"));
    int rc = pktgpu_pcap_finish(ctx, n_out);
    if (rc != PKT_SUCCESS) return ingest_fail(ig, rc);
    const uint64_t m = std::min(*n_out, ig.cap);
    if (m && offsets && (e = hipMemcpyAsync(offsets, hp.ioffs, m * 8, hipMemcpyDeviceToHost, hp.s[1])) != hipSuccess)
        return ingest_fail(ig, hip_fail(ctx, e, "hipMemcpyAsync D2H (offsets)"));
    if (m && lens && (e = hipMemcpyAsync(lens, hp.ilens, m * 4, hipMemcpyDeviceToHost, hp.s[1])) != hipSuccess)
        return ingest_fail(ig, hip_fail(ctx, e, "hipMemcpyAsync D2H (lens)"));
    if ((e = hipStreamSynchronize(hp.s[1])) != hipSuccess || (e = hipStreamSynchronize(hp.s[2])) != hipSuccess)
        return ingest_fail(ig, hip_fail(ctx, e, "hipStreamSynchronize"));
    return PKT_SUCCESS;
}

// pkt_parse_pcap_host with pinned columns: the file copied in pieces of `piece` bytes, one step per piece
// (blocking = false, pkt_parse_pcap_host_async: everything queued, the capture left pending on the ctx).
static int pcap_host_pieces(pkt_ctx_t* ctx, const uint8_t* buf, uint64_t len, int entry, const pkt_out_t* out,
                            const pkt_out_t& hout, uint64_t* offsets, uint32_t* lens, uint64_t cap,
                            uint64_t* n_out, uint64_t piece, bool blocking) {
    Ingest ig;
    int rc = ingest_begin(ig, ctx, len, cap, entry, out, &hout);
    if (rc != PKT_SUCCESS) return rc;
    // at most kMaxHostSteps pieces per capture: each step costs ~50 us of host API time (13 calls), so
    // tiny pieces over a large file would make the host the bottleneck (1 MiB pieces: 12.2 ms per 195 MB
    // against 4.8 ms at 16 MiB, r06)
    constexpr uint64_t kMaxHostSteps = 1024;
    piece = std::max<uint64_t>(piece, (len + kMaxHostSteps - 1) / kMaxHostSteps);
    // the copies run kAhead pieces ahead of the steps that wait for them (queued before the step's
    // kernels on the host: a copy queued behind an export waited for that export's parse, r06e trace)
    constexpr uint64_t kAhead = 3;
    static_assert(kAhead < HostPipe::kCopyRing, "a step's copy is among the last kCopyRing");
    const uint64_t np = (len + piece - 1) / piece;
    for (uint64_t p = 0; p < np && p < kAhead; p++)
        if ((rc = ingest_copy(ig, buf + p * piece, std::min(len, (p + 1) * piece) - p * piece)) != PKT_SUCCESS) return rc;
    for (uint64_t p = 0; p < np; p++) {
        const uint64_t q = p + kAhead;
        if (q < np && (rc = ingest_copy(ig, buf + q * piece, std::min(len, (q + 1) * piece) - q * piece)) != PKT_SUCCESS)
            return rc;
        if ((rc = ingest_step(ig, p + 1 == np, std::min(len, (p + 1) * piece))) != PKT_SUCCESS) return rc;
    }
    if (!blocking) {
        ctx->pc.pending = true;
        ctx->pc.pending_stream = ctx->hp.s[0];
        return PKT_SUCCESS;
    }
    return ingest_wait(ig, n_out, offsets, lens);
}

extern "C" {

int pkt_parse_pcap_host(pkt_ctx_t* ctx, const uint8_t* buf, uint64_t len, int entry, const pkt_out_t* out,
                        uint64_t* offsets, uint32_t* lens, uint64_t cap, uint64_t* n_out) {
    if (!ctx || !buf || !out || !n_out) return fail(ctx, PKT_ERR_INVALID_ARG, "null argument");
    if (entry < 0 || entry >= PKT_ENTRY_COUNT) return fail(ctx, PKT_ERR_INVALID_ARG, "bad entry");
    *n_out = 0;
    hipError_t e;
    int rc = pcap_host_buffers(ctx, len, cap);
    if (rc != PKT_SUCCESS) return rc;
    HostPipe& hp = ctx->hp;
    hipStream_t s = hp.s[0];
    {  // pinned columns: copy, index, parse and export piece by piece (one piece for a short file)
        pkt_out_t dout;
        const uint64_t piece = ctx->host_piece ? ctx->host_piece : kHostPiece;
        if (len >= 24 && cap && cap <= kLaunchChunk && out_mapped(out, dout))
            return pcap_host_pieces(ctx, buf, len, entry, out, dout, offsets, lens, cap, n_out, piece, true);
    }
    // every error return after the first queued copy waits for the ctx's streams first: a copy from
    // `buf` or into `offsets` / `lens` must not outlive the call
    auto bail = [&](int code) {
        (void)hipStreamSynchronize(hp.s[0]);
        (void)hipStreamSynchronize(hp.s[1]);
        return code;
    };
    // in: the whole file, one copy (the record chain is sequential: the index needs all of it)
    if ((e = hipMemcpyAsync(hp.file, buf, len, hipMemcpyHostToDevice, s)) != hipSuccess)
        return bail(hip_fail(ctx, e, "hipMemcpyAsync H2D (pcap file)"));
    uint64_t n = 0;
    rc = pkt_pcap_index_device(ctx, hp.file, len, hp.ioffs, hp.ilens, cap, &n, s);
    if (rc != PKT_SUCCESS) return bail(rc);
    *n_out = n;
    const uint64_t m = std::min(n, cap);
    if (m == 0) return PKT_SUCCESS;
    if (offsets && (e = hipMemcpyAsync(offsets, hp.ioffs, m * 8, hipMemcpyDeviceToHost, hp.s[1])) != hipSuccess)
        return bail(hip_fail(ctx, e, "hipMemcpyAsync D2H (offsets)"));
    if (lens && (e = hipMemcpyAsync(lens, hp.ilens, m * 4, hipMemcpyDeviceToHost, hp.s[1])) != hipSuccess)
        return bail(hip_fail(ctx, e, "hipMemcpyAsync D2H (lens)"));
    pkt_batch_t db;
    db.slab = hp.file;
    db.slab_len = len;
    db.offsets = hp.ioffs;
    db.lens = hp.ilens;
    db.stride = 0;
    db.reserved = 0;
    db.n = m;
    // out: pinned (mapped) columns are written by the parse kernel over the link directly; else the
    // staged pipeline (device output slots, copies per chunk)
    pkt_out_t dout;
    if (out_mapped(out, dout)) {
        rc = parse_impl(ctx, &db, entry, &dout, s, 0, ctx->staging, nullptr, cap);
        if (rc != PKT_SUCCESS) return bail(rc);
        for (int k = 0; k < 2; k++)
            if ((e = hipStreamSynchronize(hp.s[k])) != hipSuccess) return hip_fail(ctx, e, "hipStreamSynchronize");
        return PKT_SUCCESS;
    }
    rc = staged_parse(ctx, &db, entry, out, 0, true, cap);
    if (rc != PKT_SUCCESS) return bail(rc);
    if ((e = hipStreamSynchronize(hp.s[1])) != hipSuccess) return hip_fail(ctx, e, "hipStreamSynchronize");
    return PKT_SUCCESS;
}

}  // extern "C"

// ---- a capture that arrives in pieces (pkt_pcap_stream_*, include/pktgpu.h) ----
struct pkt_pcap_stream {
    pkt_ctx_t* ctx = nullptr;  // its own: the open capture holds the ctx's index scratch and host pipeline
    Ingest ig;
    uint64_t max_bytes = 0;
    uint64_t step = 0;  // bytes of new data that start a step at a push
    bool done = false;
    std::string err;
    // Pushes below kStageMax bytes are gathered in a pinned staging ring (host memcpy) and copied in
    // by the slot, so push returns without waiting for a copy (a wait per push is ~20 us: 64 KiB
    // pushes ran at 3.2 GB/s, r06z4; staged 16.6, r06z6); larger pushes are copied from the caller's
    // buffer directly and waited for (195 MB in pushes of 256 KiB: 17.6 ms direct, 8.3 staged; 512 KiB
    // direct 11.2; 1 MiB direct 7.7).  A slot is refilled once its copy has landed (stage_ev).
    static constexpr uint32_t kStageSlots = 4;
    static constexpr uint64_t kStageSlot = 1ull << 20;
    static constexpr uint64_t kStageMax = 1ull << 20;
    uint8_t* stage = nullptr;  // pinned, kStageSlots x kStageSlot
    hipEvent_t stage_ev[kStageSlots] = {};
    bool stage_used[kStageSlots] = {};
    uint32_t cur = 0;   // the slot being filled
    uint64_t fill = 0;  // its bytes
};

namespace {
constexpr uint64_t kStreamStep = 4ull << 20;
int st_fail(pkt_pcap_stream* st, int code, const std::string& msg) {
    if (st) st->err = msg;
    return code;
}
int st_ctx_fail(pkt_pcap_stream* st, int code) { return st_fail(st, code, st->ctx ? st->ctx->err : "ctx"); }
// The staged bytes of the current slot to the device (in order with every earlier copy: one copy stream).
int st_flush(pkt_pcap_stream* st) {
    if (!st->fill) return PKT_SUCCESS;
    const uint32_t c = st->cur;
    int rc = ingest_copy(st->ig, st->stage + (uint64_t)c * pkt_pcap_stream::kStageSlot, st->fill);
    if (rc != PKT_SUCCESS) return rc;
    const hipError_t e = hipEventRecord(st->stage_ev[c], st->ctx->hp.s[1]);
    if (e != hipSuccess) return ingest_fail(st->ig, hip_fail(st->ctx, e, "hipEventRecord (staging)"));
    st->stage_used[c] = true;
    st->cur = (c + 1) % pkt_pcap_stream::kStageSlots;
    st->fill = 0;
    return PKT_SUCCESS;
}
}  // namespace

extern "C" {

int pkt_pcap_stream_open(int device, uint64_t max_bytes, uint64_t cap, int entry, const pkt_out_t* out,
                         uint64_t step_bytes, pkt_pcap_stream_t** out_st) {
    if (!out_st || !out || !cap || max_bytes < 24) return PKT_ERR_INVALID_ARG;
    *out_st = nullptr;
    if (entry < 0 || entry >= PKT_ENTRY_COUNT || cap > kLaunchChunk) return PKT_ERR_INVALID_ARG;
    pkt_out_t dout;
    const bool pinned = out_mapped(out, dout);
    if (!pinned) {  // then every requested column is device memory (none mapped host memory)
        const uint8_t* const* oc = reinterpret_cast<const uint8_t* const*>(out);
        for (int c = 0; c < 49; c++) {
            const uint8_t* unused = nullptr;
            if (oc[c] && host_mapped(oc[c], unused)) return PKT_ERR_INVALID_ARG;  // mixed host / device columns
        }
    }
    pkt_pcap_stream* st = new pkt_pcap_stream();
    int rc = pkt_ctx_create(device, &st->ctx);
    if (rc == PKT_SUCCESS) rc = ingest_begin(st->ig, st->ctx, max_bytes, cap, entry, out, pinned ? &dout : nullptr);
    if (rc != PKT_SUCCESS) {
        pkt_pcap_stream_close(st);
        return rc;
    }
    st->max_bytes = max_bytes;
    st->step = step_bytes ? step_bytes : kStreamStep;
    hipError_t e = hipHostMalloc(reinterpret_cast<void**>(&st->stage), pkt_pcap_stream::kStageSlots * pkt_pcap_stream::kStageSlot, 0);
    for (uint32_t k = 0; k < pkt_pcap_stream::kStageSlots && e == hipSuccess; k++)
        e = hipEventCreateWithFlags(&st->stage_ev[k], hipEventDisableTiming);
    if (e != hipSuccess) {
        rc = hip_fail(st->ctx, e, "pinned staging ring");
        pkt_pcap_stream_close(st);
        return rc;
    }
    *out_st = st;
    return PKT_SUCCESS;
}

int pkt_pcap_stream_push(pkt_pcap_stream_t* st, const uint8_t* bytes, uint64_t n) {
    if (!st || (n && !bytes)) return st_fail(st, PKT_ERR_INVALID_ARG, "null argument");
    if (st->done) return st_fail(st, PKT_ERR_INVALID_ARG, "the capture is finished");
    if (n > st->max_bytes - st->ig.hi - st->fill) return st_fail(st, PKT_ERR_INVALID_ARG, "push past the capture's max_bytes");
    if (!n) return PKT_SUCCESS;
    if (st->ig.rc != PKT_SUCCESS) return st_ctx_fail(st, st->ig.rc);
    int rc = PKT_SUCCESS;
    // the caller may reuse its buffer once this returns: its bytes are staged, or their copy has landed
    if (n < pkt_pcap_stream::kStageMax) {
        while (n && rc == PKT_SUCCESS) {
            const uint32_t c = st->cur;
            if (!st->fill && st->stage_used[c]) {  // the slot's previous copy must have landed
                const hipError_t e = hipEventSynchronize(st->stage_ev[c]);
                if (e != hipSuccess) rc = ingest_fail(st->ig, hip_fail(st->ctx, e, "hipEventSynchronize (staging)"));
                st->stage_used[c] = false;
            }
            const uint64_t take = std::min(n, pkt_pcap_stream::kStageSlot - st->fill);
            if (rc == PKT_SUCCESS) std::memcpy(st->stage + (uint64_t)c * pkt_pcap_stream::kStageSlot + st->fill, bytes, take);
            st->fill += take;
            bytes += take;
            n -= take;
            if (rc == PKT_SUCCESS && st->fill == pkt_pcap_stream::kStageSlot) rc = st_flush(st);
        }
        // a step is due: its bytes go now (steps run over copied bytes)
        const uint64_t have = st->ig.hi + st->fill;
        if (rc == PKT_SUCCESS && have >= 24 && have - st->ig.indexed >= st->step) rc = st_flush(st);
    } else {
        rc = st_flush(st);  // the staged bytes first: the file's order
        if (rc == PKT_SUCCESS) rc = ingest_copy(st->ig, bytes, n);
        const hipEvent_t landed = rc == PKT_SUCCESS ? ingest_copied(st->ig, st->ig.hi) : nullptr;
        const hipError_t e = landed ? hipEventSynchronize(landed) : hipSuccess;
        if (e != hipSuccess) rc = ingest_fail(st->ig, hip_fail(st->ctx, e, "hipEventSynchronize (push)"));
    }
    if (rc == PKT_SUCCESS && st->ig.hi >= 24 && st->ig.hi - st->ig.indexed >= st->step) rc = ingest_step(st->ig, false);
    return rc == PKT_SUCCESS ? rc : st_ctx_fail(st, rc);
}

int pkt_pcap_stream_poll(pkt_pcap_stream_t* st, uint64_t* n_records, uint64_t* offsets, uint32_t* lens) {
    if (!st || !n_records) return st_fail(st, PKT_ERR_INVALID_ARG, "null argument");
    *n_records = 0;
    int rc = st->done ? PKT_SUCCESS : st_flush(st);
    if (rc != PKT_SUCCESS) return st_ctx_fail(st, rc);
    if (st->ig.hi < 24) return st->ig.rc;  // not even the global header yet
    if (!st->done && st->ig.hi > st->ig.indexed) rc = ingest_step(st->ig, false);
    if (rc == PKT_SUCCESS) rc = ingest_wait(st->ig, n_records, offsets, lens);
    return rc == PKT_SUCCESS ? rc : st_ctx_fail(st, rc);
}

int pkt_pcap_stream_finish(pkt_pcap_stream_t* st, uint64_t* n_records, uint64_t* offsets, uint32_t* lens) {
    if (!st || !n_records) return st_fail(st, PKT_ERR_INVALID_ARG, "null argument");
    *n_records = 0;
    int rc = st->done ? PKT_SUCCESS : st_flush(st);
    if (rc != PKT_SUCCESS) return st_ctx_fail(st, rc);
    if (st->ig.hi < 24) return st_fail(st, PKT_ERR_INVALID_ARG, "pcap shorter than its global header");
    if (!st->done) rc = ingest_step(st->ig, true);  // the tail as pkt_pcap_index takes it (errors included)
    st->done = true;
    if (rc == PKT_SUCCESS) rc = ingest_wait(st->ig, n_records, offsets, lens);
    return rc == PKT_SUCCESS ? rc : st_ctx_fail(st, rc);
}

pkt_ctx_t* pkt_pcap_stream_ctx(pkt_pcap_stream_t* st) { return st ? st->ctx : nullptr; }

const char* pkt_pcap_stream_last_error(const pkt_pcap_stream_t* st) { return st ? st->err.c_str() : "null stream"; }

int pkt_pcap_stream_close(pkt_pcap_stream_t* st) {
    if (!st) return PKT_SUCCESS;
    if (st->ctx) pkt_ctx_destroy(st->ctx);  // waits for its streams (the staging ring's copies too)
    for (hipEvent_t ev : st->stage_ev)
        if (ev) (void)hipEventDestroy(ev);
    if (st->stage) (void)hipHostFree(st->stage);
    delete st;
    return PKT_SUCCESS;
}

}  // extern "C"
