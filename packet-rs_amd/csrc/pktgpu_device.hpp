// pktgpu_device.hpp — device code of the batched parser (gfx950 / CDNA4).
//
// One lane per packet.  A wave owns a tile of 64 packets and an LDS "window" region laid out
// chunk-major: chunk c (16 bytes) of lane l lives at win + c*1024 + l*16.  That layout is what
// one `global_load_lds_dwordx4` wave-instruction writes (wave-uniform base + lane*16), so each
// wave stages its 64 packets' first W bytes with W/16 (+1 when packet starts are not 16-byte
// aligned) LDS-DMA loads, each lane gathering its own packet's chunk c.  A lane then walks its
// packet's header chain out of LDS with dword reads at per-lane byte offsets (v_alignbyte for
// the unaligned part, v_perm for the big-endian swap); a chain that runs past the window falls
// back to byte loads from global memory.  Waves never share LDS, so there is no barrier.
//
// The walk is the forward, iterative form of the reference's recursion
// (src/parser/fast.rs:5-227): each step checks the bounds the reference's slice indexing would
// panic on (-> PKT_TRUNCATED), then the depth bound, then reads the dispatch field, records
// (type, offset) and moves on.  GRE options are recorded GRE, SeqNum, Key, ChksumOffset
// (fast.rs:154-163, Q2).  Field values use the make_header! MSB-first convention
// (headers.rs:195-201, 252-263) with shifts/masks fixed at compile time per header.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/pktgpu.h"

namespace pktgpu {

constexpr int kWave = 64;
constexpr int kWavesPerBlock = 4;
constexpr int kBlock = kWave * kWavesPerBlock;
constexpr int kChunkRow = kWave * 16;  // bytes of one chunk row (one LDS-DMA instruction)

// Walk states = the parse_* functions of fast.rs (+ accept / done markers).
enum State : uint32_t {
    S_PARSE = 0, S_DOT3, S_LLC, S_SNAP, S_ETHER, S_VLAN, S_MPLS, S_MPLS_BOS, S_IPV4, S_IPV6,
    S_GRE, S_ERSPAN2, S_ERSPAN3, S_ARP, S_ICMP, S_TCP, S_UDP, S_VXLAN, S_ACCEPT, S_DONE
};

// pkt_entry_t -> first state (entries 1..17 map 1:1 onto S_DOT3..S_VXLAN)
__device__ __forceinline__ uint32_t entry_state(int entry) { return (uint32_t)entry; }

struct KParams {
    const uint8_t* slab;
    uint64_t slab_len;
    const uint64_t* offsets;
    const uint32_t* lens;
    uint32_t stride;
    int entry;
    uint64_t n;
    pkt_out_t out;
};

// EtherType dispatch (types.rs:51-75 as matched in fast.rs:38-45 / 52-59)
__device__ __forceinline__ uint32_t etype_next(uint32_t et) {
    uint32_t s = S_ACCEPT;
    s = (et == 0x8100u) ? S_VLAN : s;
    s = (et == 0x0806u) ? S_ARP : s;
    s = (et == 0x0800u) ? S_IPV4 : s;
    s = (et == 0x86DDu) ? S_IPV6 : s;
    s = (et == 0x8847u) ? S_MPLS : s;
    return s;
}
// IpProtocol dispatch after IPv4 (fast.rs:87-95) and IPv6 (fast.rs:102-110; Q6)
__device__ __forceinline__ uint32_t ipproto_next(uint32_t p, bool v6) {
    uint32_t s = S_ACCEPT;
    s = (p == (v6 ? 58u : 1u)) ? S_ICMP : s;
    s = (p == 4u) ? S_IPV4 : s;
    s = (p == 6u) ? S_TCP : s;
    s = (p == 17u) ? S_UDP : s;
    s = (p == 41u) ? S_IPV6 : s;
    s = (p == 47u) ? S_GRE : s;
    return s;
}
// GRE proto dispatch (fast.rs:147-153)
__device__ __forceinline__ uint32_t gre_next(uint32_t p) {
    uint32_t s = S_ACCEPT;
    s = (p == 0x0800u) ? S_IPV4 : s;
    s = (p == 0x86DDu) ? S_IPV6 : s;
    s = (p == 0x88BEu) ? S_ERSPAN2 : s;
    s = (p == 0x22EBu) ? S_ERSPAN3 : s;
    return s;
}

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

// A lane's view of its packet: LDS window + global fallback.
struct PacketView {
    const uint8_t* lw;        // LDS window base of this wave (chunk-major), already + lane*16
    const uint8_t* gbase;     // packet start in global memory
    uint32_t shift;           // packet start - aligned window start (0..15)
    uint32_t win_end;         // packet bytes [0, win_end) are in the window
    uint32_t len;             // packet length

    // aligned dword k of the window
    __device__ __forceinline__ uint32_t wdw(uint32_t k) const {
        return *reinterpret_cast<const uint32_t*>(lw + (k >> 2) * kChunkRow + (k & 3) * 4);
    }
    // n (1..4) bytes at packet offset b, little-endian in the low bytes (garbage above n).
    // Caller guarantees b + n <= len.
    __device__ __forceinline__ uint32_t le(uint32_t b, uint32_t n) const {
        if (b + n <= win_end) {
            uint32_t wb = b + shift;
            uint32_t k = wb >> 2, sh = wb & 3;
            uint32_t lo = wdw(k);
            uint32_t hi = (sh + n > 4) ? wdw(k + 1) : 0u;
            return __builtin_amdgcn_alignbyte(hi, lo, sh);
        }
        uint32_t v = 0;
        for (uint32_t i = 0; i < n; i++) v |= (uint32_t)gbase[b + i] << (8 * i);
        return v;
    }
    __device__ __forceinline__ uint32_t u8(uint32_t b) const { return le(b, 1) & 0xFFu; }
    __device__ __forceinline__ uint32_t be16(uint32_t b) const { return bswap32(le(b, 2)) >> 16; }

    // NW big-endian dwords of header bytes [b, b + nbytes) (bytes beyond nbytes read as
    // whatever follows in the window, or 0 on the global path).  Caller: b + nbytes <= len.
    template <int NW>
    __device__ __forceinline__ void hdr(uint32_t b, uint32_t nbytes, uint32_t (&d)[NW]) const {
        if (b + 4 * NW <= win_end) {
            uint32_t wb = b + shift;
            uint32_t k = wb >> 2, sh = wb & 3;
            uint32_t a[NW + 1];
#pragma unroll
            for (int i = 0; i <= NW; i++) a[i] = wdw(k + i);
#pragma unroll
            for (int i = 0; i < NW; i++) d[i] = bswap32(__builtin_amdgcn_alignbyte(a[i + 1], a[i], sh));
        } else {
#pragma unroll
            for (int i = 0; i < NW; i++) {
                uint32_t v = 0;
                for (uint32_t j = 0; j < 4; j++) {
                    uint32_t bb = b + 4 * i + j;
                    v = (v << 8) | ((4 * i + j < nbytes) ? (uint32_t)gbase[bb] : 0u);
                }
                d[i] = v;
            }
        }
    }
};

struct WalkResult {
    uint32_t status, n, payload_off, mask;
    int32_t f_eth, f_vlan, f_ipv4, f_ipv6, f_tcp, f_udp;  // first offsets, -1 = absent
};

// The walk.  `push` records (type, offset) in list slot `n`.
template <class Push>
__device__ __forceinline__ void walk(const PacketView& pv, uint32_t state, bool active, Push&& push,
                                     WalkResult& r) {
    r.status = PKT_OK;
    r.n = 0;
    r.payload_off = 0;
    r.mask = 0;
    r.f_eth = r.f_vlan = r.f_ipv4 = r.f_ipv6 = r.f_tcp = r.f_udp = -1;
    uint32_t o = 0;
    const uint32_t len = pv.len;
    bool live = active;

    auto rec = [&](uint32_t t, uint32_t off) {
        push(r.n, t, off);
        r.n++;
        r.mask |= 1u << t;
        if (t == PKT_HDR_ETHER && r.f_eth < 0) r.f_eth = (int32_t)off;
        if (t == PKT_HDR_VLAN && r.f_vlan < 0) r.f_vlan = (int32_t)off;
        if (t == PKT_HDR_IPV4 && r.f_ipv4 < 0) r.f_ipv4 = (int32_t)off;
        if (t == PKT_HDR_IPV6 && r.f_ipv6 < 0) r.f_ipv6 = (int32_t)off;
        if (t == PKT_HDR_TCP && r.f_tcp < 0) r.f_tcp = (int32_t)off;
        if (t == PKT_HDR_UDP && r.f_udp < 0) r.f_udp = (int32_t)off;
    };
    auto fail = [&](uint32_t st) {
        r.status = st;
        live = false;
    };

    // Each iteration consumes >= 1 header (or resolves S_PARSE / accepts), so this bound is
    // never the one that stops a walk; it only guarantees termination.
    for (int it = 0; it < PKT_MAX_HDRS + 3; it++) {
        if (!__any(live)) break;
        if (!live) continue;
        if (state == S_ACCEPT) {  // fast.rs:223-227
            r.payload_off = o;
            live = false;
            continue;
        }
        if (state == S_PARSE) {  // fast.rs:5-12: arr[12], arr[13]
            if (o + 14 > len) { fail(PKT_TRUNCATED); continue; }
            state = (pv.be16(o + 12) < 1500u) ? S_DOT3 : S_ETHER;
            continue;
        }
        // header size and type of this state
        uint32_t sz, t;
        switch (state) {
            case S_DOT3: sz = 14; t = PKT_HDR_DOT3; break;
            case S_LLC: sz = 3; t = PKT_HDR_LLC; break;
            case S_SNAP: sz = 5; t = PKT_HDR_SNAP; break;
            case S_ETHER: sz = 14; t = PKT_HDR_ETHER; break;
            case S_VLAN: sz = 4; t = PKT_HDR_VLAN; break;
            case S_MPLS: sz = 4; t = PKT_HDR_MPLS; break;
            case S_MPLS_BOS: sz = 4; t = PKT_HDR_MPLS; break;
            case S_IPV4: sz = 20; t = PKT_HDR_IPV4; break;
            case S_IPV6: sz = 40; t = PKT_HDR_IPV6; break;
            case S_GRE: sz = 4; t = PKT_HDR_GRE; break;
            case S_ERSPAN2: sz = 8; t = PKT_HDR_ERSPAN2; break;
            case S_ERSPAN3: sz = 12; t = PKT_HDR_ERSPAN3; break;
            case S_ARP: sz = 28; t = PKT_HDR_ARP; break;
            case S_ICMP: sz = 4; t = PKT_HDR_ICMP; break;
            case S_TCP: sz = 20; t = PKT_HDR_TCP; break;
            case S_UDP: sz = 8; t = PKT_HDR_UDP; break;
            default: sz = 8; t = PKT_HDR_VXLAN; break;  // S_VXLAN
        }
        if (o + sz > len) { fail(PKT_TRUNCATED); continue; }   // `&arr[0..X::size()]`
        if (r.n >= PKT_MAX_HDRS) { fail(PKT_DEPTH_LIMIT); continue; }
        uint32_t next = S_ETHER;
        bool advanced = false;  // multi-header steps (GRE, ERSPAN3) record and advance themselves
        switch (state) {
            case S_DOT3: next = S_LLC; break;
            case S_LLC:  // fast.rs:21: aa aa 03 -> SNAP
                next = ((pv.le(o, 3) & 0xFFFFFFu) == 0x03AAAAu) ? S_SNAP : S_ACCEPT;
                break;
            case S_ETHER: next = etype_next(pv.be16(o + 12)); break;
            case S_VLAN: next = etype_next(pv.be16(o + 2)); break;
            case S_MPLS: next = (pv.u8(o + 2) & 1u) ? S_MPLS_BOS : S_MPLS; break;  // bos = bit 23
            case S_MPLS_BOS: {  // fast.rs:74-83: arr[MPLS::size()] must exist
                if (o + 5 > len) { fail(PKT_TRUNCATED); advanced = true; break; }
                uint32_t nib = pv.u8(o + 4) >> 4;
                next = (nib == 4u) ? S_IPV4 : ((nib == 6u) ? S_IPV6 : S_ETHER);
                break;
            }
            case S_IPV4: next = ipproto_next(pv.u8(o + 9), false); break;
            case S_IPV6: next = ipproto_next(pv.u8(o + 6), true); break;
            case S_GRE: {  // fast.rs:114-165; options sliced C, K, S; listed S, K, C (Q2)
                advanced = true;
                uint32_t w = bswap32(pv.le(o, 4));
                uint32_t c = w >> 31, k = (w >> 29) & 1u, s = (w >> 28) & 1u;
                rec(t, o);
                uint32_t q = o + 4, oc = 0, okey = 0, oseq = 0;
                if (c) {
                    if (q + 4 > len) { fail(PKT_TRUNCATED); break; }
                    if (r.n >= PKT_MAX_HDRS) { fail(PKT_DEPTH_LIMIT); break; }
                    oc = q; q += 4;
                }
                if (k) {
                    if (q + 4 > len) { fail(PKT_TRUNCATED); break; }
                    if (r.n + c >= PKT_MAX_HDRS) { fail(PKT_DEPTH_LIMIT); break; }
                    okey = q; q += 4;
                }
                if (s) {
                    if (q + 4 > len) { fail(PKT_TRUNCATED); break; }
                    if (r.n + c + k >= PKT_MAX_HDRS) { fail(PKT_DEPTH_LIMIT); break; }
                    oseq = q; q += 4;
                }
                if (s) rec(PKT_HDR_GRE_SEQUENCE_NUM, oseq);
                if (k) rec(PKT_HDR_GRE_KEY, okey);
                if (c) rec(PKT_HDR_GRE_CHKSUM_OFFSET, oc);
                o = q;
                state = gre_next(w & 0xFFFFu);
                break;
            }
            case S_ERSPAN2: next = S_ETHER; break;
            case S_ERSPAN3: {  // fast.rs:172-192: o bit = bit 95 -> ERSPANPLATFORM
                advanced = true;
                uint32_t ob = pv.u8(o + 11) & 1u;
                rec(t, o);
                uint32_t q = o + 12;
                if (ob) {
                    if (q + 8 > len) { fail(PKT_TRUNCATED); break; }
                    if (r.n >= PKT_MAX_HDRS) { fail(PKT_DEPTH_LIMIT); break; }
                    rec(PKT_HDR_ERSPAN_PLATFORM, q);
                    q += 8;
                }
                o = q;
                state = S_ETHER;
                break;
            }
            case S_SNAP: case S_ARP: case S_ICMP: case S_TCP: next = S_ACCEPT; break;
            case S_UDP: next = (pv.be16(o + 2) == 4789u) ? S_VXLAN : S_ACCEPT; break;  // types.rs:7
            default: next = S_ETHER; break;  // S_VXLAN
        }
        if (advanced) continue;
        rec(t, o);
        o += sz;
        state = next;
    }
    if (live) r.status = PKT_DEPTH_LIMIT;  // unreachable bound (see loop comment)
}

}  // namespace pktgpu
