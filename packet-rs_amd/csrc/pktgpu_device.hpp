// pktgpu_device.hpp — device code of the batched parser (gfx950 / CDNA4).
//
// One lane per packet, 256-packet blocks.  The wave loads its packets' first NCH 16-byte chunks
// cooperatively into each lane's own LDS window (packet-major, odd dword stride: conflict-free
// per-lane dword reads).  Aligned Ether/0-2 Vlan/IPv4/UDP|TCP packets have their chain decided by a
// few compares (the fast path); every other lane walks its header chain out of LDS with dword reads
// at per-lane byte offsets (v_alignbyte for the unaligned part, a byte swap for big-endian); a
// chain that runs past the window falls back to dword loads from global memory.  No barrier
// beyond the wave's own: a lane reads only its own window.
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
#ifndef PKTGPU_WAVES_PER_BLOCK
#define PKTGPU_WAVES_PER_BLOCK 4
#endif
constexpr int kWavesPerBlock = PKTGPU_WAVES_PER_BLOCK;
constexpr int kBlock = kWave * kWavesPerBlock;

// Walk states = the parse_* functions of fast.rs (+ accept / done markers).
enum State : uint32_t {
    S_PARSE = 0, S_DOT3, S_LLC, S_SNAP, S_ETHER, S_VLAN, S_MPLS, S_MPLS_BOS, S_IPV4, S_IPV6,
    S_GRE, S_ERSPAN2, S_ERSPAN3, S_ARP, S_ICMP, S_TCP, S_UDP, S_VXLAN, S_ACCEPT, S_DONE
};

// pkt_entry_t -> first state (entries 1..17 map 1:1 onto S_DOT3..S_VXLAN)
__device__ __forceinline__ uint32_t entry_state(int entry) { return (uint32_t)entry; }

// One launch covers packets [i0, i0 + n) of a batch, n <= kLaunchChunk, so that every per-packet
// column byte offset (at most i * 16, the IPv6 addresses) fits 32 bits; offsets/lens/per-packet
// columns are pre-offset by i0 on the host, the slot-major hdr_type/hdr_off columns are pre-offset
// by i0 and strided by the batch size (64-bit offsets).
constexpr uint64_t kLaunchChunk = 1ull << 26;
static_assert(kLaunchChunk * 16 <= (1ull << 32), "per-packet column offsets must fit 32 bits");
struct KParams {
    const uint8_t* slab;
    uint64_t slab_len;
    const uint64_t* offsets;
    const uint32_t* lens;
    uint64_t off_bias;  // subtracted from every offsets[i] (host path: chunk span copied alone)
    uint64_t i0;
    uint64_t n_slot_stride;
    uint32_t stride;
    uint32_t n;
    int entry;
    int fast;  // register fast path for Ether/IPv4/UDP|TCP (entries PARSE / ETHERNET)
    pkt_out_t out;
    const uint64_t* n_dev;  // non-NULL: the batch holds min(n, *n_dev) packets (a count produced on the
                            // device, e.g. by the pcap indexer; blocks past it exit)
    const uint64_t* i0_dev;  // non-NULL (with n_dev): this launch parses packets [*i0_dev, min(n, *n_dev)) —
                             // block b takes packets *i0_dev + 256 b ... (pkt_parse_pcap_host's pieces: the
                             // records a prefix index added to the one before)
    uint32_t* nh_max;  // non-NULL: the batch's largest n_hdrs (the used slot rows), spread over kMaxSpread
                       // words (wave maxima atomicMax'ed into word blockIdx % kMaxSpread; the host
                       // takes the max of the words)
};
// Words the n_hdrs maximum is spread over: one device-scope atomic per wave on ONE word serialised —
// 2^18 of them took 2.6-3 ms per 2^24-packet parse (bench c5 r04a); spread over 256 words they do not.
constexpr uint32_t kMaxSpread = 256;

// The largest value of v over the wave (butterfly; every lane gets it).
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, m, 64));
    return v;
}

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

// Dispatch tables of the lockstep step, in LDS (built per block by dispatch_init, 576 bytes):
//   et[h(v)]  for the 16-bit dispatch values of parse_ethernet / parse_vlan (types.rs:51-75) and
//             parse_gre (fast.rs:147-153): key v << 10 | GRE next state << 5 | EtherType next state,
//             h(v) = (v * 355 >> 12) & 15 — a perfect hash of the 7 values that dispatch anywhere
//             (8100 0806 0800 86DD 8847 88BE 22EB); every other value misses its slot's key -> accept
//   ip[p]     the IPv4 (low 5 bits) and IPv6 (next 5 bits) next state of protocol byte p
//             (fast.rs:87-95, 102-110; Q6)
// One LDS read each instead of the compare chains (which the compiler turned into divergent
// branches, all taken by a mixed wave).
struct DispatchLds {
    uint32_t et[16];
    uint16_t ip[256];
};
constexpr uint32_t kDispatchKeys[7] = {0x8100u, 0x0806u, 0x0800u, 0x86DDu, 0x8847u, 0x88BEu, 0x22EBu};
__host__ __device__ constexpr uint32_t et_hash(uint32_t v) { return ((v * 355u) >> 12) & 15u; }
constexpr bool et_hash_perfect() {
    for (int a = 0; a < 7; a++)
        for (int b = a + 1; b < 7; b++)
            if (et_hash(kDispatchKeys[a]) == et_hash(kDispatchKeys[b])) return false;
    return true;
}
static_assert(et_hash_perfect(), "the dispatch hash must separate the 7 dispatching values");

// Thread t of a block of nt threads builds its share of the tables (the caller then syncs).
__device__ __forceinline__ void dispatch_init(DispatchLds* T, uint32_t t, uint32_t nt) {
    for (uint32_t p = t; p < 256u; p += nt) T->ip[p] = (uint16_t)(ipproto_next(p, false) | (ipproto_next(p, true) << 5));
    for (uint32_t h = t; h < 16u; h += nt) {
        uint32_t e = (0x1FFFFu << 10) | ((uint32_t)S_ACCEPT << 5) | S_ACCEPT;  // a key no 16-bit value has
#pragma unroll
        for (int k = 0; k < 7; k++)
            if (et_hash(kDispatchKeys[k]) == h)
                e = (kDispatchKeys[k] << 10) | (gre_next(kDispatchKeys[k]) << 5) | etype_next(kDispatchKeys[k]);
        T->et[h] = e;
    }
}

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

// A lane's view of its packet: LDS window + global fallback.
struct PacketView {
    const uint8_t* lw;        // LDS window of this packet (dword-aligned)
    const uint8_t* slab;      // slab base (16-byte aligned)
    uint64_t off;             // packet start in the slab
    uint64_t last4;           // last readable aligned dword offset of the slab
    uint32_t shift;           // LDS byte of packet byte b = b + shift (mod 2^32: "negative" after a slide)
    uint32_t win_lo;          // packet bytes [win_lo, win_end) are in the window (win_lo > 0 only
    uint32_t win_end;         //   after the lockstep walk slid the window forward)
    uint32_t len;             // packet length

    // aligned dword k of the window
    __device__ __forceinline__ uint32_t wdw(uint32_t k) const {
        return reinterpret_cast<const uint32_t*>(lw)[k];
    }
    // aligned dword of the slab containing slab byte a (clamped to the readable end)
    __device__ __forceinline__ uint32_t gdw(uint64_t a) const {
        uint64_t d = a & ~(uint64_t)3;
        d = d > last4 ? last4 : d;
        return *reinterpret_cast<const uint32_t*>(slab + d);
    }
    // n (1..4) bytes at packet offset b, little-endian in the low bytes (garbage above n).
    // Caller guarantees b + n <= len.  Bytes past the window come from global memory (L2).
    __device__ __forceinline__ uint32_t le(uint32_t b, uint32_t n) const {
        if (b >= win_lo && b + n <= win_end) {
            uint32_t wb = b + shift;
            uint32_t k = wb >> 2, sh = wb & 3;
            uint32_t lo = wdw(k);
            uint32_t hi = (sh + n > 4) ? wdw(k + 1) : 0u;
            return __builtin_amdgcn_alignbyte(hi, lo, sh);
        }
        const uint64_t a = off + b;
        const uint32_t sh = (uint32_t)(a & 3);
        // (one 8-byte load at the 4-byte-aligned address instead of the two dword loads changed
        // neither the C4 reads nor the time: profiles/ab/r05b_c4_le_dwordx2.txt)
        const uint32_t lo = gdw(a);
        const uint32_t hi = (sh + n > 4) ? gdw(a + 4) : 0u;
        return __builtin_amdgcn_alignbyte(hi, lo, sh);
    }
    __device__ __forceinline__ uint32_t u8(uint32_t b) const { return le(b, 1) & 0xFFu; }
    __device__ __forceinline__ uint32_t be16(uint32_t b) const { return bswap32(le(b, 2)) >> 16; }

    // NW big-endian dwords of header bytes [b, b + 4*NW) (bytes past the header's own
    // `nbytes` are whatever follows and are never interpreted).  Caller: b + nbytes <= len.
    template <int NW>
    __device__ __forceinline__ void hdr(uint32_t b, uint32_t nbytes, uint32_t (&d)[NW]) const {
        (void)nbytes;
        uint32_t a[NW + 1];
        uint32_t sh;
        if (b >= win_lo && b + 4 * NW <= win_end) {
            // unaligned LDS reads (gfx950 unaligned-ds-access): the header's bytes as they lie, not
            // dword pairs + v_alignbyte (C2 isolated 28.9 -> 27.3 us,
            // profiles/ab/r02ulds_unaligned_lds.txt; le() keeps the dword pair: as one unaligned load
            // it made extract_kernel's 19 getters 68.6 -> 79.5 us)
            uint32_t u[NW];
            __builtin_memcpy(u, lw + (uint32_t)(b + shift), 4 * NW);
#pragma unroll
            for (int i = 0; i < NW; i++) d[i] = bswap32(u[i]);
            return;
        } else {
            const uint64_t ga = off + b, g4 = ga & ~(uint64_t)3;
            sh = (uint32_t)(ga & 3);
            // The header's dwords by 16-byte loads (4-byte aligned: one instruction and one wait
            // per 16 bytes instead of per dword; C4 pipelined -2..-4 %, the line-request count is
            // unchanged, profiles/ab/r02hv_header_vector_loads.txt); per dword near the slab's
            // readable end.
            constexpr int NQ = (NW + 1 + 3) / 4;
            if (g4 + 16u * NQ <= last4 + 4) {
#pragma unroll
                for (int q = 0; q < NQ; q++) {
                    uint32_t v[4];
                    __builtin_memcpy(v, __builtin_assume_aligned(slab + g4 + 16u * q, 4), 16);
#pragma unroll
                    for (int j = 0; j < 4; j++)
                        if (4 * q + j <= NW) a[4 * q + j] = v[j];
                }
            } else {
#pragma unroll
                for (int i = 0; i <= NW; i++) a[i] = gdw(ga + 4u * i);
            }
        }
#pragma unroll
        for (int i = 0; i < NW; i++) d[i] = bswap32(__builtin_amdgcn_alignbyte(a[i + 1], a[i], sh));
    }
};

struct WalkResult {
    uint32_t status, n, payload_off, mask;
    int32_t f_eth, f_vlan, f_ipv4, f_ipv6, f_tcp, f_udp;  // first offsets, -1 = absent
};

// Header type and size recorded by the walk state S (make_header! sizes, headers.rs:529-827).
template <uint32_t S> struct StateHdr;
template <> struct StateHdr<S_DOT3> { static constexpr uint32_t T = PKT_HDR_DOT3, SZ = 14; };
template <> struct StateHdr<S_LLC> { static constexpr uint32_t T = PKT_HDR_LLC, SZ = 3; };
template <> struct StateHdr<S_SNAP> { static constexpr uint32_t T = PKT_HDR_SNAP, SZ = 5; };
template <> struct StateHdr<S_ETHER> { static constexpr uint32_t T = PKT_HDR_ETHER, SZ = 14; };
template <> struct StateHdr<S_VLAN> { static constexpr uint32_t T = PKT_HDR_VLAN, SZ = 4; };
template <> struct StateHdr<S_MPLS> { static constexpr uint32_t T = PKT_HDR_MPLS, SZ = 4; };
template <> struct StateHdr<S_MPLS_BOS> { static constexpr uint32_t T = PKT_HDR_MPLS, SZ = 4; };
template <> struct StateHdr<S_IPV4> { static constexpr uint32_t T = PKT_HDR_IPV4, SZ = 20; };
template <> struct StateHdr<S_IPV6> { static constexpr uint32_t T = PKT_HDR_IPV6, SZ = 40; };
template <> struct StateHdr<S_GRE> { static constexpr uint32_t T = PKT_HDR_GRE, SZ = 4; };
template <> struct StateHdr<S_ERSPAN2> { static constexpr uint32_t T = PKT_HDR_ERSPAN2, SZ = 8; };
template <> struct StateHdr<S_ERSPAN3> { static constexpr uint32_t T = PKT_HDR_ERSPAN3, SZ = 12; };
template <> struct StateHdr<S_ARP> { static constexpr uint32_t T = PKT_HDR_ARP, SZ = 28; };
template <> struct StateHdr<S_ICMP> { static constexpr uint32_t T = PKT_HDR_ICMP, SZ = 4; };
template <> struct StateHdr<S_TCP> { static constexpr uint32_t T = PKT_HDR_TCP, SZ = 20; };
template <> struct StateHdr<S_UDP> { static constexpr uint32_t T = PKT_HDR_UDP, SZ = 8; };
template <> struct StateHdr<S_VXLAN> { static constexpr uint32_t T = PKT_HDR_VXLAN, SZ = 8; };

// Per-lane walk state.
struct Lane {
    uint32_t st, o, steps;
    bool live;
    WalkResult r;
};

// Record (type T, offset) in list slot r.n (PacketSlice::insert order, packet.rs:724-726).
template <uint32_t T, class Push>
__device__ __forceinline__ void rec(Lane& L, uint32_t off, Push& push) {
    push(L.r.n, T, off);
    L.r.n++;
    L.r.mask |= 1u << T;
    if constexpr (T == PKT_HDR_ETHER) { if (L.r.f_eth < 0) L.r.f_eth = (int32_t)off; }
    if constexpr (T == PKT_HDR_VLAN) { if (L.r.f_vlan < 0) L.r.f_vlan = (int32_t)off; }
    if constexpr (T == PKT_HDR_IPV4) { if (L.r.f_ipv4 < 0) L.r.f_ipv4 = (int32_t)off; }
    if constexpr (T == PKT_HDR_IPV6) { if (L.r.f_ipv6 < 0) L.r.f_ipv6 = (int32_t)off; }
    if constexpr (T == PKT_HDR_TCP) { if (L.r.f_tcp < 0) L.r.f_tcp = (int32_t)off; }
    if constexpr (T == PKT_HDR_UDP) { if (L.r.f_udp < 0) L.r.f_udp = (int32_t)off; }
}

__device__ __forceinline__ void fail(Lane& L, uint32_t st) {
    L.r.status = st;
    L.live = false;
}

// One step of the walk for a lane in state S: bounds (the reference's slice panic, Q7), then
// depth, then the dispatch field, record, advance.  fast.rs line numbers per state.
template <uint32_t S, class Push>
__device__ __forceinline__ void step(Lane& L, const PacketView& pv, Push& push) {
    const uint32_t o = L.o, len = pv.len;
    if constexpr (S == S_ACCEPT) {  // fast.rs:223-227
        L.r.payload_off = o;
        L.live = false;
    } else if constexpr (S == S_PARSE) {  // fast.rs:5-12 reads arr[12], arr[13]
        if (o + 14 > len) { fail(L, PKT_TRUNCATED); return; }
        L.st = (pv.be16(o + 12) < 1500u) ? S_DOT3 : S_ETHER;
    } else {
        constexpr uint32_t T = StateHdr<S>::T, SZ = StateHdr<S>::SZ;
        if (o + SZ > len) { fail(L, PKT_TRUNCATED); return; }     // `&arr[0..X::size()]`
        if (L.r.n >= PKT_MAX_HDRS) { fail(L, PKT_DEPTH_LIMIT); return; }
        if constexpr (S == S_GRE) {  // fast.rs:114-165: options sliced C,K,S; listed S,K,C (Q2)
            const uint32_t w = bswap32(pv.le(o, 4));
            const uint32_t c = w >> 31, k = (w >> 29) & 1u, s = (w >> 28) & 1u;
            rec<T>(L, o, push);
            uint32_t q = o + 4, oc = 0, okey = 0, oseq = 0;
            if (c) {
                if (q + 4 > len) { fail(L, PKT_TRUNCATED); return; }
                if (L.r.n >= PKT_MAX_HDRS) { fail(L, PKT_DEPTH_LIMIT); return; }
                oc = q; q += 4;
            }
            if (k) {
                if (q + 4 > len) { fail(L, PKT_TRUNCATED); return; }
                if (L.r.n + c >= PKT_MAX_HDRS) { fail(L, PKT_DEPTH_LIMIT); return; }
                okey = q; q += 4;
            }
            if (s) {
                if (q + 4 > len) { fail(L, PKT_TRUNCATED); return; }
                if (L.r.n + c + k >= PKT_MAX_HDRS) { fail(L, PKT_DEPTH_LIMIT); return; }
                oseq = q; q += 4;
            }
            if (s) rec<PKT_HDR_GRE_SEQUENCE_NUM>(L, oseq, push);
            if (k) rec<PKT_HDR_GRE_KEY>(L, okey, push);
            if (c) rec<PKT_HDR_GRE_CHKSUM_OFFSET>(L, oc, push);
            L.o = q;
            L.st = gre_next(w & 0xFFFFu);
        } else if constexpr (S == S_ERSPAN3) {  // fast.rs:172-192: o bit (95) -> ERSPANPLATFORM
            const uint32_t ob = pv.u8(o + 11) & 1u;
            rec<T>(L, o, push);
            uint32_t q = o + 12;
            if (ob) {
                if (q + 8 > len) { fail(L, PKT_TRUNCATED); return; }
                if (L.r.n >= PKT_MAX_HDRS) { fail(L, PKT_DEPTH_LIMIT); return; }
                rec<PKT_HDR_ERSPAN_PLATFORM>(L, q, push);
                q += 8;
            }
            L.o = q;
            L.st = S_ETHER;
        } else {
            uint32_t next;
            if constexpr (S == S_DOT3) next = S_LLC;
            else if constexpr (S == S_LLC)  // fast.rs:21: aa aa 03 -> SNAP
                next = ((pv.le(o, 3) & 0xFFFFFFu) == 0x03AAAAu) ? S_SNAP : S_ACCEPT;
            else if constexpr (S == S_ETHER) next = etype_next(pv.be16(o + 12));
            else if constexpr (S == S_VLAN) next = etype_next(pv.be16(o + 2));
            else if constexpr (S == S_MPLS) next = (pv.u8(o + 2) & 1u) ? S_MPLS_BOS : S_MPLS;  // bos bit 23
            else if constexpr (S == S_MPLS_BOS) {  // fast.rs:74-83: arr[MPLS::size()] must exist (Q3)
                if (o + 5 > len) { fail(L, PKT_TRUNCATED); return; }
                const uint32_t nib = pv.u8(o + 4) >> 4;
                next = (nib == 4u) ? S_IPV4 : ((nib == 6u) ? S_IPV6 : S_ETHER);
            } else if constexpr (S == S_IPV4) next = ipproto_next(pv.u8(o + 9), false);
            else if constexpr (S == S_IPV6) next = ipproto_next(pv.u8(o + 6), true);
            else if constexpr (S == S_UDP) next = (pv.be16(o + 2) == 4789u) ? S_VXLAN : S_ACCEPT;  // types.rs:7
            else if constexpr (S == S_SNAP || S == S_ARP || S == S_ICMP || S == S_TCP) next = S_ACCEPT;
            else next = S_ETHER;  // ERSPAN2, VXLAN
            rec<T>(L, o, push);
            L.o = o + SZ;
            L.st = next;
        }
    }
}

// The walk: a waterfall over the distinct states present in the wave.  Each iteration takes the
// state of the first live lane (v_readlane), and every live lane in that state advances one
// step under a SCALAR switch — a wave whose packets share a layout runs exactly one case per
// header, a mixed wave one case per distinct state.
// ---- lockstep step: one header for a lane in ANY state, with the per-state constants read from
// packed tables and the next state chosen by selects (no divergent branch per state).
// Semantics are exactly step<S>'s: same checks in the same order, same records.

// 6-bit fields per state (states 0..9 in lo, 10..18 in hi): header size (PARSE: the 14 bytes
// fast.rs:6 reads; ACCEPT: 0).
constexpr uint64_t pack6(const uint32_t (&v)[10], int k0) {
    uint64_t r = 0;
    for (int i = 0; i < 10; i++)
        if (k0 + i < 19) r |= (uint64_t)(v[i] & 63u) << (6 * i);
    return r;
}
//                                    PARSE DOT3 LLC SNAP ETHER VLAN MPLS BOS IPV4 IPV6
constexpr uint32_t kSzLo[10]       = {14,   14,  3,  5,   14,   4,   4,   4,  20,  40};
//                                    GRE  ER2 ER3 ARP ICMP TCP UDP VXLAN ACCEPT
constexpr uint32_t kSzHi[10]       = {4,   8,  12, 28, 4,   20, 8,  8,    0, 0};
constexpr uint32_t kTyLo[10]       = {0, PKT_HDR_DOT3, PKT_HDR_LLC, PKT_HDR_SNAP, PKT_HDR_ETHER, PKT_HDR_VLAN,
                                      PKT_HDR_MPLS, PKT_HDR_MPLS, PKT_HDR_IPV4, PKT_HDR_IPV6};
constexpr uint32_t kTyHi[10]       = {PKT_HDR_GRE, PKT_HDR_ERSPAN2, PKT_HDR_ERSPAN3, PKT_HDR_ARP, PKT_HDR_ICMP,
                                      PKT_HDR_TCP, PKT_HDR_UDP, PKT_HDR_VXLAN, 0, 0};
// byte offset of the big-endian dword holding the dispatch field
//                                    PARSE DOT3 LLC SNAP ETHER VLAN MPLS BOS IPV4 IPV6
constexpr uint32_t kDwLo[10]       = {12,   0,   0,  0,   12,   2,   0,   4,  8,   4};
//                                    GRE  ER2 ER3 ARP ICMP TCP UDP VXLAN ACCEPT
constexpr uint32_t kDwHi[10]       = {0,   0,  8,  0,  0,   0,  2,  0,    0, 0};
constexpr uint64_t kSz0 = pack6(kSzLo, 0), kSz1 = pack6(kSzHi, 10);
constexpr uint64_t kTy0 = pack6(kTyLo, 0), kTy1 = pack6(kTyHi, 10);
constexpr uint64_t kDw0 = pack6(kDwLo, 0), kDw1 = pack6(kDwHi, 10);
// states whose next state (or option / platform test) depends on their dispatch dword D (lstep)
constexpr uint32_t kNeedsD = (1u << S_PARSE) | (1u << S_LLC) | (1u << S_ETHER) | (1u << S_VLAN) | (1u << S_MPLS) |
                             (1u << S_MPLS_BOS) | (1u << S_IPV4) | (1u << S_IPV6) | (1u << S_GRE) |
                             (1u << S_ERSPAN3) | (1u << S_UDP);

__device__ __forceinline__ uint32_t tab6(uint64_t lo, uint64_t hi, uint32_t st) {
    const bool h = st >= 10u;
    const uint64_t t = h ? hi : lo;
    // 24-bit multiply (full rate; a 32-bit v_mul_lo_u32 issues at quarter rate)
    return (uint32_t)(t >> __umul24(6u, h ? st - 10u : st)) & 63u;
}

// One lockstep iteration for every live lane: the header of the lane's state is checked, read and
// recorded with the state kept in a few registers and the checks folded into one failure code (no
// early returns: a branchy form made the compiler copy the whole lane state at every exit).  Only
// GRE options and the ERSPAN3 platform header take a branch, taken when a lane needs it.
// Semantics are exactly step<S>'s: same checks in the same order, same records.  The first offset
// of each field group's type (Ether, Vlan, IPv4, IPv6, TCP, UDP; Q11) is kept in f[] when the type is
// first recorded.
struct LockLane {
    uint32_t st, o, n, mask, status, pay, steps;
    bool live;
    int32_t f[6];  // first offsets of types 1, 2, 3, 4, 6, 7 (-1 = none)
};

// Record (t, off) in slot L.n without touching the first offsets: the GRE option and ERSPAN
// platform types (14-16, 19) are never one of the six field groups.
template <class Push>
__device__ __forceinline__ void lrec_opt(LockLane& L, uint32_t t, uint32_t off, Push& push) {
    push(L.n, t, off);
    L.mask |= 1u << t;
    L.n++;
}

// One lockstep iteration for lane state L and its dispatch dword D (big-endian), `live` = the lane
// takes part.  Every new value is computed for every lane and committed by selects (only the
// slot stores and the rare GRE-option / ERSPAN-platform records branch), so the compiler keeps
// one copy of the lane state instead of re-materialising it at every divergent merge.
template <class Push>
__device__ __forceinline__ void lstep(LockLane& L, uint32_t len, uint32_t D, Push& push, bool live,
                                      const DispatchLds* T) {
    const uint32_t st = L.st, o = L.o;
    const uint32_t sz = tab6(kSz0, kSz1, st);
    const uint32_t hw = D >> 16;
    // table dispatch: the 16-bit value (EtherType, or GRE's protocol in the dword's low half) and
    // the IP protocol byte, one LDS read each
    const uint32_t k16 = st == S_GRE ? (D & 0xFFFFu) : hw;
    const uint32_t te = T->et[et_hash(k16)];
    const bool hit = (te >> 10) == k16;
    const uint32_t et_next = hit ? (te & 31u) : (uint32_t)S_ACCEPT;
    const uint32_t gr_next = hit ? ((te >> 5) & 31u) : (uint32_t)S_ACCEPT;
    const bool v6 = st == S_IPV6;
    const uint32_t ti = T->ip[v6 ? (D >> 8) & 0xFFu : hw & 0xFFu];
    const uint32_t ip_next = v6 ? (uint32_t)(ti >> 5) : (uint32_t)(ti & 31u);
    uint32_t nx = S_ACCEPT;  // SNAP, ARP, ICMP, TCP
    nx = (st == S_PARSE) ? (hw < 1500u ? S_DOT3 : S_ETHER) : nx;
    nx = (st == S_DOT3) ? S_LLC : nx;
    nx = (st == S_LLC) ? ((D >> 8) == 0xAAAA03u ? S_SNAP : S_ACCEPT) : nx;
    nx = (st == S_ETHER || st == S_VLAN) ? et_next : nx;
    nx = (st == S_MPLS) ? (((D >> 8) & 1u) ? S_MPLS_BOS : S_MPLS) : nx;
    nx = (st == S_MPLS_BOS) ? ((D >> 28) == 4u ? S_IPV4 : ((D >> 28) == 6u ? S_IPV6 : S_ETHER)) : nx;
    nx = (st == S_IPV4 || st == S_IPV6) ? ip_next : nx;
    nx = (st == S_GRE) ? gr_next : nx;
    nx = (st == S_ERSPAN2 || st == S_ERSPAN3 || st == S_VXLAN) ? S_ETHER : nx;
    nx = (st == S_UDP) ? (hw == 4789u ? S_VXLAN : S_ACCEPT) : nx;
    // the reference's panics in its order: iteration bound (walk), `&arr[0..X::size()]`, depth,
    // parse_mpls_bos's arr[4] (fast.rs:74-83, Q3); accept ends the walk (fast.rs:223-227)
    const uint32_t steps = L.steps + 1;
    const bool acc = st == S_ACCEPT;
    uint32_t f = 0;
    f = (st == S_MPLS_BOS && o + 5 > len) ? (uint32_t)PKT_TRUNCATED : f;
    f = (st != S_PARSE && L.n >= PKT_MAX_HDRS) ? (uint32_t)PKT_DEPTH_LIMIT : f;
    f = (o + sz > len) ? (uint32_t)PKT_TRUNCATED : f;
    f = acc ? 0u : f;
    f = (steps > PKT_MAX_HDRS + 3) ? (uint32_t)PKT_DEPTH_LIMIT : f;
    const bool go = live && f == 0 && !acc;
    const bool rec = go && st != S_PARSE;
    // the record of this step's header (branch-free; the slot stores are masked by `rec`)
    const uint32_t t = tab6(kTy0, kTy1, st);
    if (rec) push(L.n, t, o);
    const bool first = rec && !((L.mask >> t) & 1u);
    L.f[0] = (first && t == PKT_HDR_ETHER) ? (int32_t)o : L.f[0];
    L.f[1] = (first && t == PKT_HDR_VLAN) ? (int32_t)o : L.f[1];
    L.f[2] = (first && t == PKT_HDR_IPV4) ? (int32_t)o : L.f[2];
    L.f[3] = (first && t == PKT_HDR_IPV6) ? (int32_t)o : L.f[3];
    L.f[4] = (first && t == PKT_HDR_TCP) ? (int32_t)o : L.f[4];
    L.f[5] = (first && t == PKT_HDR_UDP) ? (int32_t)o : L.f[5];
    L.mask = rec ? (L.mask | (1u << t)) : L.mask;
    L.n = rec ? L.n + 1 : L.n;
    uint32_t q = rec ? o + sz : o;
    const bool gopt = rec && st == S_GRE && (D & 0xB0000000u) != 0;
    const bool plat = rec && st == S_ERSPAN3 && (D & 1u);
    if (gopt) {  // fast.rs:114-165: options sliced C,K,S; listed S,K,C (Q2)
        const uint32_t c = D >> 31, k = (D >> 29) & 1u, sb = (D >> 28) & 1u;
        if (c) f = (q + 4 > len) ? (uint32_t)PKT_TRUNCATED : (L.n >= PKT_MAX_HDRS ? (uint32_t)PKT_DEPTH_LIMIT : 0u);
        const uint32_t oc = q;
        q += 4u * c;
        if (!f && k) f = (q + 4 > len) ? (uint32_t)PKT_TRUNCATED : (L.n + c >= PKT_MAX_HDRS ? (uint32_t)PKT_DEPTH_LIMIT : 0u);
        const uint32_t okey = q;
        q += 4u * k;
        if (!f && sb) f = (q + 4 > len) ? (uint32_t)PKT_TRUNCATED : (L.n + c + k >= PKT_MAX_HDRS ? (uint32_t)PKT_DEPTH_LIMIT : 0u);
        const uint32_t oseq = q;
        q += 4u * sb;
        if (!f) {
            if (sb) lrec_opt(L, PKT_HDR_GRE_SEQUENCE_NUM, oseq, push);
            if (k) lrec_opt(L, PKT_HDR_GRE_KEY, okey, push);
            if (c) lrec_opt(L, PKT_HDR_GRE_CHKSUM_OFFSET, oc, push);
        }
    } else if (plat) {  // fast.rs:172-192: o bit -> ERSPANPLATFORM
        f = (q + 8 > len) ? (uint32_t)PKT_TRUNCATED : (L.n >= PKT_MAX_HDRS ? (uint32_t)PKT_DEPTH_LIMIT : 0u);
        if (!f) {
            lrec_opt(L, PKT_HDR_ERSPAN_PLATFORM, q, push);
            q += 8;
        }
    }
    // commit (lanes not taking part keep their state).  A lane whose next state is ACCEPT takes
    // that step now instead of in one more iteration (fast.rs:223-227: the payload starts at q),
    // with the walk's iteration bound for it — the only check the accept step has.
    const bool cont = go && f == 0;
    const bool facc = cont && nx == S_ACCEPT;
    const uint32_t fa = (steps + 1 > PKT_MAX_HDRS + 3) ? (uint32_t)PKT_DEPTH_LIMIT : 0u;
    L.steps = live ? steps + (facc ? 1u : 0u) : L.steps;
    L.pay = (live && acc && f == 0) ? o : ((facc && fa == 0) ? q : L.pay);
    L.status = (live && f) ? f : ((facc && fa) ? fa : L.status);
    L.live = cont && !facc;
    L.o = live ? q : L.o;
    L.st = live ? nx : L.st;
}

// The walk.  WK = 0, waterfall: each iteration takes the state of the first live lane and every
// live lane in that state advances one step under a SCALAR switch — a wave whose packets share a
// layout runs exactly one case per header, a mixed wave one case per distinct (state, depth).
// WK = 1, lockstep: every live lane advances one header per iteration through lstep() — a mixed
// wave runs (its longest chain + 2) iterations (C4: 10 instead of ~38).
// (Refilling the window for headers past it, one round trip per wave instead of one dependent read
// per header, measured slower: C4 status-only 88-90 vs 66-68 us; so did prefetching the sectors past
// the window into L2, 78 vs 67 us — profiles/ab/r02o_c4_refill_prefetch.txt.  Round 3 instead sizes
// indexed windows to hold every header the 22 templates carry, parse_kernel.)
template <int WK, class Push>
__device__ __forceinline__ void walk(PacketView& pv, uint32_t state, bool active, Push&& push,
                                     WalkResult& out, const DispatchLds* T = nullptr) {
    if constexpr (WK == 1) {
        LockLane L{state, 0, 0, 0, PKT_OK, 0, 0, active, {-1, -1, -1, -1, -1, -1}};
        if (state == S_PARSE) {
            // fast.rs:5-12's dispatch, lstep's PARSE case taken before the loop (no record, no
            // offset change): >= 14 bytes go to Dot3 (EtherType field < 1500) or Ether, shorter
            // records are truncated
            const uint32_t hw = active ? pv.be16(12) : 0u;
            L.steps = active ? 1u : 0u;
            L.status = (active && pv.len < 14u) ? (uint32_t)PKT_TRUNCATED : (uint32_t)PKT_OK;
            L.live = active && pv.len >= 14u;
            L.st = hw < 1500u ? S_DOT3 : S_ETHER;
        }
        const uint32_t* w = reinterpret_cast<const uint32_t*>(pv.lw);
        while (__ballot(L.live)) {
            const bool live = L.live;
            // the dispatch dword of this step (big-endian; bytes past the header are read but
            // never used): from the window when it holds it (every lane reads, at an in-window
            // address), else from global memory — only if the step gets past its iteration and
            // slice checks (a rare divergent branch)
            const uint32_t b = L.o + tab6(kDw0, kDw1, L.st);
            const bool in_win = b >= pv.win_lo && b + 4 <= pv.win_end;
            const uint32_t wb = in_win ? b + pv.shift : 0u, k = wb >> 2, sh = wb & 3;
            uint32_t D = __builtin_amdgcn_alignbyte(w[k + 1], w[k], sh);
            // (only states whose next state depends on D read it from memory: DOT3 -> LLC, SNAP / ARP /
            // ICMP / TCP -> accept and ERSPAN2 / VXLAN -> Ether whatever their bytes hold, so a lane
            // in one of them past the window issues no read — C4's inner TCP / ICMP headers)
            const bool far = live && !in_win && ((kNeedsD >> L.st) & 1u) && L.steps < PKT_MAX_HDRS + 3 &&
                             L.o + tab6(kSz0, kSz1, L.st) <= pv.len;
            if (__ballot(far)) {
                if (far) D = pv.le(b, 4);
            }
            lstep(L, pv.len, bswap32(D), push, live, T);
        }
        out.status = L.status;
        out.n = L.n;
        out.payload_off = L.pay;
        out.mask = L.mask;
        const bool ok = L.status == PKT_OK;
        out.f_eth = ok ? L.f[0] : -1;
        out.f_vlan = ok ? L.f[1] : -1;
        out.f_ipv4 = ok ? L.f[2] : -1;
        out.f_ipv6 = ok ? L.f[3] : -1;
        out.f_tcp = ok ? L.f[4] : -1;
        out.f_udp = ok ? L.f[5] : -1;
        return;
    }
    Lane L;
    L.st = state;
    L.o = 0;
    L.steps = 0;
    L.live = active;
    L.r.status = PKT_OK;
    L.r.n = 0;
    L.r.payload_off = 0;
    L.r.mask = 0;
    L.r.f_eth = L.r.f_vlan = L.r.f_ipv4 = L.r.f_ipv6 = L.r.f_tcp = L.r.f_udp = -1;
    for (;;) {
        const uint64_t pend = __ballot(L.live);
        if (pend == 0) break;
        uint32_t s0 = __builtin_amdgcn_readlane(L.st, (uint32_t)__builtin_ctzll(pend));
        const bool mine = L.live && L.st == s0;
        // Make s0 opaque: inside `mine` the compiler would otherwise substitute the lane's own
        // (VGPR) state for s0 and turn the uniform scalar switch into a divergent compare tree
        // with an exec-mask save/restore per level.
        asm volatile("" : "+s"(s0));
        if (mine) {
            // at most PKT_MAX_HDRS headers + parse + accept + the failing step
            if (++L.steps > PKT_MAX_HDRS + 3) {
                fail(L, PKT_DEPTH_LIMIT);
            } else {
                switch (s0) {
                    case S_PARSE: step<S_PARSE>(L, pv, push); break;
                    case S_DOT3: step<S_DOT3>(L, pv, push); break;
                    case S_LLC: step<S_LLC>(L, pv, push); break;
                    case S_SNAP: step<S_SNAP>(L, pv, push); break;
                    case S_ETHER: step<S_ETHER>(L, pv, push); break;
                    case S_VLAN: step<S_VLAN>(L, pv, push); break;
                    case S_MPLS: step<S_MPLS>(L, pv, push); break;
                    case S_MPLS_BOS: step<S_MPLS_BOS>(L, pv, push); break;
                    case S_IPV4: step<S_IPV4>(L, pv, push); break;
                    case S_IPV6: step<S_IPV6>(L, pv, push); break;
                    case S_GRE: step<S_GRE>(L, pv, push); break;
                    case S_ERSPAN2: step<S_ERSPAN2>(L, pv, push); break;
                    case S_ERSPAN3: step<S_ERSPAN3>(L, pv, push); break;
                    case S_ARP: step<S_ARP>(L, pv, push); break;
                    case S_ICMP: step<S_ICMP>(L, pv, push); break;
                    case S_TCP: step<S_TCP>(L, pv, push); break;
                    case S_UDP: step<S_UDP>(L, pv, push); break;
                    case S_VXLAN: step<S_VXLAN>(L, pv, push); break;
                    default: step<S_ACCEPT>(L, pv, push); break;
                }
            }
        }
    }
    out = L.r;
}

// A 16-byte run of packet bytes as a 128-bit big-endian integer (bit 0 of the make_header!
// numbering = the MSB of hi), for setting fields with one shift and mask (pktgpu_gen.hip,
// pktgpu_rewrite.hip).
struct U128 {
    uint64_t hi, lo;  // big-endian: hi = bytes 0..7, lo = bytes 8..15
};

__device__ __forceinline__ U128 shl(U128 x, uint32_t s) {  // s < 128
    if (s == 0) return x;
    if (s >= 64) return {x.lo << (s - 64), 0};
    return {(x.hi << s) | (x.lo >> (64 - s)), x.lo << s};
}
__device__ __forceinline__ U128 shr(U128 x, uint32_t s) {  // s < 128
    if (s == 0) return x;
    if (s >= 64) return {0, x.hi >> (s - 64)};
    return {x.hi >> s, (x.lo >> s) | (x.hi << (64 - s))};
}

// set_bit_range (headers.rs:315-324) of bits [s, e] (MSB-first numbering, e - s < 64) to v's low w
// bits, on the 128-bit run whose first bit is `b0` (the field overlaps the run; bits outside the
// run are dropped).
__device__ __forceinline__ void put_bits(U128& x, uint32_t s, uint32_t e, uint32_t w, uint64_t v, uint32_t b0) {
    (void)s;
    const uint64_t m = w >= 64 ? ~0ull : ((1ull << w) - 1ull);
    const int32_t sh = 127 - ((int32_t)e - (int32_t)b0);  // where value bit 0 lands (from the LSB)
    U128 V{0, v & m}, M{0, m};
    if (sh >= 0) {
        V = shl(V, (uint32_t)sh);
        M = shl(M, (uint32_t)sh);
    } else {
        V = shr(V, (uint32_t)-sh);
        M = shr(M, (uint32_t)-sh);
    }
    x.hi = (x.hi & ~M.hi) | V.hi;
    x.lo = (x.lo & ~M.lo) | V.lo;
}

}  // namespace pktgpu
