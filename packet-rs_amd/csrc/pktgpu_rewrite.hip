// pktgpu_rewrite.hip — batched work over an already parsed batch and the
// small helpers around it.  Every kernel reads the chain columns pkt_parse_batch wrote.
//
//   extract_kernel     `<Hdr>Slice::<field>()` (headers.rs:195-201 -> bit_range 252-263) for any
//                      (type, occurrence, bits), EVERY spec in one launch: a lane copies its packet's
//                      chain and its first 80 bytes into LDS once and answers all specs from there
//                      (bytes past the window from global memory).
//   to_vec_kernel      PacketSlice::to_vec / Packet::to_vec (packet.rs:733-740, 385-392).  Headers lie
//                      back to back on the wire and the list is in wire order except after a GRE with
//                      two or more options (Q2), so for every other packet to_vec IS the packet's bytes
//                      [0, len) — known from hdr_mask alone (at most one GRE option type), else checked
//                      against the slot rows.  One wave per 64 packets: lane k reads packet k's
//                      metadata; the wave's packets then form one list of 16-byte destination chunks
//                      (a wave scan of the per-packet counts) that the lanes copy 64 at a time
//                      (a funnel shift when source and destination differ in alignment).  Q2
//                      packets are gathered through the list by the whole wave, one at a time.
//   tv_window_kernel   the same into a capture's own layout (records in order, none sharing a
//                      16-byte chunk: tv_overlap_kernel checks on the device): one wave per 4 KiB of
//                      destination, its source loads issued first, records found per chunk from a
//                      map of the record starts in the window; chunks shared with the record
//                      headers between records merged with the destination's own bytes.
//   set_fields_kernel  set_bit_range (headers.rs:315-324) per spec, in spec order, in place; chain in
//                      LDS, all specs (up to 32) in one launch.  The wave loads its packets' first 80
//                      bytes into LDS cooperatively, every setter whose field lies there is applied in
//                      LDS (one shift and mask on a 16-byte piece), and the chunks holding set bytes
//                      are stored back cooperatively, the packet's own bytes only; a packet with a
//                      field past its window or wider than 64 bits is set in global memory instead.
//                      pkt_set_fields_csum refreshes one IPv4 header's checksum in the same pass.
//                      (extract / set_fields: spec tables in LDS, every prologue load in flight
//                      before the first wait: no memory round trip per spec.)
//   ipv4_update_kernel / ipv4_csum_kernel   Packet::ipv4_checksum (packet.rs:93-107, Q1 fold).
//   broadcast_kernel   n copies of one packet (the clone step of the pktgen loop).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

#include "pktgpu_ctx.hpp"
#include "pktgpu_device.hpp"

using namespace pktgpu;

namespace {

__constant__ uint8_t kHdrSize[PKT_HDR_COUNT] = {0, 14, 4, 20, 40, 4, 20, 8, 28, 8, 14, 3, 5, 4, 4, 4, 4, 8, 12, 8, 35, 4};

constexpr uint32_t kRwBlock = 256;
constexpr int kMaxSpecs = 32;  // specs per launch (extract / set_fields)
static_assert(kRwBlock >= (uint32_t)kMaxSpecs, "one thread copies each spec into the LDS spec table");

struct BatchRef {
    const uint8_t* slab;
    uint64_t slab_len;
    const uint64_t* offsets;
    const uint32_t* lens;
    uint32_t stride;
    uint64_t n;
    const uint8_t* n_hdrs;
    const uint8_t* hdr_type;   // [PKT_MAX_HDRS][n]
    const uint16_t* hdr_off;   // [PKT_MAX_HDRS][n]
};

__device__ __forceinline__ uint64_t pkt_off(const BatchRef& b, uint64_t i) {
    return b.offsets ? b.offsets[i] : i * (uint64_t)b.stride;
}

// aligned dword of the slab containing byte a, clamped to the readable end (round_up(len, 16))
__device__ __forceinline__ uint32_t slab_dw(const BatchRef& b, uint64_t a) {
    const uint64_t last4 = ((b.slab_len + 15) & ~(uint64_t)15) - 4;
    uint64_t d = a & ~(uint64_t)3;
    d = d > last4 ? last4 : d;
    return *reinterpret_cast<const uint32_t*>(b.slab + d);
}

// The lane's chain: its first kChainLds slots in LDS (slot-major [slot][lane]: per-lane byte /
// u16 reads of one slot are consecutive addresses, conflict-free), deeper slots read from the
// chain columns in global memory when a search gets there (chains of > 8 headers are rare, and
// the smaller LDS footprint buys occupancy).
constexpr uint32_t kChainLds = 8;
struct ChainLds {
    uint8_t type[kChainLds][kRwBlock];
    uint16_t off[kChainLds][kRwBlock];
};

// Stage packet i's first slots in LDS: chain_load issues n_hdrs and the first 4 slot rows
// unconditionally (the columns are [PKT_MAX_HDRS][n], so rows past n_hdrs are readable; their
// bytes are never used), so that they are in flight together with the caller's other loads: one
// memory round trip for the common chains instead of one per slot.  chain_store writes them and
// loads any deeper slots; returns n_hdrs (clamped to PKT_MAX_HDRS).
static_assert(PKT_MAX_HDRS >= 4 && kChainLds >= 4, "first 4 slot rows staged unconditionally");
struct ChainPre {
    uint32_t nh, ty[4], of[4];
};
__device__ __forceinline__ ChainPre chain_load(const BatchRef& b, uint64_t i) {
    ChainPre c;
    c.nh = b.n_hdrs[i];
#pragma unroll
    for (uint32_t j = 0; j < 4; j++) {
        c.ty[j] = b.hdr_type[(uint64_t)j * b.n + i];
        c.of[j] = b.hdr_off[(uint64_t)j * b.n + i];
    }
    return c;
}
__device__ __forceinline__ uint32_t chain_store(const BatchRef& b, uint64_t i, uint32_t t, ChainLds& L, const ChainPre& c) {
    const uint32_t nh = c.nh > PKT_MAX_HDRS ? PKT_MAX_HDRS : c.nh;
#pragma unroll
    for (uint32_t j = 0; j < 4; j++) {
        L.type[j][t] = (uint8_t)c.ty[j];
        L.off[j][t] = (uint16_t)c.of[j];
    }
    for (uint32_t j = 4; j < nh && j < kChainLds; j++) {
        L.type[j][t] = b.hdr_type[(uint64_t)j * b.n + i];
        L.off[j][t] = b.hdr_off[(uint64_t)j * b.n + i];
    }
    return nh;
}

__device__ __forceinline__ uint32_t stage_chain(const BatchRef& b, uint64_t i, uint32_t t, ChainLds& L) {
    return chain_store(b, i, t, L, chain_load(b, i));
}

// offset of the occurrence-th header of `type` in packet i's chain, or -1
__device__ __forceinline__ int32_t find_lds(const ChainLds& L, const BatchRef& b, uint64_t i, uint32_t t, uint32_t nh,
                                            uint32_t type, uint32_t occ) {
    uint32_t c = 0;
    for (uint32_t j = 0; j < nh; j++) {
        const bool in = j < kChainLds;
        const uint32_t ty = in ? L.type[j][t] : b.hdr_type[(uint64_t)j * b.n + i];
        if (ty == type) {
            if (c == occ) return (int32_t)(in ? L.off[j][t] : b.hdr_off[(uint64_t)j * b.n + i]);
            c++;
        }
    }
    return -1;
}

// The same search over the chain's first 4 slots held in registers (chain_load's, branch-free
// selects: no loop, no LDS read); only a chain of more than 4 headers without a match among them
// goes on to find_lds.  (extract 19 getters 61.7 -> 57.8 us, set_fields + checksum 49.8 -> 40.4 us
// together with set_in_window's dword write-back, profiles/ab/r03p_rewrite_kernels.txt)
__device__ __forceinline__ int32_t find_pre(const ChainPre& c, const ChainLds& L, const BatchRef& b, uint64_t i,
                                            uint32_t t, uint32_t nh, uint32_t type, uint32_t occ) {
    int32_t r = -1;
    uint32_t cnt = 0;
#pragma unroll
    for (uint32_t j = 0; j < 4; j++) {
        const bool m = j < nh && c.ty[j] == type;
        r = (m && cnt == occ && r < 0) ? (int32_t)c.of[j] : r;
        cnt += m ? 1u : 0u;
    }
    if (r < 0 && nh > 4) r = find_lds(L, b, i, t, nh, type, occ);
    return r;
}

struct XSpec {
    pkt_field_spec_t f;
    uint64_t* values;
    uint8_t* found;
};
struct XParams {
    BatchRef b;
    uint32_t nspec;
    XSpec s[kMaxSpecs];
};

// Window of a lane's packet: its first NCH aligned 16-byte chunks, in LDS at an odd dword stride
// (per-lane dword reads conflict-free); bytes past it come from global memory (PacketView).  NCH =
// 4 for fixed-stride batches of <= 64-byte slots (a fifth chunk would be the next packet's), else 5.

template <int NCH>
__global__ __launch_bounds__(kRwBlock) void extract_kernel(XParams p) {
    constexpr uint32_t kXstride = 4 * NCH + 1;  // dwords
    __shared__ ChainLds L;
    __shared__ uint32_t win[kRwBlock * kXstride];
    // The spec table in LDS: indexed by the loop counter, the kernel-argument copy is read with a
    // vector load and a full memory round trip per spec; from LDS it is one broadcast read.
    __shared__ XSpec S[kMaxSpecs];
    const uint32_t t = threadIdx.x, lane = t & 63u, wave0 = t & ~63u;
    const uint64_t i = (uint64_t)blockIdx.x * kRwBlock + t;
    const bool act = i < p.b.n;  // no early exit: the wave loads its windows together
    const uint64_t off = act ? pkt_off(p.b, i) : 0u;
    const uint64_t last16 = ((p.b.slab_len + 15) & ~(uint64_t)15) - 16;
    uint32_t* w = win + t * kXstride;
    // cooperative window loads, issued before the chain is staged so that both are in flight
    // together: the wave's 64 windows as 64*NCH (packet, chunk) pairs, pair 64k + lane in load k
    // (consecutive lanes, consecutive chunks of one packet, as in the parse kernel)
    uint4 v[NCH];
#pragma unroll
    for (uint32_t k = 0; k < (uint32_t)NCH; k++) {
        const uint32_t pid = 64u * k + lane, r = pid / (uint32_t)NCH, c = pid % (uint32_t)NCH;
        const uint64_t offr = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(off >> 32), (int)r, 64) << 32) |
                              (uint32_t)__shfl((int)(uint32_t)off, (int)r, 64);
        uint64_t a = (offr & ~(uint64_t)15) + 16u * c;
        a = a > last16 ? last16 : a;
        v[k] = *reinterpret_cast<const uint4*>(p.b.slab + a);
    }
    ChainPre cp{};
    if (act) cp = chain_load(p.b, i);
    XSpec xs{};
    if (t < p.nspec) xs = p.s[t];
    // every load above is in flight; now the LDS stores
    if (t < p.nspec) S[t] = xs;
#pragma unroll
    for (uint32_t k = 0; k < (uint32_t)NCH; k++) {
        const uint32_t pid = 64u * k + lane, r = pid / (uint32_t)NCH, c = pid % (uint32_t)NCH;
        uint32_t* wr = win + (wave0 + r) * kXstride + 4 * c;
        wr[0] = v[k].x, wr[1] = v[k].y, wr[2] = v[k].z, wr[3] = v[k].w;
    }
    const uint32_t nh = act ? chain_store(p.b, i, t, L, cp) : 0u;
    __syncthreads();  // the spec table (and every wave's windows)
    if (!act) return;
    PacketView pv;
    pv.lw = reinterpret_cast<const uint8_t*>(w);
    pv.slab = p.b.slab;
    pv.off = off;
    pv.last4 = ((p.b.slab_len + 15) & ~(uint64_t)15) - 4;
    pv.shift = (uint32_t)(off & 15);
    pv.win_lo = 0;
    pv.win_end = 16u * NCH - pv.shift;
    pv.len = 0xFFFFFFFFu;  // (le() does not use it)
    uint32_t last_ty = 0xFFFFFFFFu, last_occ = 0;
    int32_t ho = -1;
    for (uint32_t s = 0; s < p.nspec; s++) {  // uniform
        const pkt_field_spec_t sp = S[s].f;
        if (sp.hdr_type != last_ty || sp.occurrence != last_occ) {  // consecutive specs of one header: one search
            ho = find_pre(cp, L, p.b, i, t, nh, sp.hdr_type, sp.occurrence);
            last_ty = sp.hdr_type;
            last_occ = sp.occurrence;
        }
        uint64_t v = 0;
        const uint32_t start = sp.start, end = sp.end, wd = end - start + 1;
        // bits [s2..end] hold the low 64 bits of the field; bit_range's release-build shifts
        // then keep the low (w mod 64, or 64) of them (headers.rs:262, Q8)
        const uint32_t s2 = wd > 64 ? end - 63 : start;
        const uint32_t b0 = s2 >> 3, b1 = end >> 3;  // <= 9 bytes
        const uint32_t rel = ho >= 0 ? (uint32_t)ho + b0 : 0u;
        const uint32_t nb = b1 - b0 + 1;
        // When every lane of the wave that has the header holds bytes rel .. rel + 11 in its window
        // (the common case), three straight LDS dword reads; else le() per lane (window or memory):
        // 19 getters 59.3 -> 54.9 us (profiles/ab/r03z_extract_uniform_window.txt).
        uint32_t x0, x1, x8;
        if (!__ballot(ho >= 0 && rel + 12u > pv.win_end)) {  // uniform
            const uint32_t wb = rel + pv.shift, k = wb >> 2, sh = wb & 3;
            const uint32_t d0 = w[k], d1 = w[k + 1], d2 = w[k + 2];
            x0 = __builtin_amdgcn_alignbyte(d1, d0, sh);
            x1 = __builtin_amdgcn_alignbyte(d2, d1, sh);
            x8 = d2 >> (8u * sh);
        } else {
            x0 = ho >= 0 ? pv.le(rel, 4) : 0u;
            x1 = ho >= 0 ? pv.le(rel + 4, 4) : 0u;
            x8 = (ho >= 0 && nb == 9) ? pv.le(rel + 8, 1) : 0u;
        }
        if (ho >= 0) {
            // bytes b0.. as big-endian: 8 in hi, the 9th (if any) in the top byte of x2
            const uint64_t hi = ((uint64_t)__builtin_bswap32(x0) << 32) | __builtin_bswap32(x1);
            const uint32_t ninth = nb == 9 ? x8 & 0xFFu : 0u;
            // value = bytes b0..b1 as a big-endian integer, shifted right by the trailing bits
            const uint32_t r = 7 - (end & 7);
            uint64_t acc, top;
            if (nb == 9) { acc = (hi << 8) | ninth; top = hi >> 56; }
            else { acc = hi >> (8 * (8 - nb)); top = 0; }
            uint64_t val = r ? ((acc >> r) | (top << (64 - r))) : acc;
            const uint32_t w2 = wd > 64 ? (wd & 63) : wd;
            if (w2 != 0 && w2 < 64) val &= (1ull << w2) - 1;
            v = val;
        }
        // non-temporal getter output columns: 19 getters 65.5 -> 62.4 us (profiles/ab/r02xnt_extract_nt.txt)
        __builtin_nontemporal_store(v, S[s].values + i);
        if (S[s].found) __builtin_nontemporal_store((uint8_t)(ho >= 0 ? 1 : 0), S[s].found + i);
    }
}

struct TParams {
    BatchRef b;
    const uint8_t* status;
    const uint16_t* payload_off;
    const uint16_t* payload_len;
    const uint32_t* hdr_mask;  // optional: rules out Q2 without reading the slot rows
    uint8_t* dst;
    uint64_t dst_len;
    const uint64_t* dst_offsets;
    uint32_t* out_len;
    // the window path (tv_window_kernel, below): *overlap == epoch when the batch is not for it
    const uint32_t* overlap;  // device word (tv_overlap_kernel stores the call's epoch there)
    uint32_t epoch;
    bool win;                 // tv_window_kernel runs too: to_vec_kernel copies only when *overlap == epoch
};

// An indexed batch written into its own layout whose records are in order with no 16-byte chunk
// shared by two of them (a capture: the 16-byte record headers lie between them) goes to
// tv_window_kernel (below); tv_overlap_kernel decides per batch, on the device.
constexpr uint32_t kTvWin = 4096;  // destination bytes per wave of tv_window_kernel

constexpr uint64_t kTvMaxWin = 128;  // windows one record (+ the gap before it) may span (a pcap
                                     // record is at most 256 KiB + 16 B: 65); more goes to to_vec_kernel

// Does any 16-byte chunk hold bytes of two records (or a record lie out of order)?  One pass over
// the index (12 B/record); if not, the pass also leaves tv_window_kernel's table: first[w] = the
// first record ending past byte kTvWin * w, i.e. record i for the windows starting in
// [end(i - 1), end(i)), written by pair (i - 1, i) (the windows before end(0) and from end(n - 1)
// on are the window kernel's to know: both ends go beside the flag).  A record past the slab's end,
// or one spanning more than kTvMaxWin windows, also sends the batch to to_vec_kernel.
__global__ __launch_bounds__(256) void tv_overlap_kernel(const uint64_t* __restrict__ offs, const uint32_t* __restrict__ lens,
                                                         uint64_t n, uint32_t* flag, uint32_t epoch,
                                                         uint32_t* __restrict__ first, uint64_t nwin, uint64_t slab_len) {
    const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;  // pairs (i - 1, i)
    bool bad = false;
    if (i < n) {
        const uint64_t o1 = offs[i], e1 = o1 + lens[i];
        bad = e1 > slab_len || lens[i] == 0;  // (an empty record has no window to write its out_len)
        if (i == 0 || i == n - 1) reinterpret_cast<uint64_t*>(flag + 2)[i == 0 ? 0 : 1] = e1;
        if (i >= 1) {
            const uint64_t o0 = offs[i - 1], l0 = lens[i - 1], e0 = o0 + l0;
            const bool pb = l0 == 0 || ((e0 - 1) >> 4) >= (o1 >> 4);
            bad |= pb;
            if (!pb) {
                const uint64_t w0 = (e0 + kTvWin - 1) / kTvWin;
                uint64_t w1 = (e1 + kTvWin - 1) / kTvWin;
                w1 = w1 < nwin ? w1 : nwin;
                if (w1 > w0 + kTvMaxWin) bad = true;
                else
                    for (uint64_t w = w0; w < w1; w++) first[w] = (uint32_t)i;
            }
        }
    }
    // (a plain vector store of the call's epoch, no reset before the call: a word left by an
    // older call holds another epoch)
    if (__ballot(bad) && (threadIdx.x & 63u) == 0) __hip_atomic_store(flag, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// bytes [lo, hi) of the 16-byte chunk at ca from o, the rest from d (the destination's own bytes)
__device__ __forceinline__ void merge_chunk(uint64_t ca, uint64_t lo, uint64_t hi, const uint32_t (&o)[4],
                                            uint32_t (&d)[4]) {
    const uint32_t a = (uint32_t)(lo - ca), z = (uint32_t)(hi - ca);  // 0 <= a < z <= 16
#pragma unroll
    for (int j = 0; j < 4; j++) {
        // byte b of dword j is in [a, z) iff a <= 4j + b < z
        const int32_t s0 = (int32_t)a - 4 * j, s1 = (int32_t)z - 4 * j;
        const uint32_t m0 = s0 <= 0 ? ~0u : (s0 >= 4 ? 0u : ~0u << (8 * s0));
        const uint32_t m1 = s1 >= 4 ? ~0u : (s1 <= 0 ? 0u : ~0u >> (8 * (4 - s1)));
        const uint32_t m = m0 & m1;
        d[j] = (o[j] & m) | (d[j] & ~m);
    }
}

__device__ __forceinline__ void put_byte(const TParams& p, uint64_t q, uint32_t v) {
    if (q < p.dst_len) p.dst[q] = (uint8_t)v;
}

// Store the bytes [lo, hi) of the 16-byte chunk at base + ca (o = its four little-endian dwords),
// nothing at or past `cap`: one 16-byte store when the chunk is whole, else whole dwords where
// covered and bytes at the edges.
__device__ __forceinline__ void store_chunk(uint8_t* base, uint64_t cap, uint64_t ca, const uint32_t (&o)[4],
                                            uint64_t lo, uint64_t hi) {
    if (lo == ca && hi == ca + 16 && ca + 16 <= cap) {
        *reinterpret_cast<uint4*>(base + ca) = make_uint4(o[0], o[1], o[2], o[3]);
        return;
    }
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const uint64_t a = ca + 4u * j;
        if (a >= lo && a + 4 <= hi && a + 4 <= cap) {
            *reinterpret_cast<uint32_t*>(base + a) = o[j];
        } else {
#pragma unroll
            for (int b = 0; b < 4; b++)
                if (a + b >= lo && a + b < hi && a + b < cap) base[a + b] = (uint8_t)(o[j] >> (8 * b));
        }
    }
}

// GRE option header types: two or more of them in one list is the only way the list order can
// differ from wire order (Q2, fast.rs:154-163)
constexpr uint32_t kGreOptMask = (1u << PKT_HDR_GRE_CHKSUM_OFFSET) | (1u << PKT_HDR_GRE_SEQUENCE_NUM) | (1u << PKT_HDR_GRE_KEY);

// Store the bytes [lo, hi) of a head / tail chunk (o = its dwords) below `cap`: the whole dwords
// it covers, then at most a byte and a short at each edge (8 store instructions, not one per
// byte); a range inside one dword goes byte by byte.
__device__ __forceinline__ void store_edge_chunk(uint8_t* base, uint64_t cap, uint64_t ca, const uint32_t (&o)[4],
                                                 uint64_t lo, uint64_t hi) {
    const uint64_t u4 = (lo + 3) & ~(uint64_t)3, d4 = hi & ~(uint64_t)3;
    if (u4 > d4) {  // within one dword
        const uint32_t v = o[((lo - ca) >> 2) & 3];
        for (uint64_t a = lo; a < hi; a++)
            if (a < cap) base[a] = (uint8_t)(v >> (8 * (a & 3)));
        return;
    }
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const uint64_t a = ca + 4u * j;
        if (a >= u4 && a + 4 <= d4 && a + 4 <= cap) *reinterpret_cast<uint32_t*>(base + a) = o[j];
    }
    if (lo < u4) {  // head: bytes lo .. u4-1 of dword (lo - ca) / 4
        const uint32_t v = o[((lo - ca) >> 2) & 3];
        uint64_t a = lo;
        if ((a & 1) && a < cap) base[a] = (uint8_t)(v >> (8 * (a & 3)));
        a += a & 1;
        if (a < u4 && a + 2 <= cap) *reinterpret_cast<uint16_t*>(base + a) = (uint16_t)(v >> 16);
    }
    if (d4 < hi) {  // tail: bytes d4 .. hi-1 of dword (d4 - ca) / 4
        const uint32_t v = o[((d4 - ca) >> 2) & 3];
        const uint32_t m = (uint32_t)(hi - d4);
        if ((m & 2) && d4 + 2 <= cap) *reinterpret_cast<uint16_t*>(base + d4) = (uint16_t)v;
        if ((m & 1) && d4 + (m & 2) < cap) base[d4 + (m & 2)] = (uint8_t)(v >> (8 * (m & 2)));
    }
}

// The source bytes of destination chunk ca of a packet copied from s to d (dwords o): one aligned
// load when source and destination share their alignment, else two and a funnel shift.
__device__ __forceinline__ void load_src_chunk(const BatchRef& b, uint64_t last16, uint64_t s, uint64_t d,
                                               uint64_t ca, uint32_t (&o)[4]) {
    if (((s ^ d) & 15) == 0) {
        uint64_t a = ca - d + s;
        a = a > last16 ? last16 : a;
        const uint4 v = *reinterpret_cast<const uint4*>(b.slab + a);
        o[0] = v.x, o[1] = v.y, o[2] = v.z, o[3] = v.w;
        return;
    }
    // source of destination byte ca: B = ca - d + s (below 0 only for bytes before the packet,
    // which are not stored)
    const int64_t B = (int64_t)(ca - d) + (int64_t)s;
    const int64_t A = B & ~(int64_t)15;
    uint64_t a0 = A < 0 ? 0 : (uint64_t)A, a1 = a0 + 16;
    a0 = a0 > last16 ? last16 : a0;
    a1 = a1 > last16 ? last16 : a1;
    const uint4 v0 = *reinterpret_cast<const uint4*>(b.slab + a0);
    const uint4 v1 = *reinterpret_cast<const uint4*>(b.slab + a1);
    const uint32_t sh = (uint32_t)(B - A), q = sh >> 2, r = sh & 3;
    const uint32_t x[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const uint32_t lo_w = q == 0 ? x[j] : q == 1 ? x[j + 1] : q == 2 ? x[j + 2] : x[j + 3];
        const uint32_t hi_w = q == 0 ? x[j + 1] : q == 1 ? x[j + 2] : q == 2 ? x[j + 3] : x[j + 4];
        o[j] = __builtin_amdgcn_alignbyte(hi_w, lo_w, r);
    }
}

constexpr uint32_t kTvMapChunks = 2048;  // chunks per wave the start map covers (32 KiB of output)

// Packet i's to_vec length and whether it is the packet's bytes [0, len) (ident); ok = parsed.
__device__ __forceinline__ void tv_meta(const TParams& p, uint64_t i, uint32_t& ok, uint32_t& ident, uint32_t& len) {
    // the four column reads issued together (no branch between them)
    const uint32_t stt = p.status[i], po = p.payload_off[i], pl = p.payload_len[i];
    const uint32_t hm = p.hdr_mask ? p.hdr_mask[i] : kGreOptMask;
    ok = stt == PKT_OK;
    ident = 1;
    len = 0;
    if (!ok) return;
    // at most one GRE option type in the list: headers lie back to back in list order, so the
    // list covers exactly [0, payload_off) and to_vec is the packet's bytes [0, len)
    const bool sure = p.hdr_mask && __builtin_popcount(hm & kGreOptMask) <= 1;
    uint32_t pos = po;
    if (!sure) {
        uint32_t nh = p.b.n_hdrs[i];
        nh = nh > PKT_MAX_HDRS ? PKT_MAX_HDRS : nh;
        pos = 0;
        for (uint32_t j = 0; j < nh; j++) {  // identity iff every header sits where the list puts it
            const uint32_t ty = p.b.hdr_type[(uint64_t)j * p.b.n + i];
            ident &= p.b.hdr_off[(uint64_t)j * p.b.n + i] == pos;
            pos += ty < PKT_HDR_COUNT ? kHdrSize[ty] : 0;
        }
        ident &= po == pos;
    }
    len = pos + pl;
}

// A Q2 packet (list order != wire order) by the whole wave: output byte q (lane q mod 64) comes
// from the list entry covering it — header slices, then the payload.
__device__ void tv_gather(const TParams& p, uint64_t ik, uint64_t s, uint64_t d, uint32_t L, uint32_t lane) {
    uint32_t nh = p.b.n_hdrs[ik];
    nh = nh > PKT_MAX_HDRS ? PKT_MAX_HDRS : nh;
    for (uint32_t q = lane; q < L; q += 64u) {
        uint32_t pos = 0, from = 0xFFFFFFFFu;
        for (uint32_t j = 0; j < nh; j++) {
            const uint32_t ty = p.b.hdr_type[(uint64_t)j * p.b.n + ik];
            const uint32_t sz = ty < PKT_HDR_COUNT ? kHdrSize[ty] : 0;
            if (from == 0xFFFFFFFFu && q < pos + sz) from = p.b.hdr_off[(uint64_t)j * p.b.n + ik] + (q - pos);
            pos += sz;
        }
        if (from == 0xFFFFFFFFu) from = p.payload_off[ik] + (q - pos);
        put_byte(p, d + q, p.b.slab[s + from]);
    }
}

__global__ __launch_bounds__(kRwBlock) void to_vec_kernel(TParams p) {
    const uint32_t lane = threadIdx.x & 63u;
    // wave-uniform values through readfirstlane (the compiler cannot tell threadIdx.x & ~63 is)
    const uint64_t base = ((uint64_t)blockIdx.x * kRwBlock +
                           __builtin_amdgcn_readfirstlane(threadIdx.x & ~63u));  // wave's first packet
    const uint64_t i = base + lane;
    if (p.win && __builtin_amdgcn_readfirstlane(*p.overlap) != p.epoch) return;  // tv_window_kernel copies
    // ---- per-lane metadata of packet i (coalesced column reads)
    uint64_t src = 0, dst = 0;
    uint32_t len = 0, ident = 1, ok = 0;
    if (i < p.b.n) {
        src = pkt_off(p.b, i);
        dst = p.dst_offsets ? p.dst_offsets[i] : src;
        tv_meta(p, i, ok, ident, len);
        if (p.out_len) p.out_len[i] = ok ? len : 0u;
    }
    // ---- identity packets: the wave's packets as ONE list of 16-byte destination chunks (a
    // packet's chunks are consecutive, packets in lane order), lane j copying chunks j, j+64, ...:
    // a wave-instruction writes 64 consecutive chunks whatever the packet lengths (records of a
    // capture lie back to back, so mostly 1 KiB of contiguous destination)
    const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    __shared__ uint32_t s_pre[kRwBlock / 64][65];
    __shared__ uint64_t s_src[kRwBlock / 64][64], s_dst[kRwBlock / 64][64];
    __shared__ uint32_t s_len[kRwBlock / 64][64];
    __shared__ uint64_t s_map[kRwBlock / 64][kTvMapChunks / 64];
    __shared__ uint64_t s_csrc[kRwBlock / 64][64], s_cdst[kRwBlock / 64][64];
    __shared__ uint32_t s_clen[kRwBlock / 64][64], s_cpre[kRwBlock / 64][64];
    const bool flat = ok && ident && len > 0;
    const uint32_t ch = flat ? (uint32_t)(((dst & 15) + len + 15) >> 4) : 0u;
    uint32_t incl = ch;  // inclusive scan over the wave
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) {
        const uint32_t t = (uint32_t)__shfl_up((int)incl, (unsigned)m, 64);
        if (lane >= (uint32_t)m) incl += t;
    }
    const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    s_pre[w][lane] = incl - ch;
    if (lane == 63) s_pre[w][64] = total;
    s_src[w][lane] = src;
    s_dst[w][lane] = dst;
    s_len[w][lane] = len;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint64_t last16 = ((p.b.slab_len + 15) & ~(uint64_t)15) - 16;
    // Chunk -> packet without a search: bit g of the wave's start map is set iff a packet's first
    // chunk is g, and the flat packets' (src, dst, len, pre) are stored compacted by rank, so chunk
    // g = 64 r + lane belongs to rank (starts before round r) + (starts at or below g within the
    // round's 64-bit word) - 1: one broadcast LDS read and a v_mbcnt per round instead of the
    // per-lane chain of dependent LDS compares (C2 30.8 -> 28.3 us; C4 unchanged,
    // profiles/ab/r03p_rewrite_kernels.txt).  Waves of more than kTvMapChunks chunks keep the search.
    const bool use_map = total <= kTvMapChunks;  // uniform
    if (use_map) {
        if (lane < kTvMapChunks / 64) s_map[w][lane] = 0;
        const uint64_t fm = __ballot(ch != 0);
        const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(fm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)fm, 0u));
        if (ch) {
            s_csrc[w][rank] = src;
            s_cdst[w][rank] = dst;
            s_clen[w][rank] = len;
            s_cpre[w][rank] = incl - ch;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (ch) {
            const uint32_t g0 = incl - ch;
            atomicOr(reinterpret_cast<uint32_t*>(s_map[w]) + (g0 >> 5), 1u << (g0 & 31u));
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    uint32_t run = 0;  // starts in the rounds before the one being located (uniform)
    // A wave whose 64 outputs lie back to back in the destination (a fixed-stride slab of whole
    // slots, or packed outputs) stores its whole chunks non-temporally: C2 33.7 -> 30.8 us, C4
    // packed 119 -> 102 us; with gaps between the outputs (a pcap's record headers left untouched)
    // the partial edge chunks share those lines and plain stores are faster (142 vs 147 us)
    // (profiles/ab/r02nt2_nt_wide_stores.txt).
    const uint64_t nd_ = __shfl_down(dst, 1u, 64);
    const bool nflat = __shfl_down((int)flat, 1u, 64) != 0;
    const bool dense = __ballot(lane == 63 || (flat && nflat && dst + len == nd_)) == ~0ull;
    // One chunk per lane per round, software-pipelined by one round: the next round's load is
    // issued before this round's store (a store may alias the next chunk's source, so the
    // compiler keeps load -> store -> load otherwise: one memory round trip per round).  (Issuing
    // 4 or 8 rounds' loads ahead was slower: C2 45 / 141 vs 33 us, C4 135 / 422 vs 125 us — 120+
    // VGPRs halve the resident waves, profiles/ab/r02tv_to_vec_unroll.txt.)
    uint32_t k = 0;
    auto locate = [&](uint32_t g, uint64_t& ca, uint64_t& lo, uint64_t& hi, uint32_t (&o)[4]) {
        uint64_t s, d;
        uint32_t L, pre;
        if (use_map) {  // rounds are located in order, each once
            const uint64_t word = s_map[w][g >> 6];
            const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(word >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)word, 0u));
            const uint32_t r = run + below + (uint32_t)((word >> lane) & 1u) - 1u;
            run += (uint32_t)__builtin_popcountll(word);
            s = s_csrc[w][r], d = s_cdst[w][r], L = s_clen[w][r], pre = s_cpre[w][r];
        } else {
            while (s_pre[w][k + 1] <= g) k++;  // packets with no chunks are skipped (pre[64] = total > g)
            s = s_src[w][k], d = s_dst[w][k], L = s_len[w][k], pre = s_pre[w][k];
        }
        ca = (d & ~(uint64_t)15) + 16u * (g - pre);  // destination chunk
        load_src_chunk(p.b, last16, s, d, ca, o);
        lo = ca > d ? ca : d;
        hi = ca + 16 < d + L ? ca + 16 : d + L;
    };
    auto put = [&](uint64_t ca, uint64_t lo, uint64_t hi, const uint32_t (&o)[4]) {
        if (lo == ca && hi == ca + 16 && ca + 16 <= p.dst_len) {
            if (dense) {
                typedef uint32_t v4u __attribute__((ext_vector_type(4)));
                __builtin_nontemporal_store(v4u{o[0], o[1], o[2], o[3]}, reinterpret_cast<v4u*>(p.dst + ca));
            } else {
                *reinterpret_cast<uint4*>(p.dst + ca) = make_uint4(o[0], o[1], o[2], o[3]);
            }
        } else {
            store_edge_chunk(p.dst, p.dst_len, ca, o, lo, hi);
        }
    };
    if (total <= 4u * 64u) {  // short waves (C2: 4 rounds): the plain loop is faster (33.7 vs 34.4 us)
        for (uint32_t g = lane; g < total; g += 64u) {
            uint64_t ca, lo, hi;
            uint32_t o[4];
            locate(g, ca, lo, hi, o);
            put(ca, lo, hi, o);
        }
    } else {  // C4: 142 vs 148 us in the input's layout, 124 vs 138 us packed (two rounds ahead:
              // 141 / 108 vs 142 / 105 us, round 3, profiles/ab/r03g_to_vec_lookahead2.txt)
        uint64_t ca = 0, lo = 0, hi = 0;
        uint32_t o[4] = {0, 0, 0, 0};
        locate(lane, ca, lo, hi, o);  // lane < 256 < total
        for (uint32_t g = lane; g < total; g += 64u) {
            uint64_t ca1 = 0, lo1 = 0, hi1 = 0;
            uint32_t o1[4] = {0, 0, 0, 0};
            if (g + 64u < total) locate(g + 64u, ca1, lo1, hi1, o1);
            put(ca, lo, hi, o);
            ca = ca1, lo = lo1, hi = hi1;
            o[0] = o1[0], o[1] = o1[1], o[2] = o1[2], o[3] = o1[3];
        }
    }
    // ---- Q2 packets (two or more GRE options), one at a time by the whole wave: output byte q
    // (lane q mod 64) comes from the list entry covering it — header slices, then the payload
    for (uint64_t q2 = __ballot(ok && !ident); q2; q2 &= q2 - 1) {  // uniform
        const uint32_t kk = (uint32_t)__builtin_ctzll(q2);
        tv_gather(p, base + kk, s_src[w][kk], s_dst[w][kk], s_len[w][kk], lane);
    }
}

// ---- to_vec in a capture's own layout, by destination window.  An indexed batch written to
// dst_offsets == its own offsets whose records are in order with no 16-byte chunk holding bytes of
// two of them (tv_overlap_kernel: a capture, whose 16-byte record headers lie between the records)
// is copied as the slab itself: wave w owns destination bytes [4096 w, 4096 (w + 1)) — 256 chunks,
// four per lane (chunks lane, lane + 64, ..), all four loads in flight before the first store —
// and finds which record owns each chunk from a 256-bit map of the record starts in the window
// (rank = starts at or below the chunk, as in to_vec_kernel's map).  Every chunk with bytes of a
// copied record is one 16-byte store: whole chunks straight from the source, the chunks a record
// shares with the record headers beside it merged with the destination's own bytes (no other
// wave holds that chunk).  Where to_vec_kernel gives each wave 64 records' chunks as a chain of
// dependent rounds (~13 per wave at C4), here each wave has one round of independent loads.
// first[w] = the first record ending past byte 4096 w (tv_overlap_kernel); records starting in
// the window write out_len; a Q2 record (list order != wire order) is gathered byte by byte by the
// wave holding its start.
constexpr uint32_t kTvWinWords = kTvWin / 16 / 64;  // 64-bit words of the start map

__global__ __launch_bounds__(kRwBlock) void tv_window_kernel(TParams p, const uint32_t* __restrict__ first,
                                                             uint64_t nwin) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t w = (uint64_t)blockIdx.x * (kRwBlock / 64) + wv;
    if (w >= nwin) return;
    __shared__ uint64_t s_map[kRwBlock / 64][kTvWinWords];
    __shared__ uint64_t s_o[kRwBlock / 64][64];
    __shared__ uint32_t s_l[kRwBlock / 64][64];
    const uint64_t wa = w * kTvWin, we = wa + kTvWin;
    const uint64_t last16 = ((p.b.slab_len + 15) & ~(uint64_t)15) - 16;
    // The window's source chunks need nothing but w (the destination is the source's layout):
    // their loads go first, in flight through the whole lookup below (a chunk outside every copied
    // record loads and drops its bytes; past the slab, the last chunk again).
    uint32_t sv[kTvWinWords][4];
#pragma unroll
    for (uint32_t q = 0; q < kTvWinWords; q++) {
        uint64_t a = wa + 16u * (64u * q + lane);
        a = a > last16 ? last16 : a;
        const uint4 v = *reinterpret_cast<const uint4*>(p.b.slab + a);
        sv[q][0] = v.x, sv[q][1] = v.y, sv[q][2] = v.z, sv[q][3] = v.w;
    }
    // the flag, end(0) and end(n - 1) (tv_overlap_kernel, same slot) and the window's table entry
    // in one round trip (first[w] is unset, and not used, for the windows before end(0))
    const uint64_t* ends = reinterpret_cast<const uint64_t*>(p.overlap + 2);
    const uint32_t flag = *p.overlap, fw = first[w];
    const uint64_t e0 = ends[0], en = ends[1];
    asm volatile("" ::"s"(flag), "s"(fw), "s"(e0), "s"(en));  // (keeps the four loads ahead of the branches)
    if (flag == p.epoch) return;  // records share chunks: to_vec_kernel
    // (every record lies inside the slab: tv_overlap_kernel)
    if (wa >= en) return;  // past the last record
    uint64_t i0 = wa < e0 ? 0u : fw;
    // 64 records at a time while they start inside the window: the first batch straight-line (a
    // loop header would wait for the source loads above), the rare further ones in a loop
    auto batch = [&](uint64_t i0) __attribute__((always_inline)) -> bool {
        const uint64_t i = i0 + lane;
        uint64_t o = ~0ull;
        uint32_t len = 0, md = 0;  // md: 1 = copied by chunks, 2 = gathered (Q2)
        bool sin = false;
        if (i < p.b.n) {
            // the record's start and its columns read together (those of records starting past
            // the window too: one round trip, not two)
            o = p.b.offsets[i];
            uint32_t ok = 0, ident = 1;
            tv_meta(p, i, ok, ident, len);
            if (o < we) {
                md = ok && len ? (ident ? 1u : 2u) : 0u;
                sin = o >= wa;
            } else {
                len = 0;
            }
        }
        if (lane < kTvWinWords) s_map[wv][lane] = 0;
        s_o[wv][lane] = o;
        s_l[wv][lane] = len | md << 30;  // len <= 2 * 65535
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const bool st = sin && o < we;  // starts at chunk (o - wa) / 16 of this window
        if (st) {
            const uint32_t g = (uint32_t)((o - wa) >> 4);
            atomicOr(reinterpret_cast<uint32_t*>(s_map[wv]) + (g >> 5), 1u << (g & 31u));
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // chunk g's record: lane (starts at or below g) - s0, s0 = 1 when the batch's first record
        // starts in the window (chunks before it are not the batch's), else it began before
        const uint32_t s0 = (uint32_t)(__ballot(st) & 1ull);
        uint32_t run = 0;
        uint32_t az[kTvWinWords];  // the record's bytes [a, z) of chunk q (a | z << 8; 0 = none)
        uint32_t dv[kTvWinWords][4];
#pragma unroll
        for (uint32_t q = 0; q < kTvWinWords; q++) {
            const uint64_t word = s_map[wv][q];
            const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(word >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)word, 0u));
            const int32_t r = (int32_t)(run + below + (uint32_t)((word >> lane) & 1u)) - (int32_t)s0;
            run += (uint32_t)__builtin_popcountll(word);
            const uint64_t ca = wa + 16u * (64u * q + lane);
            az[q] = 0;
            if (r >= 0 && r < 64) {
                const uint64_t ro = s_o[wv][r];
                const uint32_t rl = s_l[wv][r];
                if ((rl >> 30) == 1u) {
                    const uint64_t re = ro + (rl & 0x3FFFFFFFu);
                    const uint64_t lo = ca > ro ? ca : ro, hi = ca + 16 < re ? ca + 16 : re;
                    if (lo < hi) az[q] = (uint32_t)(lo - ca) | (uint32_t)(hi - ca) << 8;
                }
            }
            // unconditional (no branch joins a loaded value: a join would wait for it, the
            // chunks' loads going one at a time): a chunk that is not an edge reloads its
            // source (same address: no new HBM traffic)
            const uint64_t a = ca > last16 ? last16 : ca;
            const uint8_t* dp = az[q] && az[q] != (16u << 8) && ca + 16 <= p.dst_len ? p.dst + ca : p.b.slab + a;
            const uint4 u = *reinterpret_cast<const uint4*>(dp);
            dv[q][0] = u.x, dv[q][1] = u.y, dv[q][2] = u.z, dv[q][3] = u.w;
        }
#pragma unroll
        for (uint32_t q = 0; q < kTvWinWords; q++) {
            if (!az[q]) continue;
            const uint64_t ca = wa + 16u * (64u * q + lane);
            const uint64_t lo = ca + (az[q] & 0xFFu), hi = ca + (az[q] >> 8);
            if (ca + 16 > p.dst_len) {  // the destination's last partial chunk
                for (uint64_t x = lo; x < hi; x++) put_byte(p, x, sv[q][(x - ca) >> 2] >> (8 * (x & 3)));
            } else if (az[q] == (16u << 8)) {
                typedef uint32_t v4u __attribute__((ext_vector_type(4)));
                __builtin_nontemporal_store(v4u{sv[q][0], sv[q][1], sv[q][2], sv[q][3]}, reinterpret_cast<v4u*>(p.dst + ca));
            } else {
                merge_chunk(ca, lo, hi, sv[q], dv[q]);
                *reinterpret_cast<uint4*>(p.dst + ca) = make_uint4(dv[q][0], dv[q][1], dv[q][2], dv[q][3]);
            }
        }
        if (sin && p.out_len) p.out_len[i] = len;  // (0 when not parsed; after the chunks' loads)
        for (uint64_t q2 = __ballot(sin && md == 2u); q2; q2 &= q2 - 1) {  // uniform
            const uint32_t kk = (uint32_t)__builtin_ctzll(q2);
            tv_gather(p, i0 + kk, s_o[wv][kk], s_o[wv][kk], s_l[wv][kk] & 0x3FFFFFFFu, lane);
        }
        // all 64 began before the window's end: the next 64 may too
        return ((__ballot(o < we) >> 63) & 1ull) != 0;
    };
    if (i0 >= p.b.n) return;
    for (bool more = batch(i0); more && i0 + 64 < p.b.n; more = batch(i0)) {  // uniform
        i0 += 64;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
}

struct SSpec {
    pkt_field_spec_t f;
    const uint64_t* values;
};
struct SParams {
    BatchRef b;
    uint8_t* slab;
    uint32_t nspec;
    int32_t csum_occ;  // >= 0: refresh that IPv4 header's checksum after the setters
    SSpec s[kMaxSpecs];
};

// The packet's first NCH 16-byte chunks (from its 16-byte-aligned start) in LDS at an odd dword
// stride, as in the parse kernel (NCH as in extract_kernel).
constexpr uint32_t kPreVals = 4;  // setter values prefetched into registers

// One setter on a <= 64-bit field whose bytes start at byte x of the lane's LDS window: its <= 9
// bytes read as one 16-byte big-endian piece, set by one shift and mask, written back to LDS.
__device__ __forceinline__ void set_in_window(uint32_t* w, uint32_t x, uint32_t lsb, uint32_t msb, uint64_t v) {
    const uint32_t b0 = lsb >> 3, nb = (msb >> 3) - b0 + 1;
    const uint32_t k = x >> 2, sh = x & 3;
    const uint32_t d0 = w[k], d1 = w[k + 1], d2 = w[k + 2], d3 = w[k + 3], d4 = w[k + 4];
    U128 W{((uint64_t)__builtin_bswap32(__builtin_amdgcn_alignbyte(d1, d0, sh)) << 32) |
               __builtin_bswap32(__builtin_amdgcn_alignbyte(d2, d1, sh)),
           ((uint64_t)__builtin_bswap32(__builtin_amdgcn_alignbyte(d3, d2, sh)) << 32) |
               __builtin_bswap32(__builtin_amdgcn_alignbyte(d4, d3, sh))};
    put_bits(W, lsb - 8 * b0, msb - 8 * b0, msb - lsb + 1, v, 0);
    // back as the aligned dwords holding the field's bytes (at most 3: sh + nb <= 12), rebuilt from
    // W's little-endian dwords e_j (bytes x + 4j ..) by a funnel shift; the bytes around the field
    // are rewritten with the values just read (the lane's own window)
    const uint32_t e0 = __builtin_bswap32((uint32_t)(W.hi >> 32)), e1 = __builtin_bswap32((uint32_t)W.hi);
    const uint32_t e2 = __builtin_bswap32((uint32_t)(W.lo >> 32));
    const uint32_t em = sh ? d0 << (32 - 8 * sh) : 0u;  // top sh bytes = d0's bytes before x
    const uint32_t s4 = 4 - sh;
    const uint32_t n0 = sh ? __builtin_amdgcn_alignbyte(e0, em, s4) : e0;
    const uint32_t n1 = sh ? __builtin_amdgcn_alignbyte(e1, e0, s4) : e1;
    const uint32_t n2 = sh ? __builtin_amdgcn_alignbyte(e2, e1, s4) : e2;
    const uint32_t jl = (sh + nb - 1) >> 2;
    w[k] = n0;
    if (jl >= 1) w[k + 1] = n1;
    if (jl >= 2) w[k + 2] = n2;
}

template <int NCH>
__global__ __launch_bounds__(kRwBlock) void set_fields_kernel(SParams p) {
    constexpr uint32_t kSstride = 4 * NCH + 1;  // dwords
    __shared__ ChainLds L;
    __shared__ uint32_t win[kRwBlock * kSstride + 8];  // +8: the last lane's 16-byte over-read
    __shared__ SSpec S[kMaxSpecs];  // the spec table in LDS (as in extract_kernel)
    const uint32_t t = threadIdx.x, lane = t & 63u, wave0 = t & ~63u;
    const uint64_t i = (uint64_t)blockIdx.x * kRwBlock + t;
    const bool act = i < p.b.n;  // no early exit: the wave loads and stores windows together
    uint32_t plen = 0;
    uint64_t off = 0;
    if (act) {
        off = pkt_off(p.b, i);
        plen = p.b.lens ? p.b.lens[i] : p.b.stride;
        const uint64_t room = off < p.b.slab_len ? p.b.slab_len - off : 0;
        plen = (uint64_t)plen > room ? (uint32_t)room : plen;
    }
    // All loads first, in flight together: the windows (cooperative: the wave's 64 windows as
    // 64*NCH (packet, chunk) pairs, pair 64k + lane in load k, so each window comes from one or
    // two wave instructions, as in the parse kernel), the chain, the first kPreVals values (their
    // pointers are kernel arguments at constant indices: scalar loads) and the spec table.
    const uint64_t last16 = ((p.b.slab_len + 15) & ~(uint64_t)15) - 16;
    uint4 v[NCH];
#pragma unroll
    for (uint32_t k = 0; k < (uint32_t)NCH; k++) {
        const uint32_t pid = 64u * k + lane, r = pid / (uint32_t)NCH, c = pid % (uint32_t)NCH;
        const uint64_t offr = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(off >> 32), (int)r, 64) << 32) |
                              (uint32_t)__shfl((int)(uint32_t)off, (int)r, 64);
        uint64_t a = (offr & ~(uint64_t)15) + 16u * c;
        a = a > last16 ? last16 : a;
        v[k] = *reinterpret_cast<const uint4*>(p.b.slab + a);
    }
    ChainPre cp{};
    if (act) cp = chain_load(p.b, i);
    uint64_t vpre[kPreVals];
#pragma unroll
    for (uint32_t s = 0; s < kPreVals; s++) vpre[s] = (act && s < p.nspec) ? p.s[s].values[i] : 0u;
    SSpec ss{};
    if (t < p.nspec) ss = p.s[t];
    if (t < p.nspec) S[t] = ss;
#pragma unroll
    for (uint32_t k = 0; k < (uint32_t)NCH; k++) {
        const uint32_t pid = 64u * k + lane, r = pid / (uint32_t)NCH, c = pid % (uint32_t)NCH;
        uint32_t* w = win + (wave0 + r) * kSstride + 4 * c;
        w[0] = v[k].x, w[1] = v[k].y, w[2] = v[k].z, w[3] = v[k].w;
    }
    const uint32_t nh = act ? chain_store(p.b, i, t, L, cp) : 0u;
    __syncthreads();  // the spec table and the windows
    const uint32_t shift = (uint32_t)(off & 15);
    // window mode iff every field this packet sets is <= 64 bits and lies inside the window
    bool inwin = act;
    for (uint32_t s = 0; s < p.nspec && inwin; s++) {
        const pkt_field_spec_t sp = S[s].f;
        const int32_t ho = act ? find_pre(cp, L, p.b, i, t, nh, sp.hdr_type, sp.occurrence) : -1;
        if (ho >= 0 && (sp.end - sp.start >= 64 || shift + (uint32_t)ho + (sp.end >> 3) + 1 > 16u * NCH)) inwin = false;
    }
    uint32_t dirty = 0;  // window chunks holding a set byte
    // one setter (specs in order: overlapping ones act as sequential setters)
    auto apply = [&](uint32_t s, uint64_t v0) {
        const pkt_field_spec_t sp = S[s].f;
        const int32_t ho = find_pre(cp, L, p.b, i, t, nh, sp.hdr_type, sp.occurrence);
        if (ho < 0) return;
        const uint32_t lsb = sp.start, msb = sp.end;
        if (inwin) {
            const uint32_t x = shift + (uint32_t)ho + (lsb >> 3);
            set_in_window(win + t * kSstride, x, lsb, msb, v0);
            dirty |= ((2u << ((x + (msb >> 3) - (lsb >> 3)) >> 4)) - 1u) & ~((1u << (x >> 4)) - 1u);
            return;
        }
        if (msb - lsb < 64) {
            // outside the window: the same RMW on one 16-byte read of global memory, only the
            // field's bytes stored (byte stores: neighbours untouched)
            const uint32_t b0 = lsb >> 3, nb = (msb >> 3) - b0 + 1;
            const uint64_t A = off + (uint32_t)ho + b0;
            const uint32_t sh = (uint32_t)(A & 3);
            const uint32_t d0 = slab_dw(p.b, A), d1 = slab_dw(p.b, A + 4), d2 = slab_dw(p.b, A + 8);
            const uint32_t d3 = slab_dw(p.b, A + 12), d4 = slab_dw(p.b, A + 16);
            U128 W{((uint64_t)__builtin_bswap32(__builtin_amdgcn_alignbyte(d1, d0, sh)) << 32) |
                       __builtin_bswap32(__builtin_amdgcn_alignbyte(d2, d1, sh)),
                   ((uint64_t)__builtin_bswap32(__builtin_amdgcn_alignbyte(d3, d2, sh)) << 32) |
                       __builtin_bswap32(__builtin_amdgcn_alignbyte(d4, d3, sh))};
            put_bits(W, lsb - 8 * b0, msb - 8 * b0, msb - lsb + 1, v0, 0);
            uint8_t* h = p.slab + A;
            for (uint32_t j = 0; j < nb; j++)
                h[j] = (uint8_t)((j < 8 ? W.hi >> (56 - 8 * j) : W.lo >> (120 - 8 * j)) & 0xFFu);
            return;
        }
        // wider fields (IPv6 addresses): set_bit_range a byte at a time from the field's last byte
        // backwards; bits above the value's 64 become 0
        uint8_t* h = p.slab + off + (uint32_t)ho;
        uint64_t v = v0;
        int32_t b = (int32_t)msb;
        while (b >= (int32_t)lsb) {
            const uint32_t byte = (uint32_t)b >> 3;
            const int32_t lo = max((int32_t)lsb, (int32_t)(byte * 8));
            const uint32_t nbit = (uint32_t)(b - lo + 1);
            const uint32_t shf = 7 - ((uint32_t)b & 7);
            const uint32_t m = (((1u << nbit) - 1u) << shf) & 0xFFu;
            const uint32_t bits = ((uint32_t)(v & ((1ull << nbit) - 1ull)) << shf) & 0xFFu;
            h[byte] = (uint8_t)(nbit == 8 ? bits : ((h[byte] & ~m) | bits));
            v = nbit >= 64 ? 0 : (v >> nbit);
            b = lo - 1;
        }
    };
    if (act) {
        // the first kPreVals values are loaded in flight together with the windows; the rest per spec
#pragma unroll
        for (uint32_t s = 0; s < kPreVals; s++)
            if (s < p.nspec) apply(s, vpre[s]);
        for (uint32_t s = kPreVals; s < p.nspec; s++) apply(s, S[s].values[i]);
    }
    // Packet::ipv4_checksum refresh of the csum_occ-th IPv4 header (ipv4_update_kernel's sum) after
    // the setters: header dwords inside the window from LDS, past it from global memory (bytes only
    // this lane wrote); the two checksum bytes into LDS (dirty) or global memory likewise.
    if (p.csum_occ >= 0 && act) {
        const int32_t ho = find_pre(cp, L, p.b, i, t, nh, PKT_HDR_IPV4, (uint32_t)p.csum_occ);
        if (ho >= 0) {
            const uint32_t x = shift + (uint32_t)ho, x0 = x & ~3u, sh = x & 3u;
            const uint64_t a0 = off & ~(uint64_t)15;  // window byte q <-> slab byte a0 + q
            const uint32_t* w = win + t * kSstride;
            uint32_t d[6];
            if (inwin && x0 + 24u <= 16u * NCH) {  // the whole header in the window (the common case)
#pragma unroll
                for (int k = 0; k < 6; k++) d[k] = w[(x0 >> 2) + k];
            } else {
#pragma unroll
                for (int k = 0; k < 6; k++) {
                    const uint32_t q = x0 + 4u * k;
                    d[k] = (inwin && q + 4 <= 16u * NCH) ? w[q >> 2] : slab_dw(p.b, a0 + q);
                }
            }
            uint32_t sum = 0;
#pragma unroll
            for (int k = 0; k < 5; k++) {
                const uint32_t v = __builtin_bswap32(__builtin_amdgcn_alignbyte(d[k + 1], d[k], sh));
                sum += (v >> 16) + (k == 2 ? 0u : (v & 0xFFFFu));  // bytes 10-11 (the checksum) skipped
            }
            sum = ((sum >> 16) + sum) & 0xFFFFu;  // packet.rs:102-104 (Q1)
            const uint32_t c = (~sum) & 0xFFFFu;
#pragma unroll
            for (uint32_t j = 0; j < 2; j++) {
                const uint32_t q = x + 10u + j;
                const uint8_t byte = (uint8_t)(j ? c : c >> 8);
                if (inwin && q < 16u * NCH) {
                    reinterpret_cast<uint8_t*>(win + t * kSstride)[q] = byte;
                    dirty |= 1u << (q >> 4);
                } else {
                    p.slab[a0 + q] = byte;
                }
            }
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // write back the dirty chunks, the packet's own bytes only, with the pairs of the loads
#pragma unroll
    for (uint32_t k = 0; k < (uint32_t)NCH; k++) {
        const uint32_t pid = 64u * k + lane, r = pid / (uint32_t)NCH, c = pid % (uint32_t)NCH;
        const uint32_t dr = (uint32_t)__shfl((int)dirty, (int)r, 64);
        const uint64_t offr = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(off >> 32), (int)r, 64) << 32) |
                              (uint32_t)__shfl((int)(uint32_t)off, (int)r, 64);
        const uint32_t plr = (uint32_t)__shfl((int)plen, (int)r, 64);
        if ((dr >> c) & 1u) {
            const uint64_t ca = (offr & ~(uint64_t)15) + 16u * c;
            const uint32_t* w = win + (wave0 + r) * kSstride + 4 * c;
            const uint32_t o[4] = {w[0], w[1], w[2], w[3]};
            store_chunk(p.slab, p.b.slab_len, ca, o, ca > offr ? ca : offr,
                        ca + 16 < offr + plr ? ca + 16 : offr + plr);
        }
    }
}

__global__ __launch_bounds__(kRwBlock) void ipv4_update_kernel(BatchRef b, uint8_t* slab, uint32_t occurrence) {
    __shared__ ChainLds L;
    const uint32_t t = threadIdx.x;
    const uint64_t i = (uint64_t)blockIdx.x * kRwBlock + t;
    if (i >= b.n) return;
    const uint32_t nh = stage_chain(b, i, t, L);
    const int32_t ho = find_lds(L, b, i, t, nh, PKT_HDR_IPV4, occurrence);
    if (ho < 0) return;
    const uint64_t a = pkt_off(b, i) + (uint32_t)ho;
    const uint32_t sh = (uint32_t)(a & 3);
    uint32_t d[6];
#pragma unroll
    for (int k = 0; k < 6; k++) d[k] = slab_dw(b, a + 4u * k);
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < 5; k++) {
        const uint32_t w = __builtin_bswap32(__builtin_amdgcn_alignbyte(d[k + 1], d[k], sh));
        s += (w >> 16) + (k == 2 ? 0u : (w & 0xFFFFu));  // bytes 10-11 (the checksum) skipped
    }
    s = ((s >> 16) + s) & 0xFFFFu;  // packet.rs:102-104 (Q1)
    const uint32_t c = (~s) & 0xFFFFu;
    slab[a + 10] = (uint8_t)(c >> 8);
    slab[a + 11] = (uint8_t)c;
}

// n copies of one packet at a fixed stride, 16 bytes per lane per step (slot-contiguous).
__global__ __launch_bounds__(kRwBlock) void broadcast_kernel(const uint8_t* src, uint32_t len, uint64_t n,
                                                             uint32_t stride, uint8_t* dst) {
    const uint64_t total = n * (uint64_t)stride;  // bytes, multiple of 16 (checked by the host)
    for (uint64_t q = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * 16; q < total;
         q += (uint64_t)gridDim.x * blockDim.x * 16) {
        const uint32_t o = (uint32_t)(q % stride);
        uint32_t w[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            uint32_t x = 0;
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const uint32_t ob = o + 4u * k + j;
                x |= (ob < len ? (uint32_t)src[ob] : 0u) << (8 * j);
            }
            w[k] = x;
        }
        *reinterpret_cast<uint4*>(dst + q) = make_uint4(w[0], w[1], w[2], w[3]);
    }
}

__global__ __launch_bounds__(kRwBlock) void ipv4_csum_kernel(const uint8_t* hdrs, uint32_t stride, uint64_t n,
                                                             uint16_t* out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint8_t* v = hdrs + i * (uint64_t)stride;
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < 20; k += 2)
        if (k != 10) s += ((uint32_t)v[k] << 8) | v[k + 1];
    s = ((s >> 16) + s) & 0xFFFFu;
    out[i] = (uint16_t)~s;
}

// Fixed-stride batches of <= 64-byte, 16-byte-aligned slots: 4-chunk windows (the packet) instead of 5.
bool narrow_slots(const pkt_batch_t* b) { return !b->offsets && b->stride <= 64 && b->stride % 16 == 0; }

int batch_ref(pkt_ctx_t* ctx, const pkt_batch_t* b, const pkt_chain_t* chain, BatchRef& r) {
    if (!b->slab || !chain || !chain->n_hdrs || !chain->hdr_type || !chain->hdr_off)
        return fail(ctx, PKT_ERR_INVALID_ARG, "null slab/chain column");
    if (b->offsets && !b->lens) return fail(ctx, PKT_ERR_INVALID_ARG, "offsets without lens");
    if (!b->offsets && b->stride == 0) return fail(ctx, PKT_ERR_INVALID_ARG, "stride 0");
    r.slab = b->slab;
    r.slab_len = b->slab_len;
    r.offsets = b->offsets;
    r.lens = b->lens;
    r.stride = b->stride;
    r.n = b->n;
    r.n_hdrs = chain->n_hdrs;
    r.hdr_type = chain->hdr_type;
    r.hdr_off = chain->hdr_off;
    return PKT_SUCCESS;
}

bool bad_spec(const pkt_field_spec_t& f) {
    return f.hdr_type == 0 || f.hdr_type >= PKT_HDR_COUNT || f.end < f.start || f.end >= 8 * pkt_hdr_size(f.hdr_type);
}

unsigned grid_of(uint64_t n) { return (unsigned)((n + kRwBlock - 1) / kRwBlock); }

}  // namespace

extern "C" {

int pkt_extract_fields(pkt_ctx_t* ctx, const pkt_batch_t* b, const pkt_chain_t* chain,
                       const pkt_field_spec_t* specs, uint32_t nspec, uint64_t* const* values,
                       uint8_t* const* found, void* stream) {
    if (!ctx || !b || !chain || (nspec && (!specs || !values)))
        return fail(ctx, PKT_ERR_INVALID_ARG, "null argument");
    if (b->n == 0 || nspec == 0) return PKT_SUCCESS;
    XParams xp;
    int rc = batch_ref(ctx, b, chain, xp.b);
    if (rc) return rc;
    for (uint32_t s = 0; s < nspec; s++)
        if (bad_spec(specs[s]) || !values[s]) return fail(ctx, PKT_ERR_INVALID_ARG, "bad field spec");
    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) return hip_fail(ctx, e, "hipSetDevice");
    // specs grouped by (header, occurrence), so that the kernel searches the chain once per group;
    // the order is kept when two specs share an output array (the later one must win)
    std::vector<uint32_t> ord(nspec);
    for (uint32_t s = 0; s < nspec; s++) ord[s] = s;
    bool shared = false;
    for (uint32_t a = 0; a < nspec && !shared; a++)
        for (uint32_t c = a + 1; c < nspec && !shared; c++)
            shared = values[a] == values[c] || (found && found[a] && found[a] == found[c]);
    if (!shared)
        std::stable_sort(ord.begin(), ord.end(), [&](uint32_t x, uint32_t y) {
            return specs[x].hdr_type != specs[y].hdr_type ? specs[x].hdr_type < specs[y].hdr_type
                                                          : specs[x].occurrence < specs[y].occurrence;
        });
    for (uint32_t s0 = 0; s0 < nspec; s0 += kMaxSpecs) {  // one launch per 32 specs
        xp.nspec = std::min<uint32_t>(kMaxSpecs, nspec - s0);
        for (uint32_t k = 0; k < xp.nspec; k++) {
            const uint32_t q = ord[s0 + k];
            xp.s[k].f = specs[q];
            xp.s[k].values = values[q];
            xp.s[k].found = found ? found[q] : nullptr;
        }
        if (narrow_slots(b))
            hipLaunchKernelGGL(extract_kernel<4>, dim3(grid_of(b->n)), dim3(kRwBlock), 0, reinterpret_cast<hipStream_t>(stream), xp);
        else
            hipLaunchKernelGGL(extract_kernel<5>, dim3(grid_of(b->n)), dim3(kRwBlock), 0, reinterpret_cast<hipStream_t>(stream), xp);
        if ((e = hipGetLastError()) != hipSuccess) return hip_fail(ctx, e, "extract_kernel launch");
    }
    return PKT_SUCCESS;
}

int pkt_to_vec_batch(pkt_ctx_t* ctx, const pkt_batch_t* b, const pkt_out_t* parsed, uint8_t* dst,
                     uint64_t dst_len, const uint64_t* dst_offsets, uint32_t* out_len, void* stream) {
    if (!ctx || !b || !parsed) return fail(ctx, PKT_ERR_INVALID_ARG, "null argument");
    if (b->n == 0) return PKT_SUCCESS;
    if (!dst || !parsed->status || !parsed->payload_off || !parsed->payload_len)
        return fail(ctx, PKT_ERR_INVALID_ARG, "null slab/dst/chain column");
    TParams tp;
    pkt_chain_t ch{parsed->n_hdrs, parsed->hdr_type, parsed->hdr_off};
    int rc = batch_ref(ctx, b, &ch, tp.b);
    if (rc) return rc;
    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) return hip_fail(ctx, e, "hipSetDevice");
    tp.status = parsed->status;
    tp.payload_off = parsed->payload_off;
    tp.payload_len = parsed->payload_len;
    tp.hdr_mask = parsed->hdr_mask;
    tp.dst = dst;
    tp.dst_len = dst_len;
    tp.dst_offsets = dst_offsets;
    tp.out_len = out_len;
    tp.overlap = nullptr;
    tp.epoch = 0;
    tp.win = false;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (!dst_offsets && b->offsets && b->lens && b->n > 1 && b->n < 0xFFFFFFFFull && b->slab_len) {
        // does any 16-byte chunk hold bytes of two records?  (one pass over the index: 12 B/record)
        if (!ctx->tv_flag &&
            (e = hipMalloc(reinterpret_cast<void**>(&ctx->tv_flag), pkt_ctx::kTvFlags * pkt_ctx::kTvSlotWords * sizeof(uint32_t))) != hipSuccess)
            return hip_fail(ctx, e, "hipMalloc (to_vec flag)");
        uint32_t ep = ctx->tv_epoch + 1;
        ep = ep ? ep : 1;
        if (ep == 1) {  // first call, or 2^32 calls on: no word may hold the epochs to come
            if ((e = hipDeviceSynchronize()) != hipSuccess) return hip_fail(ctx, e, "hipDeviceSynchronize");
            if ((e = hipMemset(ctx->tv_flag, 0, pkt_ctx::kTvFlags * pkt_ctx::kTvSlotWords * sizeof(uint32_t))) != hipSuccess)
                return hip_fail(ctx, e, "hipMemset (to_vec flag)");
        }
        ctx->tv_epoch = ep;
        const uint32_t slot = ctx->tv_next++ % pkt_ctx::kTvFlags;
        uint32_t* flag = ctx->tv_flag + slot * pkt_ctx::kTvSlotWords;
        hipEvent_t& ev = ctx->tv_ev[slot];
        if (!ev && (e = hipEventCreateWithFlags(&ev, hipEventDisableTiming)) != hipSuccess)
            return hip_fail(ctx, e, "hipEventCreate (to_vec flag)");
        // the word's previous user (a call 256 calls ago, maybe on another stream) has read it
        if ((e = hipStreamWaitEvent(s, ev, 0)) != hipSuccess) return hip_fail(ctx, e, "hipStreamWaitEvent");
        // the window table: first[w] per 4 KiB window of the slab (records indexed by u32)
        const uint64_t nwin = (b->slab_len + kTvWin - 1) / kTvWin;
        if (!ctx->tv_win_ev && (e = hipEventCreateWithFlags(&ctx->tv_win_ev, hipEventDisableTiming)) != hipSuccess)
            return hip_fail(ctx, e, "hipEventCreate (to_vec windows)");
        if (nwin > ctx->tv_win_cap) {
            if (ctx->tv_win) {
                if ((e = hipEventSynchronize(ctx->tv_win_ev)) != hipSuccess) return hip_fail(ctx, e, "hipEventSynchronize");
                (void)hipFree(ctx->tv_win);
                ctx->tv_win = nullptr, ctx->tv_win_cap = 0;
            }
            if ((e = hipMalloc(reinterpret_cast<void**>(&ctx->tv_win), nwin * sizeof(uint32_t))) != hipSuccess)
                return hip_fail(ctx, e, "hipMalloc (to_vec windows)");
            ctx->tv_win_cap = nwin;
        }
        // the previous call's window kernel has read the table
        if ((e = hipStreamWaitEvent(s, ctx->tv_win_ev, 0)) != hipSuccess) return hip_fail(ctx, e, "hipStreamWaitEvent");
        hipLaunchKernelGGL(tv_overlap_kernel, dim3((unsigned)((b->n + 255) / 256)), dim3(256), 0, s, b->offsets,
                           b->lens, b->n, flag, ctx->tv_epoch, ctx->tv_win, nwin, b->slab_len);
        if ((e = hipGetLastError()) != hipSuccess) return hip_fail(ctx, e, "tv_overlap_kernel launch");
        tp.overlap = flag;
        tp.epoch = ctx->tv_epoch;
        tp.win = true;
        hipLaunchKernelGGL(tv_window_kernel, dim3((unsigned)((nwin + kRwBlock / 64 - 1) / (kRwBlock / 64))),
                           dim3(kRwBlock), 0, s, tp, (const uint32_t*)ctx->tv_win, nwin);
        if ((e = hipGetLastError()) != hipSuccess) return hip_fail(ctx, e, "tv_window_kernel launch");
        if ((e = hipEventRecord(ctx->tv_win_ev, s)) != hipSuccess) return hip_fail(ctx, e, "hipEventRecord");
    }
    hipLaunchKernelGGL(to_vec_kernel, dim3(grid_of(b->n)), dim3(kRwBlock), 0, reinterpret_cast<hipStream_t>(stream), tp);
    if ((e = hipGetLastError()) != hipSuccess) return hip_fail(ctx, e, "to_vec_kernel launch");
    if (tp.overlap && (e = hipEventRecord(ctx->tv_ev[(ctx->tv_next - 1) % pkt_ctx::kTvFlags], s)) != hipSuccess)
        return hip_fail(ctx, e, "hipEventRecord (to_vec flag)");
    return PKT_SUCCESS;
}

int pkt_set_fields_csum(pkt_ctx_t* ctx, const pkt_batch_t* b, const pkt_chain_t* chain,
                        const pkt_field_spec_t* specs, uint32_t nspec, const uint64_t* const* values,
                        int32_t ipv4_occurrence, void* stream) {
    if (!ctx || !b || (nspec && (!specs || !values))) return fail(ctx, PKT_ERR_INVALID_ARG, "null argument");
    if (b->n == 0 || (nspec == 0 && ipv4_occurrence < 0)) return PKT_SUCCESS;
    SParams sp;
    int rc = batch_ref(ctx, b, chain, sp.b);
    if (rc) return rc;
    sp.slab = const_cast<uint8_t*>(b->slab);
    for (uint32_t s = 0; s < nspec; s++)
        if (bad_spec(specs[s]) || !values[s]) return fail(ctx, PKT_ERR_INVALID_ARG, "bad field spec");
    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) return hip_fail(ctx, e, "hipSetDevice");
    // one thread per packet applies its specs in order; more than 32 specs: ordered launches, the
    // checksum refresh in the last one
    uint32_t s0 = 0;
    do {
        sp.nspec = std::min<uint32_t>(kMaxSpecs, nspec - s0);
        sp.csum_occ = s0 + sp.nspec >= nspec ? ipv4_occurrence : -1;
        for (uint32_t k = 0; k < sp.nspec; k++) {
            sp.s[k].f = specs[s0 + k];
            sp.s[k].values = values[s0 + k];
        }
        if (narrow_slots(b))
            hipLaunchKernelGGL(set_fields_kernel<4>, dim3(grid_of(b->n)), dim3(kRwBlock), 0, reinterpret_cast<hipStream_t>(stream), sp);
        else
            hipLaunchKernelGGL(set_fields_kernel<5>, dim3(grid_of(b->n)), dim3(kRwBlock), 0, reinterpret_cast<hipStream_t>(stream), sp);
        if ((e = hipGetLastError()) != hipSuccess) return hip_fail(ctx, e, "set_fields_kernel launch");
        s0 += sp.nspec;
    } while (s0 < nspec);
    return PKT_SUCCESS;
}

int pkt_set_fields(pkt_ctx_t* ctx, const pkt_batch_t* b, const pkt_chain_t* chain,
                   const pkt_field_spec_t* specs, uint32_t nspec, const uint64_t* const* values,
                   void* stream) {
    if (ctx && b && nspec == 0) return PKT_SUCCESS;
    return pkt_set_fields_csum(ctx, b, chain, specs, nspec, values, -1, stream);
}

int pkt_ipv4_update_checksum(pkt_ctx_t* ctx, const pkt_batch_t* b, const pkt_chain_t* chain,
                             uint32_t occurrence, void* stream) {
    if (!ctx || !b) return fail(ctx, PKT_ERR_INVALID_ARG, "null argument");
    if (b->n == 0) return PKT_SUCCESS;
    BatchRef r;
    int rc = batch_ref(ctx, b, chain, r);
    if (rc) return rc;
    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) return hip_fail(ctx, e, "hipSetDevice");
    hipLaunchKernelGGL(ipv4_update_kernel, dim3(grid_of(b->n)), dim3(kRwBlock), 0, reinterpret_cast<hipStream_t>(stream),
                       r, const_cast<uint8_t*>(b->slab), occurrence);
    if ((e = hipGetLastError()) != hipSuccess) return hip_fail(ctx, e, "ipv4_update_kernel launch");
    return PKT_SUCCESS;
}

int pkt_broadcast(pkt_ctx_t* ctx, const uint8_t* src, uint32_t len, uint64_t n, uint32_t stride,
                  uint8_t* dst, void* stream) {
    if (!ctx || (n && (!src || !dst))) return fail(ctx, PKT_ERR_INVALID_ARG, "null argument");
    if (n == 0) return PKT_SUCCESS;
    if (stride == 0 || stride % 16 || len > stride || ((uintptr_t)dst & 15))
        return fail(ctx, PKT_ERR_INVALID_ARG, "stride must be a non-zero multiple of 16 >= len, dst 16-byte aligned");
    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) return hip_fail(ctx, e, "hipSetDevice");
    const uint64_t chunks = n * (uint64_t)stride / 16;
    const unsigned grid = (unsigned)std::min<uint64_t>((chunks + kRwBlock - 1) / kRwBlock, 256u * 64u);
    hipLaunchKernelGGL(broadcast_kernel, dim3(grid), dim3(kRwBlock), 0, reinterpret_cast<hipStream_t>(stream), src, len, n,
                       stride, dst);
    if ((e = hipGetLastError()) != hipSuccess) return hip_fail(ctx, e, "broadcast_kernel launch");
    return PKT_SUCCESS;
}

int pkt_ipv4_checksum_batch(pkt_ctx_t* ctx, const uint8_t* hdrs, uint32_t stride, uint64_t n,
                            uint16_t* out, void* stream) {
    if (!ctx || (n && (!hdrs || !out)) || (n && stride < 20)) return fail(ctx, PKT_ERR_INVALID_ARG, "bad argument");
    if (n == 0) return PKT_SUCCESS;
    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) return hip_fail(ctx, e, "hipSetDevice");
    hipLaunchKernelGGL(ipv4_csum_kernel, dim3(grid_of(n)), dim3(kRwBlock), 0, reinterpret_cast<hipStream_t>(stream), hdrs,
                       stride, n, out);
    if ((e = hipGetLastError()) != hipSuccess) return hip_fail(ctx, e, "ipv4_csum_kernel launch");
    return PKT_SUCCESS;
}

}  // extern "C"
