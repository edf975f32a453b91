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
//                      metadata, then lane groups of G (the wave's largest packet in 16-byte chunks,
//                      rounded up to a power of two) copy 64/G packets per pass as 16-byte chunks
//                      (dwords shifted into place when source and destination differ in alignment).
//                      Q2 packets take a per-byte gather through the list.
//   set_fields_kernel  set_bit_range (headers.rs:315-324) per spec, in spec order, in place; chain in
//                      LDS, all specs (up to 32) in one launch; a field of <= 64 bits is read as one
//                      16-byte window (one round trip), set by a shift and mask, its bytes stored.
//   ipv4_update_kernel / ipv4_csum_kernel   Packet::ipv4_checksum (packet.rs:93-107, Q1 fold).
//   broadcast_kernel   n copies of one packet (the clone step of the pktgen loop).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "pktgpu_ctx.hpp"
#include "pktgpu_device.hpp"

using namespace pktgpu;

namespace {

__constant__ uint8_t kHdrSize[PKT_HDR_COUNT] = {0, 14, 4, 20, 40, 4, 20, 8, 28, 8, 14, 3, 5, 4, 4, 4, 4, 8, 12, 8, 35, 4};

constexpr uint32_t kRwBlock = 256;
constexpr int kMaxSpecs = 32;  // specs per launch (extract / set_fields)

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

// The lane's chain in LDS (slot-major [slot][lane]: per-lane byte / u16 reads of one slot are
// consecutive addresses, conflict-free).  Returns n_hdrs.
struct ChainLds {
    uint8_t type[PKT_MAX_HDRS][kRwBlock];
    uint16_t off[PKT_MAX_HDRS][kRwBlock];
};

__device__ __forceinline__ uint32_t stage_chain(const BatchRef& b, uint64_t i, uint32_t t, ChainLds& L) {
    uint32_t nh = b.n_hdrs[i];
    nh = nh > PKT_MAX_HDRS ? PKT_MAX_HDRS : nh;
    for (uint32_t j = 0; j < nh; j++) {
        L.type[j][t] = b.hdr_type[(uint64_t)j * b.n + i];
        L.off[j][t] = b.hdr_off[(uint64_t)j * b.n + i];
    }
    return nh;
}

// offset of the occurrence-th header of `type` in the lane's chain, or -1
__device__ __forceinline__ int32_t find_lds(const ChainLds& L, uint32_t t, uint32_t nh, uint32_t type, uint32_t occ) {
    uint32_t c = 0;
    for (uint32_t j = 0; j < nh; j++) {
        if (L.type[j][t] == type) {
            if (c == occ) return (int32_t)L.off[j][t];
            c++;
        }
    }
    return -1;
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

// Window of a lane's packet: its first kXnch aligned 16-byte chunks, in LDS at an odd dword stride
// (per-lane dword reads conflict-free); bytes past it come from global memory (PacketView).
constexpr int kXnch = 5;
constexpr uint32_t kXstride = 4 * kXnch + 1;  // dwords

__global__ __launch_bounds__(kRwBlock) void extract_kernel(XParams p) {
    __shared__ ChainLds L;
    __shared__ uint32_t win[kRwBlock * kXstride];
    const uint32_t t = threadIdx.x;
    const uint64_t i = (uint64_t)blockIdx.x * kRwBlock + t;
    if (i >= p.b.n) return;  // no barrier below: a lane reads only its own LDS
    const uint32_t nh = stage_chain(p.b, i, t, L);
    const uint64_t off = pkt_off(p.b, i);
    const uint64_t last16 = ((p.b.slab_len + 15) & ~(uint64_t)15) - 16;
    uint32_t* w = win + t * kXstride;
#pragma unroll
    for (int c = 0; c < kXnch; c++) {
        uint64_t o = (off & ~(uint64_t)15) + 16u * c;
        o = o > last16 ? last16 : o;
        const uint4 v = *reinterpret_cast<const uint4*>(p.b.slab + o);
        w[4 * c] = v.x;
        w[4 * c + 1] = v.y;
        w[4 * c + 2] = v.z;
        w[4 * c + 3] = v.w;
    }
    PacketView pv;
    pv.lw = reinterpret_cast<const uint8_t*>(w);
    pv.slab = p.b.slab;
    pv.off = off;
    pv.last4 = ((p.b.slab_len + 15) & ~(uint64_t)15) - 4;
    pv.shift = (uint32_t)(off & 15);
    pv.win_lo = 0;
    pv.win_end = 16u * kXnch - pv.shift;
    pv.len = 0xFFFFFFFFu;  // (le() does not use it)
    __builtin_amdgcn_wave_barrier();
    for (uint32_t s = 0; s < p.nspec; s++) {  // uniform
        const pkt_field_spec_t sp = p.s[s].f;
        const int32_t ho = find_lds(L, t, nh, sp.hdr_type, sp.occurrence);
        uint64_t v = 0;
        if (ho >= 0) {
            const uint32_t start = sp.start, end = sp.end, wd = end - start + 1;
            // bits [s2..end] hold the low 64 bits of the field; bit_range's release-build shifts
            // then keep the low (w mod 64, or 64) of them (headers.rs:262, Q8)
            const uint32_t s2 = wd > 64 ? end - 63 : start;
            const uint32_t b0 = s2 >> 3, b1 = end >> 3;  // <= 9 bytes
            const uint32_t rel = (uint32_t)ho + b0;
            // bytes b0.. as big-endian: 8 in hi, the 9th (if any) in the top byte of x2
            const uint64_t hi = ((uint64_t)__builtin_bswap32(pv.le(rel, 4)) << 32) | __builtin_bswap32(pv.le(rel + 4, 4));
            const uint32_t nb = b1 - b0 + 1;
            const uint32_t ninth = nb == 9 ? pv.le(rel + 8, 1) & 0xFFu : 0u;
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
        p.s[s].values[i] = v;
        if (p.s[s].found) p.s[s].found[i] = ho >= 0 ? 1 : 0;
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
};

__device__ __forceinline__ void put_byte(const TParams& p, uint64_t q, uint32_t v) {
    if (q < p.dst_len) p.dst[q] = (uint8_t)v;
}
__device__ __forceinline__ uint64_t shfl64(uint64_t v, uint32_t k) {
    return ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(v >> 32), (int)k, 64) << 32) | (uint32_t)__shfl((int)(uint32_t)v, (int)k, 64);
}

// GRE option header types: two or more of them in one list is the only way the list order can
// differ from wire order (Q2, fast.rs:154-163)
constexpr uint32_t kGreOptMask = (1u << PKT_HDR_GRE_CHKSUM_OFFSET) | (1u << PKT_HDR_GRE_SEQUENCE_NUM) | (1u << PKT_HDR_GRE_KEY);

__global__ __launch_bounds__(kRwBlock) void to_vec_kernel(TParams p) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t base = ((uint64_t)blockIdx.x * kRwBlock + (threadIdx.x & ~63u));  // wave's first packet
    const uint64_t i = base + lane;
    // ---- per-lane metadata of packet i (coalesced column reads)
    uint64_t src = 0, dst = 0;
    uint32_t len = 0, ident = 1, ok = 0;
    if (i < p.b.n) {
        ok = p.status[i] == PKT_OK;
        src = pkt_off(p.b, i);
        dst = p.dst_offsets ? p.dst_offsets[i] : src;
        if (ok) {
            const uint32_t po = p.payload_off[i], pl = p.payload_len[i];
            // at most one GRE option type in the list: headers lie back to back in list order, so
            // the list covers exactly [0, payload_off) and to_vec is the packet's bytes [0, len)
            const bool sure = p.hdr_mask && __builtin_popcount(p.hdr_mask[i] & kGreOptMask) <= 1;
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
        if (p.out_len) p.out_len[i] = ok ? len : 0u;
    }
    // ---- lane groups of G = the wave's largest packet in 16-byte chunks (power of two): 64 / G
    // packets are copied per pass, each by its own group
    uint32_t ch = ok ? (uint32_t)(((dst & 15) + len + 15) >> 4) : 0u;
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) ch = max(ch, (uint32_t)__shfl_xor((int)ch, m, 64));
    ch = __builtin_amdgcn_readfirstlane(ch);  // wave-uniform after the butterfly
    if (ch == 0) return;
    uint32_t G = 1;
    while (G < ch && G < 64u) G <<= 1;
    const uint32_t per = 64u / G, sub = lane & (G - 1u);
    for (uint32_t k0 = 0; k0 < 64u; k0 += per) {  // uniform
        const uint32_t k = k0 + lane / G;
        const uint64_t s = shfl64(src, k), d = shfl64(dst, k);
        const uint32_t L = (uint32_t)__shfl((int)len, (int)k, 64);
        const uint32_t okk = (uint32_t)__shfl((int)ok, (int)k, 64), idk = (uint32_t)__shfl((int)ident, (int)k, 64);
        if (!okk) continue;
        if (idk && ((s ^ d) & 15) == 0) {
            // same alignment: 16-byte chunks of [d, d+L); partial head/tail chunks by bytes
            const uint64_t c1 = (d + L + 15) & ~(uint64_t)15;
            for (uint64_t c = (d & ~(uint64_t)15) + 16u * sub; c < c1; c += 16u * G) {
                const uint4 v = *reinterpret_cast<const uint4*>(p.b.slab + (c - d + s));  // 16-byte aligned too
                if (c >= d && c + 16 <= d + L && c + 16 <= p.dst_len) {
                    *reinterpret_cast<uint4*>(p.dst + c) = v;
                } else {
                    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                    for (int q = 0; q < 16; q++)
                        if (c + q >= d && c + q < d + L) put_byte(p, c + q, w[q >> 2] >> (8 * (q & 3)));
                }
            }
        } else if (idk) {
            // different alignment: destination dwords, source bytes shifted into place
            const uint64_t w1 = (d + L + 3) & ~(uint64_t)3;
            for (uint64_t a = (d & ~(uint64_t)3) + 4u * sub; a < w1; a += 4u * G) {
                const uint64_t sa = a - d + s;  // source of this dword's first byte (may be < s)
                const uint32_t v = __builtin_amdgcn_alignbyte(slab_dw(p.b, sa + 4), slab_dw(p.b, sa), (uint32_t)(sa & 3));
                if (a >= d && a + 4 <= d + L && a + 4 <= p.dst_len) {
                    *reinterpret_cast<uint32_t*>(p.dst + a) = v;
                } else {
#pragma unroll
                    for (int q = 0; q < 4; q++)
                        if (a + q >= d && a + q < d + L) put_byte(p, a + q, v >> (8 * q));
                }
            }
        } else {
            // Q2: output byte q comes from the list entry covering it (header slices, then payload)
            const uint64_t ik = base + k;
            uint32_t nh = p.b.n_hdrs[ik];
            nh = nh > PKT_MAX_HDRS ? PKT_MAX_HDRS : nh;
            for (uint32_t q = sub; q < L; q += G) {
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
    SSpec s[kMaxSpecs];
};

__global__ __launch_bounds__(kRwBlock) void set_fields_kernel(SParams p) {
    __shared__ ChainLds L;
    const uint32_t t = threadIdx.x;
    const uint64_t i = (uint64_t)blockIdx.x * kRwBlock + t;
    if (i >= p.b.n) return;
    const uint32_t nh = stage_chain(p.b, i, t, L);
    const uint64_t off = pkt_off(p.b, i);
    for (uint32_t s = 0; s < p.nspec; s++) {  // specs in order: overlapping ones act as sequential setters
        const pkt_field_spec_t sp = p.s[s].f;
        const int32_t ho = find_lds(L, t, nh, sp.hdr_type, sp.occurrence);
        if (ho < 0) continue;
        const uint32_t lsb = sp.start, msb = sp.end;
        const uint64_t v0 = p.s[s].values[i];
        if (msb - lsb < 64) {
            // the field's <= 9 bytes from one 16-byte window read in a single round trip: set by one
            // shift and mask, then only the field's bytes stored (byte stores: neighbours untouched)
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
            for (uint32_t j = 0; j < nb; j++)  // uniform trip count
                h[j] = (uint8_t)((j < 8 ? W.hi >> (56 - 8 * j) : W.lo >> (120 - 8 * j)) & 0xFFu);
            continue;
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
    }
}

__global__ __launch_bounds__(kRwBlock) void ipv4_update_kernel(BatchRef b, uint8_t* slab, uint32_t occurrence) {
    __shared__ ChainLds L;
    const uint32_t t = threadIdx.x;
    const uint64_t i = (uint64_t)blockIdx.x * kRwBlock + t;
    if (i >= b.n) return;
    const uint32_t nh = stage_chain(b, i, t, L);
    const int32_t ho = find_lds(L, t, nh, PKT_HDR_IPV4, occurrence);
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
    for (uint32_t s0 = 0; s0 < nspec; s0 += kMaxSpecs) {  // one launch per 32 specs
        xp.nspec = std::min<uint32_t>(kMaxSpecs, nspec - s0);
        for (uint32_t k = 0; k < xp.nspec; k++) {
            xp.s[k].f = specs[s0 + k];
            xp.s[k].values = values[s0 + k];
            xp.s[k].found = found ? found[s0 + k] : nullptr;
        }
        hipLaunchKernelGGL(extract_kernel, dim3(grid_of(b->n)), dim3(kRwBlock), 0, reinterpret_cast<hipStream_t>(stream), xp);
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
    hipLaunchKernelGGL(to_vec_kernel, dim3(grid_of(b->n)), dim3(kRwBlock), 0, reinterpret_cast<hipStream_t>(stream), tp);
    if ((e = hipGetLastError()) != hipSuccess) return hip_fail(ctx, e, "to_vec_kernel launch");
    return PKT_SUCCESS;
}

int pkt_set_fields(pkt_ctx_t* ctx, const pkt_batch_t* b, const pkt_chain_t* chain,
                   const pkt_field_spec_t* specs, uint32_t nspec, const uint64_t* const* values,
                   void* stream) {
    if (!ctx || !b || (nspec && (!specs || !values))) return fail(ctx, PKT_ERR_INVALID_ARG, "null argument");
    if (b->n == 0 || nspec == 0) return PKT_SUCCESS;
    SParams sp;
    int rc = batch_ref(ctx, b, chain, sp.b);
    if (rc) return rc;
    sp.slab = const_cast<uint8_t*>(b->slab);
    for (uint32_t s = 0; s < nspec; s++)
        if (bad_spec(specs[s]) || !values[s]) return fail(ctx, PKT_ERR_INVALID_ARG, "bad field spec");
    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) return hip_fail(ctx, e, "hipSetDevice");
    // one thread per packet applies its specs in order; more than 32 specs: ordered launches
    for (uint32_t s0 = 0; s0 < nspec; s0 += kMaxSpecs) {
        sp.nspec = std::min<uint32_t>(kMaxSpecs, nspec - s0);
        for (uint32_t k = 0; k < sp.nspec; k++) {
            sp.s[k].f = specs[s0 + k];
            sp.s[k].values = values[s0 + k];
        }
        hipLaunchKernelGGL(set_fields_kernel, dim3(grid_of(b->n)), dim3(kRwBlock), 0, reinterpret_cast<hipStream_t>(stream), sp);
        if ((e = hipGetLastError()) != hipSuccess) return hip_fail(ctx, e, "set_fields_kernel launch");
    }
    return PKT_SUCCESS;
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
