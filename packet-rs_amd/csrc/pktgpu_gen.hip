// pktgpu_gen.hip — batched packet generation: the reference's pktgen loop
// (tests/lib.rs:756-788: build a packet with a utils::create_* builder, clone it, update a field,
// to_vec) as one device pass per batch.
//
// The builder runs once on the host and hands over its bytes (the template).  pkt_gen_create parses
// the template ON THE DEVICE with the same walk as pkt_parse_batch (so a field named by (header,
// occurrence, bits) resolves exactly as Packet's Index<&str> would find it, packet.rs:64-66) and
// turns every field into an absolute MSB-first bit range of the packet.  pkt_gen_run then writes
// n packets of `stride` bytes with one kernel.  Both kernels store the output as consecutive 1 KiB
// per wave-instruction (a lane-per-packet kernel storing its 16-byte pieces at the packet stride
// measured 5.5x slower on a 160-byte stride) and treat a 16-byte piece as a 128-bit big-endian
// integer (bit 0 of the make_header! numbering = its MSB), where a field is set_bit_range
// (headers.rs:315-324: the field's bits get the value's low `width` bits, bit `end` the value's
// bit 0) by one shift and mask.
//
//   gen_region_kernel (fields or checksums, stride <= 1 KiB): one lane per packet; the pieces of
//   the wave's 64 packets that a field or checksum touches are built in LDS (template, then each
//   field applied once per packet to the 1-2 pieces it overlaps, then Packet::ipv4_checksum
//   (packet.rs:93-107, Q1 fold) of each refreshed IPv4 header read back from the row, as the
//   builders do, utils.rs:233-236), then the packets are stored, untouched pieces straight from
//   the template (test_tcp_packet: 3 of 10 pieces in LDS; 11 fields + checksum 53 -> 42 us,
//   profiles/ab/r02gendirty_pktgen_touched_pieces.txt).
//   gen_kernel (pure clones, wider strides): one lane per 16-byte piece; a lane applies the fields
//   overlapping its piece and, if it holds checksum bytes, rebuilds that IPv4 header's pieces.
// Measured on test_tcp_packet (154 B, stride 160), 2^20 packets: clone 27 us (gen_kernel) / 30.5 us
// (region); one INC field 30.9 us (region) vs 37 us (gen_kernel); 11 splitmix64 fields + checksum
// 53.7 us (region) vs 351 us (gen_kernel: every field's value and shift computed for the whole wave).
// Nothing is read back: HBM traffic = the slab written + the per-packet value arrays read
// (PKT_GEN_VALUES fields only).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "pktgpu_ctx.hpp"
#include "pktgpu_device.hpp"

using pktgpu::U128;
using pktgpu::put_bits;

namespace {

#ifndef PKTGPU_GEN_NT
// non-temporal stores of the generated packets (region kernel): value arrays 58.7 -> 46.1 us, new
// packets 42.9 -> 41.5 us (profiles/ab/r02nt2_nt_wide_stores.txt)
#define PKTGPU_GEN_NT 1
#endif
constexpr int kMaxGenFields = 32;
constexpr int kMaxGenCsum = 8;
constexpr uint32_t kGenBlock = 256;
constexpr uint32_t kRegionMaxStride = 1024;  // gen_region_kernel: strides up to 64 pieces (LDS: 64 x the touched pieces)
// pieces per launch: lane indices stay 32-bit (a launch covers whole packets)
constexpr uint64_t kGenChunkPieces = 1ull << 31;

struct GenField {
    uint32_t s, e;        // absolute MSB-first bit range [s, e] in the packet (e - s < 64)
    uint32_t kind;        // pkt_gen_kind_t
    uint32_t w;           // e - s + 1
    uint64_t base, step, count;
    const uint64_t* values;  // PKT_GEN_VALUES: [n] of this launch
};

// A field's placement in the region kernel's LDS row, precomputed on the host by pkt_gen_create (the
// field's position is the same for every packet): for each of the <= 2 pieces its bits overlap, the
// piece's byte offset in the row, where the value's bit 0 lands in the piece's 128-bit big-endian
// integer (sh, from its LSB; negative = right shift) and the field's bits there (m).  The kernel then
// sets a field with one uniform shift of the value, an and-not and an or — round 3 rebuilt the masks
// and shifts per field in every wave (932 SALU + 890 VALU instructions per wave for 11 fields and a
// checksum, r04h PMC).
struct GenPut {
    uint32_t lds_off;
    int32_t sh;
    uint64_t mhi, mlo;
};
struct GenFieldPlan {
    GenPut p[2];
    uint32_t np;
    uint32_t pad[3];
};

struct GenParams {
    const uint8_t* tpl;   // device template, zero-padded to tpl_bytes (a multiple of 16)
    uint8_t* dst;         // first packet of this launch
    uint64_t first;       // global index of this launch's first packet (INC / RANDOM)
    uint32_t tpl_bytes;
    uint32_t ppp;         // 16-byte pieces per packet = stride / 16
    uint32_t nd;          // gen_region_kernel: pieces a field or checksum touches (staged in LDS)
    uint32_t pk_magic;    // ceil(2^20 / ppp): packet of output piece q = (q * pk_magic) >> 20
    int8_t slot[64];      // piece -> its LDS slot in the packet's row, -1 = the template's bytes
    uint32_t npieces;     // pieces of this launch (gen_kernel)
    uint32_t npkts;       // packets of this launch (gen_region_kernel)
    uint32_t nf, ncs;
    uint32_t csum_at[kMaxGenCsum];  // byte offset of each refreshed IPv4 header
    uint32_t csum_lds[kMaxGenCsum];  // gen_region_kernel: that header's byte offset in the LDS row
    const GenFieldPlan* plan;  // gen_region_kernel: [nf] (device)
    GenField f[kMaxGenFields];
};

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// Value of field f for packet i of this launch (global index g = first + i).
__device__ __forceinline__ uint64_t field_value(const GenField& f, uint32_t i, uint64_t g) {
    if (f.kind == PKT_GEN_VALUES) return f.values[i];
    if (f.kind == PKT_GEN_RANDOM) return splitmix64(f.base + g);
    uint64_t k = g;
    if (f.count) k = (g < (1ull << 32) && f.count < (1ull << 32)) ? (uint64_t)((uint32_t)g % (uint32_t)f.count)
                                                                    : g % f.count;
    return f.base + f.step * k;
}

// Template piece k of packet i with every field applied (checksums not yet refreshed).
__device__ __forceinline__ U128 build_piece(const GenParams& p, uint32_t k, uint32_t i, uint64_t g) {
    U128 x{0, 0};
    const uint32_t b = k * 16u;
    if (b < p.tpl_bytes) {
        const uint4 t = *reinterpret_cast<const uint4*>(p.tpl + b);
        x.hi = ((uint64_t)__builtin_bswap32(t.x) << 32) | __builtin_bswap32(t.y);
        x.lo = ((uint64_t)__builtin_bswap32(t.z) << 32) | __builtin_bswap32(t.w);
    }
    const uint32_t b0 = b * 8u;
    for (uint32_t j = 0; j < p.nf; j++) {  // uniform loop
        const GenField& f = p.f[j];
        if (f.s <= b0 + 127u && f.e >= b0) put_bits(x, f.s, f.e, f.w, field_value(f, i, g), b0);
    }
    return x;
}

// byte q (0..47) of three consecutive pieces (selects, not an indexed array: no scratch)
__device__ __forceinline__ uint32_t byte3(const U128& w0, const U128& w1, const U128& w2, uint32_t q) {
    const uint32_t sel = q >> 4;
    const U128 x = sel == 0 ? w0 : (sel == 1 ? w1 : w2);
    const uint32_t r = q & 15u;
    const uint64_t h = r < 8 ? x.hi : x.lo;
    return (uint32_t)(h >> (8u * (7u - (r & 7u)))) & 0xFFu;
}

// Packet::ipv4_checksum's folded sum (packet.rs:93-107, Q1) over the IPv4 header at byte hb of
// packet i as generated; piece `have` (== x) is reused, the others are rebuilt.
__device__ __forceinline__ uint32_t ipv4_sum(const GenParams& p, uint32_t hb, uint32_t have, const U128& x,
                                             uint32_t i, uint64_t g) {
    const uint32_t k0 = hb >> 4, r = hb & 15u;
    const U128 w0 = k0 == have ? x : build_piece(p, k0, i, g);
    const U128 w1 = k0 + 1u == have ? x : build_piece(p, k0 + 1u, i, g);
    const U128 w2 = r + 20u > 32u ? (k0 + 2u == have ? x : build_piece(p, k0 + 2u, i, g)) : U128{0, 0};
    uint32_t s = 0;
#pragma unroll
    for (uint32_t j = 0; j < 20; j += 2)
        if (j != 10) s += (byte3(w0, w1, w2, r + j) << 8) | byte3(w0, w1, w2, r + j + 1);
    return ((s >> 16) + s) & 0xFFFFu;  // packet.rs:102-104 (Q1)
}

__device__ __forceinline__ void store_piece(uint8_t* at, const U128& x) {
    uint4 o;
    o.x = __builtin_bswap32((uint32_t)(x.hi >> 32));
    o.y = __builtin_bswap32((uint32_t)x.hi);
    o.z = __builtin_bswap32((uint32_t)(x.lo >> 32));
    o.w = __builtin_bswap32((uint32_t)x.lo);
    *reinterpret_cast<uint4*>(at) = o;
}

__global__ __launch_bounds__(kGenBlock) void gen_kernel(GenParams p) {
    const uint32_t q = blockIdx.x * kGenBlock + threadIdx.x;
    if (q >= p.npieces) return;
    const uint32_t i = q / p.ppp;       // packet within this launch
    const uint32_t k = q - i * p.ppp;   // piece within the packet
    const uint64_t g = p.first + i;
    U128 x = build_piece(p, k, i, g);
    // IPv4 checksum refresh: the lane holding bytes hb+10 / hb+11 rebuilds the header's pieces
    for (uint32_t c = 0; c < p.ncs; c++) {
        const uint32_t hb = p.csum_at[c];
        const uint32_t cb = hb + 10u;
        if (cb + 1u < k * 16u || cb >= k * 16u + 16u) continue;
        const uint32_t s = ipv4_sum(p, hb, k, x, i, g);
        put_bits(x, cb * 8u, cb * 8u + 15u, 16u, (uint64_t)(~s & 0xFFFFu), k * 128u);
    }
    store_piece(p.dst + (uint64_t)q * 16u, x);
}

// One lane per packet, the wave's WHOLE output region (64 packets x stride) built in LDS (one
// wave per block), then stored with the contiguous 1 KiB-per-instruction shape of gen_kernel.  Each
// lane writes the template into its row, then applies the fields in order — one field at a time,
// read-modify-write of the 1-2 pieces it overlaps, so a field's parameters are read once per
// packet group and its value computed once per packet — then refreshes the checksums from the row.
__device__ __forceinline__ U128 lds_get(const uint8_t* at) {
    const uint4 t = *reinterpret_cast<const uint4*>(at);
    return U128{((uint64_t)__builtin_bswap32(t.x) << 32) | __builtin_bswap32(t.y),
                ((uint64_t)__builtin_bswap32(t.z) << 32) | __builtin_bswap32(t.w)};
}
__device__ __forceinline__ void lds_put(uint8_t* at, const U128& x) {
    *reinterpret_cast<uint4*>(at) = make_uint4(__builtin_bswap32((uint32_t)(x.hi >> 32)), __builtin_bswap32((uint32_t)x.hi),
                                               __builtin_bswap32((uint32_t)(x.lo >> 32)), __builtin_bswap32((uint32_t)x.lo));
}

__global__ __launch_bounds__(64) void gen_region_kernel(GenParams p) {
    extern __shared__ __attribute__((aligned(16))) uint8_t region[];
    __shared__ uint4 tp[64];      // the template's pieces (zeros past it)
    __shared__ int32_t sl[64];    // piece -> slot
    const uint32_t lane = threadIdx.x;
    const uint32_t w0 = blockIdx.x * 64u;
    const uint32_t i = w0 + lane;
    const bool act = i < p.npkts;
    const uint64_t g = p.first + i;
    const uint32_t stride = p.ppp * 16u;
    if (lane < p.ppp) {
        tp[lane] = lane * 16u < p.tpl_bytes ? *reinterpret_cast<const uint4*>(p.tpl + lane * 16u) : make_uint4(0, 0, 0, 0);
        sl[lane] = p.slot[lane];
    }
    __syncthreads();
    // Only the pieces a field or a checksum touches are built in LDS (the row holds nd of them);
    // the rest of each packet is the template, stored straight from `tp`.
    uint8_t* row = region + lane * p.nd * 16u;
    for (uint32_t k = 0; k < p.ppp; k++)
        if (sl[k] >= 0) *reinterpret_cast<uint4*>(row + sl[k] * 16u) = tp[k];
    for (uint32_t j = 0; j < p.nf; j++) {  // fields in order (uniform)
        const GenField& f = p.f[j];
        const GenFieldPlan& fp = p.plan[j];
        const uint64_t v = act ? field_value(f, i, g) : 0;
        for (uint32_t q = 0; q < fp.np; q++) {
            const GenPut& pp = fp.p[q];
            const int32_t sh = pp.sh;  // uniform: the branches below are scalar
            U128 V;
            if (sh >= 64) V = U128{v << (sh - 64), 0};
            else if (sh > 0) V = U128{v >> (64 - sh), v << sh};
            else if (sh == 0) V = U128{0, v};
            else V = U128{0, v >> (-sh)};
            uint8_t* at = row + pp.lds_off;
            U128 x = lds_get(at);
            x.hi = (x.hi & ~pp.mhi) | (V.hi & pp.mhi);
            x.lo = (x.lo & ~pp.mlo) | (V.lo & pp.mlo);
            lds_put(at, x);
        }
    }
    for (uint32_t c = 0; c < p.ncs; c++) {  // checksums last (uniform)
        // the header's 20 bytes lie contiguous in the row (its pieces are dirty, so their slots are
        // consecutive): five unaligned dwords, the nine big-endian words but the checksum's (Q1 fold)
        uint8_t* h = row + p.csum_lds[c];
        uint32_t d[5];
        __builtin_memcpy(d, h, 20);
        uint32_t sum = 0;
#pragma unroll
        for (int k = 0; k < 5; k++) {
            const uint32_t b = __builtin_bswap32(d[k]);
            sum += (b >> 16) + (k == 2 ? 0u : (b & 0xFFFFu));  // bytes 10-11: the checksum itself
        }
        const uint32_t cv = ~(((sum >> 16) + sum) & 0xFFFFu) & 0xFFFFu;  // packet.rs:102-104 (Q1)
        h[10] = (uint8_t)(cv >> 8);
        h[11] = (uint8_t)cv;
    }
    __syncthreads();
    const uint32_t npk = p.npkts - w0 < 64u ? p.npkts - w0 : 64u;
    const uint32_t bytes = npk * stride;
    uint8_t* d = p.dst + (uint64_t)w0 * stride;
    // the wave's packets as consecutive 1 KiB per store instruction: output piece q is piece k of
    // packet pk, from its LDS slot or the template
    for (uint32_t o = lane * 16u; o < bytes; o += 1024u) {
        const uint32_t q = o >> 4, pk = (q * p.pk_magic) >> 20, k = q - pk * p.ppp;
        const int32_t sk = sl[k];
        const uint4 v = sk >= 0 ? *reinterpret_cast<const uint4*>(region + (pk * p.nd + (uint32_t)sk) * 16u) : tp[k];
#if PKTGPU_GEN_NT
        typedef uint32_t v4u __attribute__((ext_vector_type(4)));
        __builtin_nontemporal_store(v4u{v.x, v.y, v.z, v.w}, reinterpret_cast<v4u*>(d + o));
#else
        *reinterpret_cast<uint4*>(d + o) = v;
#endif
    }
}
}  // namespace

struct pkt_gen {
    pkt_ctx_t* ctx = nullptr;
    uint8_t* tpl = nullptr;  // device, zero-padded to tpl_bytes
    uint32_t len = 0, tpl_bytes = 0;
    std::vector<GenField> fields;
    std::vector<uint32_t> csum_at;
    // region-kernel placement (pieces < 64 only): slot per piece, dirty pieces, the field plans
    int8_t slot[64];
    uint32_t nd = 0;
    bool region_ok = false;  // every touched piece < 64
    GenFieldPlan* plan = nullptr;  // device, [fields]
};

extern "C" {

size_t pkt_sizeof_gen_field(void) { return sizeof(pkt_gen_field_t); }

int pkt_gen_create(pkt_ctx_t* ctx, const uint8_t* tpl, uint32_t len, int entry, const pkt_gen_field_t* fields,
                   uint32_t nfields, uint32_t ipv4_csum_mask, pkt_gen_t** out) {
    if (!ctx || !out || !tpl || len == 0 || (nfields && !fields)) return fail(ctx, PKT_ERR_INVALID_ARG, "null argument");
    *out = nullptr;
    if (entry < 0 || entry >= PKT_ENTRY_COUNT) return fail(ctx, PKT_ERR_INVALID_ARG, "bad entry");
    if (len > 0xFFFFu) return fail(ctx, PKT_ERR_INVALID_ARG, "template longer than 65535 bytes");
    if (nfields > (uint32_t)kMaxGenFields) return fail(ctx, PKT_ERR_INVALID_ARG, "more than 32 fields");
    for (uint32_t j = 0; j < nfields; j++) {
        const pkt_field_spec_t& f = fields[j].field;
        if (f.hdr_type == 0 || f.hdr_type >= PKT_HDR_COUNT || f.end < f.start || f.end - f.start >= 64 ||
            f.end >= 8 * pkt_hdr_size(f.hdr_type) || fields[j].kind > PKT_GEN_RANDOM)
            return fail(ctx, PKT_ERR_INVALID_ARG, "bad generator field (width 1..64 bits inside its header)");
    }
    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) return hip_fail(ctx, e, "hipSetDevice");

    // Parse the template on the device (chain columns of one packet) to place every field.
    const uint32_t tb = (len + 15u) & ~15u;
    uint8_t* dtpl = nullptr;
    uint8_t* dcol = nullptr;  // status, n_hdrs, hdr_type[16], hdr_off[16], lens[1]
    if ((e = hipMalloc(reinterpret_cast<void**>(&dtpl), tb)) != hipSuccess ||
        (e = hipMalloc(reinterpret_cast<void**>(&dcol), 256)) != hipSuccess) {
        (void)hipFree(dtpl);
        return hip_fail(ctx, e, "hipMalloc (generator template)");
    }
    std::vector<uint8_t> padded(tb, 0);
    std::memcpy(padded.data(), tpl, len);
    pkt_out_t o;
    std::memset(&o, 0, sizeof(o));
    o.status = dcol;
    o.n_hdrs = dcol + 16;
    o.hdr_type = dcol + 32;
    o.hdr_off = reinterpret_cast<uint16_t*>(dcol + 64);
    uint32_t* dlen = reinterpret_cast<uint32_t*>(dcol + 128);
    pkt_batch_t b;
    std::memset(&b, 0, sizeof(b));
    b.slab = dtpl;
    b.slab_len = tb;  // >= 16; the packet itself is `len` bytes (lens)
    b.lens = dlen;
    b.stride = tb;
    b.n = 1;
    uint8_t st = 0, nh = 0, ty[PKT_MAX_HDRS] = {};
    uint16_t off[PKT_MAX_HDRS] = {};
    int rc = PKT_SUCCESS;
    e = hipMemcpy(dtpl, padded.data(), tb, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(dlen, &len, 4, hipMemcpyHostToDevice);
    if (e == hipSuccess) {
        rc = pkt_parse_batch(ctx, &b, entry, &o, nullptr);
        if (rc == PKT_SUCCESS) {
            e = hipDeviceSynchronize();
            if (e == hipSuccess) e = hipMemcpy(&st, o.status, 1, hipMemcpyDeviceToHost);
            if (e == hipSuccess) e = hipMemcpy(&nh, o.n_hdrs, 1, hipMemcpyDeviceToHost);
            if (e == hipSuccess) e = hipMemcpy(ty, o.hdr_type, PKT_MAX_HDRS, hipMemcpyDeviceToHost);
            if (e == hipSuccess) e = hipMemcpy(off, o.hdr_off, 2 * PKT_MAX_HDRS, hipMemcpyDeviceToHost);
        }
    }
    (void)hipFree(dcol);
    if (rc == PKT_SUCCESS && e != hipSuccess) rc = hip_fail(ctx, e, "template parse");
    if (rc == PKT_SUCCESS && st != PKT_OK) rc = fail(ctx, PKT_ERR_INVALID_ARG, "template does not parse (status not OK)");
    auto find = [&](uint32_t type, uint32_t occ) -> int {
        for (uint32_t j = 0, c = 0; j < nh; j++)
            if (ty[j] == type && c++ == occ) return (int)off[j];
        return -1;
    };
    pkt_gen* G = nullptr;
    if (rc == PKT_SUCCESS) {
        G = new pkt_gen();
        G->ctx = ctx;
        G->len = len;
        G->tpl_bytes = tb;
        for (uint32_t j = 0; j < nfields && rc == PKT_SUCCESS; j++) {
            const pkt_gen_field_t& f = fields[j];
            const int at = find(f.field.hdr_type, f.field.occurrence);
            if (at < 0) { rc = fail(ctx, PKT_ERR_INVALID_ARG, "generator field: header not in the template's chain"); break; }
            GenField gf;
            gf.s = (uint32_t)at * 8u + f.field.start;
            gf.e = (uint32_t)at * 8u + f.field.end;
            gf.w = gf.e - gf.s + 1u;
            gf.kind = f.kind;
            gf.base = f.base;
            gf.step = f.step;
            gf.count = f.count;
            gf.values = nullptr;
            G->fields.push_back(gf);
        }
        for (uint32_t occ = 0; occ < 32 && rc == PKT_SUCCESS; occ++) {
            if (!(ipv4_csum_mask >> occ & 1u)) continue;
            const int at = find(PKT_HDR_IPV4, occ);
            if (at < 0) { rc = fail(ctx, PKT_ERR_INVALID_ARG, "checksum mask names an IPv4 header the template lacks"); break; }
            if (G->csum_at.size() == (size_t)kMaxGenCsum) { rc = fail(ctx, PKT_ERR_INVALID_ARG, "more than 8 checksum refreshes"); break; }
            G->csum_at.push_back((uint32_t)at);
        }
    }
    if (rc == PKT_SUCCESS) {
        // the region kernel's placement: the pieces a field or a checksum (its whole 20-byte header)
        // touches get consecutive LDS slots, and each field's puts are precomputed
        bool dirty[64] = {};
        G->region_ok = true;
        auto touch = [&](uint32_t k) {
            if (k < 64) dirty[k] = true;
            else G->region_ok = false;
        };
        for (const GenField& f : G->fields)
            for (uint32_t k = f.s >> 7; k <= (f.e >> 7); k++) touch(k);
        for (uint32_t at : G->csum_at)
            for (uint32_t k = at >> 4; k <= ((at + 19u) >> 4); k++) touch(k);
        G->nd = 0;
        for (uint32_t k = 0; k < 64; k++) G->slot[k] = dirty[k] ? (int8_t)G->nd++ : (int8_t)-1;
        std::vector<GenFieldPlan> plan(std::max<size_t>(1, G->fields.size()));
        for (size_t j = 0; j < G->fields.size() && G->region_ok; j++) {
            const GenField& f = G->fields[j];
            GenFieldPlan& fp = plan[j];
            std::memset(&fp, 0, sizeof(fp));
            for (uint32_t k = f.s >> 7; k <= (f.e >> 7); k++) {
                GenPut& pp = fp.p[fp.np++];
                pp.lds_off = (uint32_t)G->slot[k] * 16u;
                pp.sh = 127 - ((int32_t)f.e - (int32_t)(k * 128u));  // value bit 0 from the piece's LSB
                // the field's bits within the piece: w ones shifted by sh (clipped to 128 bits)
                const uint64_t ones = f.w >= 64 ? ~0ull : ((1ull << f.w) - 1ull);
                uint64_t mhi = 0, mlo = 0;
                const int32_t sh = pp.sh;
                if (sh >= 64) mhi = sh - 64 < 64 ? ones << (sh - 64) : 0;
                else if (sh > 0) mhi = ones >> (64 - sh), mlo = ones << sh;
                else if (sh == 0) mlo = ones;
                else mlo = -sh < 64 ? ones >> (-sh) : 0;
                pp.mhi = mhi;
                pp.mlo = mlo;
            }
        }
        e = hipMalloc(reinterpret_cast<void**>(&G->plan), plan.size() * sizeof(GenFieldPlan));
        if (e == hipSuccess) e = hipMemcpy(G->plan, plan.data(), plan.size() * sizeof(GenFieldPlan), hipMemcpyHostToDevice);
        if (e != hipSuccess) rc = hip_fail(ctx, e, "hipMalloc (generator plan)");
    }
    if (rc != PKT_SUCCESS) {
        if (G) (void)hipFree(G->plan);
        delete G;
        (void)hipFree(dtpl);
        return rc;
    }
    G->tpl = dtpl;
    *out = G;
    return PKT_SUCCESS;
}

int pkt_gen_destroy(pkt_gen_t* g) {
    if (!g) return PKT_SUCCESS;
    if (g->tpl) {
        (void)hipSetDevice(g->ctx->device);
        (void)hipDeviceSynchronize();  // runs still in flight read the template
        (void)hipFree(g->tpl);
        (void)hipFree(g->plan);
    }
    delete g;
    return PKT_SUCCESS;
}

int pkt_gen_run(pkt_gen_t* g, uint64_t first, uint64_t n, uint32_t stride, const uint64_t* const* values,
                uint8_t* dst, void* stream) {
    if (!g) return PKT_ERR_INVALID_ARG;
    pkt_ctx_t* ctx = g->ctx;
    if (n == 0) return PKT_SUCCESS;
    if (!dst || ((uintptr_t)dst & 15)) return fail(ctx, PKT_ERR_INVALID_ARG, "dst null or not 16-byte aligned");
    if (stride == 0 || stride % 16 || stride < g->len)
        return fail(ctx, PKT_ERR_INVALID_ARG, "stride must be a multiple of 16 and >= the template length");
    for (size_t j = 0; j < g->fields.size(); j++)
        if (g->fields[j].kind == PKT_GEN_VALUES && (!values || !values[j]))
            return fail(ctx, PKT_ERR_INVALID_ARG, "PKT_GEN_VALUES field without a value array");
    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) return hip_fail(ctx, e, "hipSetDevice");
    GenParams p;
    std::memset(&p, 0, sizeof(p));
    p.tpl = g->tpl;
    p.tpl_bytes = std::min<uint32_t>(g->tpl_bytes, stride);
    p.ppp = stride / 16;
    p.nf = (uint32_t)g->fields.size();
    p.ncs = (uint32_t)g->csum_at.size();
    for (uint32_t c = 0; c < p.ncs; c++) p.csum_at[c] = g->csum_at[c];
    // the region kernel's placement (pkt_gen_create)
    p.nd = g->nd;
    for (uint32_t k = 0; k < 64; k++) p.slot[k] = k < p.ppp ? g->slot[k] : (int8_t)-1;
    for (uint32_t c = 0; c < p.ncs; c++) p.csum_lds[c] = (uint32_t)g->slot[p.csum_at[c] >> 4] * 16u + (p.csum_at[c] & 15u);
    p.plan = g->plan;
    p.pk_magic = ((1u << 20) + p.ppp - 1) / p.ppp;
    const uint64_t per = std::max<uint64_t>(1, kGenChunkPieces / p.ppp);  // packets per launch
    for (uint64_t i0 = 0; i0 < n; i0 += per) {
        const uint64_t m = std::min(per, n - i0);
        for (uint32_t j = 0; j < p.nf; j++) {
            p.f[j] = g->fields[j];
            if (p.f[j].kind == PKT_GEN_VALUES) p.f[j].values = values[j] + i0;
        }
        p.first = first + i0;
        p.dst = dst + i0 * stride;
        p.npieces = (uint32_t)(m * p.ppp);
        p.npkts = (uint32_t)m;
        // region kernel whenever a field or checksum is applied and the 64-packet region fits LDS;
        // pure clones (and strides over 1 KiB) take the lane-per-piece kernel
        if ((p.nf || p.ncs) && stride <= kRegionMaxStride && g->region_ok)
            hipLaunchKernelGGL(gen_region_kernel, dim3((p.npkts + 63) / 64), dim3(64), 64u * 16u * p.nd,
                               reinterpret_cast<hipStream_t>(stream), p);
        else
            hipLaunchKernelGGL(gen_kernel, dim3((p.npieces + kGenBlock - 1) / kGenBlock), dim3(kGenBlock), 0,
                               reinterpret_cast<hipStream_t>(stream), p);
        e = hipGetLastError();
        if (e != hipSuccess) return hip_fail(ctx, e, "gen_kernel launch");
    }
    return PKT_SUCCESS;
}

}  // extern "C"
