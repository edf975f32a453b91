// pktgpu.hip — kernels and the C ABI (include/pktgpu.h) of the MI355X batched parser.
//
// Kernels
//   parse_kernel<NCH>     fast::parse_<entry> over a batch: LDS-DMA staging of NCH 16-byte
//                         chunks per packet, the chain walk, and the fused field/checksum
//                         extraction of the first Ether/Vlan/IPv4/IPv6/TCP/UDP (Q11).
//   extract_kernel        batched make_header! getter for arbitrary (type, occurrence, bits).
//   ipv4_csum_kernel      Packet::ipv4_checksum over a strided array of 20-byte headers.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>

#include "pktgpu_device.hpp"

using namespace pktgpu;

struct pkt_ctx {
    int device;
    uint32_t window;  // 0 = auto
    std::string err;
};

namespace {

// Fields of the first header of each group (Q11), from the walk's first offsets.
__device__ __forceinline__ void emit_fields(const pkt_out_t& out, uint64_t i, const PacketView& pv,
                                            const WalkResult& r, bool ok) {
    // Ether (headers.rs:530-540): dst 0-47, src 48-95, etype 96-111
    if (out.eth_dst || out.eth_src || out.eth_etype) {
        uint32_t d[4] = {0, 0, 0, 0};
        bool h = ok && r.f_eth >= 0;
        if (h) pv.hdr<4>((uint32_t)r.f_eth, 14, d);
        if (out.eth_dst) out.eth_dst[i] = h ? (((uint64_t)d[0] << 16) | (d[1] >> 16)) : 0ull;
        if (out.eth_src) out.eth_src[i] = h ? (((uint64_t)(d[1] & 0xFFFFu) << 32) | d[2]) : 0ull;
        if (out.eth_etype) out.eth_etype[i] = h ? (uint16_t)(d[3] >> 16) : (uint16_t)0;
    }
    // Vlan (headers.rs:543-552): pcp 0-2, cfi 3, vid 4-15, etype 16-31
    if (out.vlan_pcp || out.vlan_cfi || out.vlan_vid || out.vlan_etype) {
        uint32_t d[1] = {0};
        bool h = ok && r.f_vlan >= 0;
        if (h) pv.hdr<1>((uint32_t)r.f_vlan, 4, d);
        if (out.vlan_pcp) out.vlan_pcp[i] = (uint8_t)(d[0] >> 29);
        if (out.vlan_cfi) out.vlan_cfi[i] = (uint8_t)((d[0] >> 28) & 1u);
        if (out.vlan_vid) out.vlan_vid[i] = (uint16_t)((d[0] >> 16) & 0xFFFu);
        if (out.vlan_etype) out.vlan_etype[i] = (uint16_t)(d[0] & 0xFFFFu);
    }
    // IPv4 (headers.rs:555-574) + Packet::ipv4_checksum (packet.rs:93-107)
    if (out.ipv4_version || out.ipv4_ihl || out.ipv4_diffserv || out.ipv4_total_len ||
        out.ipv4_identification || out.ipv4_flags || out.ipv4_frag_startset || out.ipv4_ttl ||
        out.ipv4_protocol || out.ipv4_header_checksum || out.ipv4_src || out.ipv4_dst ||
        out.ipv4_csum_calc) {
        uint32_t d[5] = {0, 0, 0, 0, 0};
        bool h = ok && r.f_ipv4 >= 0;
        if (h) pv.hdr<5>((uint32_t)r.f_ipv4, 20, d);
        if (out.ipv4_version) out.ipv4_version[i] = (uint8_t)(d[0] >> 28);
        if (out.ipv4_ihl) out.ipv4_ihl[i] = (uint8_t)((d[0] >> 24) & 0xFu);
        if (out.ipv4_diffserv) out.ipv4_diffserv[i] = (uint8_t)((d[0] >> 16) & 0xFFu);
        if (out.ipv4_total_len) out.ipv4_total_len[i] = (uint16_t)(d[0] & 0xFFFFu);
        if (out.ipv4_identification) out.ipv4_identification[i] = (uint16_t)(d[1] >> 16);
        if (out.ipv4_flags) out.ipv4_flags[i] = (uint8_t)((d[1] >> 13) & 7u);
        if (out.ipv4_frag_startset) out.ipv4_frag_startset[i] = (uint16_t)(d[1] & 0x1FFFu);
        if (out.ipv4_ttl) out.ipv4_ttl[i] = (uint8_t)(d[2] >> 24);
        if (out.ipv4_protocol) out.ipv4_protocol[i] = (uint8_t)((d[2] >> 16) & 0xFFu);
        if (out.ipv4_header_checksum) out.ipv4_header_checksum[i] = (uint16_t)(d[2] & 0xFFFFu);
        if (out.ipv4_src) out.ipv4_src[i] = d[3];
        if (out.ipv4_dst) out.ipv4_dst[i] = d[4];
        if (out.ipv4_csum_calc) {
            // nine BE words, word 5 (byte offset 10) skipped; fold ((s>>16)+s)&0xFFFF (Q1)
            uint32_t s = (d[0] >> 16) + (d[0] & 0xFFFFu) + (d[1] >> 16) + (d[1] & 0xFFFFu) +
                         (d[2] >> 16) + (d[3] >> 16) + (d[3] & 0xFFFFu) + (d[4] >> 16) +
                         (d[4] & 0xFFFFu);
            s = ((s >> 16) + s) & 0xFFFFu;
            out.ipv4_csum_calc[i] = h ? (uint16_t)(~s) : (uint16_t)0;
        }
    }
    // IPv6 (headers.rs:577-592); src/dst as the raw 16 bytes of bytes(msb, lsb)
    if (out.ipv6_version || out.ipv6_traffic_class || out.ipv6_flow_label || out.ipv6_payload_len ||
        out.ipv6_next_hdr || out.ipv6_hop_limit || out.ipv6_src || out.ipv6_dst) {
        uint32_t d[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
        bool h = ok && r.f_ipv6 >= 0;
        if (h) pv.hdr<10>((uint32_t)r.f_ipv6, 40, d);
        if (out.ipv6_version) out.ipv6_version[i] = (uint8_t)(d[0] >> 28);
        if (out.ipv6_traffic_class) out.ipv6_traffic_class[i] = (uint8_t)((d[0] >> 20) & 0xFFu);
        if (out.ipv6_flow_label) out.ipv6_flow_label[i] = d[0] & 0xFFFFFu;
        if (out.ipv6_payload_len) out.ipv6_payload_len[i] = (uint16_t)(d[1] >> 16);
        if (out.ipv6_next_hdr) out.ipv6_next_hdr[i] = (uint8_t)((d[1] >> 8) & 0xFFu);
        if (out.ipv6_hop_limit) out.ipv6_hop_limit[i] = (uint8_t)(d[1] & 0xFFu);
        if (out.ipv6_src)
            *reinterpret_cast<uint4*>(out.ipv6_src + 16 * i) =
                make_uint4(bswap32(d[2]), bswap32(d[3]), bswap32(d[4]), bswap32(d[5]));
        if (out.ipv6_dst)
            *reinterpret_cast<uint4*>(out.ipv6_dst + 16 * i) =
                make_uint4(bswap32(d[6]), bswap32(d[7]), bswap32(d[8]), bswap32(d[9]));
    }
    // TCP (headers.rs:606-622)
    if (out.tcp_src || out.tcp_dst || out.tcp_seq_no || out.tcp_ack_no || out.tcp_data_startset ||
        out.tcp_res || out.tcp_flags || out.tcp_window || out.tcp_checksum || out.tcp_urgent_ptr) {
        uint32_t d[5] = {0, 0, 0, 0, 0};
        bool h = ok && r.f_tcp >= 0;
        if (h) pv.hdr<5>((uint32_t)r.f_tcp, 20, d);
        if (out.tcp_src) out.tcp_src[i] = (uint16_t)(d[0] >> 16);
        if (out.tcp_dst) out.tcp_dst[i] = (uint16_t)(d[0] & 0xFFFFu);
        if (out.tcp_seq_no) out.tcp_seq_no[i] = d[1];
        if (out.tcp_ack_no) out.tcp_ack_no[i] = d[2];
        if (out.tcp_data_startset) out.tcp_data_startset[i] = (uint8_t)(d[3] >> 28);
        if (out.tcp_res) out.tcp_res[i] = (uint8_t)((d[3] >> 24) & 0xFu);
        if (out.tcp_flags) out.tcp_flags[i] = (uint8_t)((d[3] >> 16) & 0xFFu);
        if (out.tcp_window) out.tcp_window[i] = (uint16_t)(d[3] & 0xFFFFu);
        if (out.tcp_checksum) out.tcp_checksum[i] = (uint16_t)(d[4] >> 16);
        if (out.tcp_urgent_ptr) out.tcp_urgent_ptr[i] = (uint16_t)(d[4] & 0xFFFFu);
    }
    // UDP (headers.rs:625-634)
    if (out.udp_src || out.udp_dst || out.udp_length || out.udp_checksum) {
        uint32_t d[2] = {0, 0};
        bool h = ok && r.f_udp >= 0;
        if (h) pv.hdr<2>((uint32_t)r.f_udp, 8, d);
        if (out.udp_src) out.udp_src[i] = (uint16_t)(d[0] >> 16);
        if (out.udp_dst) out.udp_dst[i] = (uint16_t)(d[0] & 0xFFFFu);
        if (out.udp_length) out.udp_length[i] = (uint16_t)(d[1] >> 16);
        if (out.udp_checksum) out.udp_checksum[i] = (uint16_t)(d[1] & 0xFFFFu);
    }
}

// Packet i's start (byte offset in the slab) and length, clamped to the slab so that no read
// can leave the caller's allocation whatever the batch description says.
__device__ __forceinline__ void packet_range(const KParams& p, uint64_t i, uint64_t& off,
                                             uint32_t& len) {
    if (p.offsets) {
        off = p.offsets[i];
        len = p.lens[i];
    } else {
        off = i * (uint64_t)p.stride;
        len = p.lens ? p.lens[i] : p.stride;
    }
    uint64_t room = off < p.slab_len ? p.slab_len - off : 0;
    if ((uint64_t)len > room) len = (uint32_t)room;
    if (len > 0xFFFFu) len = 0xFFFFu;  // u16 offsets/lengths in the ABI
}

template <int NCH>
__global__ __launch_bounds__(kBlock) void parse_kernel(KParams p) {
    // (NCH + 1) chunk rows per wave: the extra row is slack so a window read of dword k+1 never
    // leaves this wave's region.
    __shared__ __attribute__((aligned(16))) uint8_t lds[kWavesPerBlock][(NCH + 1) * kChunkRow];
    const int lane = threadIdx.x & (kWave - 1);
    const int wv = threadIdx.x / kWave;
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    const bool active = i < p.n;

    uint64_t off = 0;
    uint32_t len = 0;
    if (active) packet_range(p, i, off, len);

    // ---- stage the first NCH*16 bytes (from the 16-byte-aligned start) of each packet
    const uint64_t gaddr = (uint64_t)(uintptr_t)p.slab + off;
    const uint64_t a0 = gaddr & ~(uint64_t)15;
    const uint32_t shift = (uint32_t)(gaddr - a0);
    const uint64_t slab_lo = (uint64_t)(uintptr_t)p.slab;
    const uint64_t slab_hi16 = (slab_lo + p.slab_len + 15) & ~(uint64_t)15;  // readable end
    uint8_t* win = &lds[wv][0];
#pragma unroll
    for (int c = 0; c < NCH; c++) {
        uint64_t src = a0 + 16u * (uint32_t)c;
        if (src + 16 > slab_hi16) src = slab_hi16 - 16;  // beyond the slab: any in-bounds chunk
        if (src < slab_lo) src = slab_lo;
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(src),
                                         (__attribute__((address_space(3))) void*)(win + c * kChunkRow),
                                         16, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

    PacketView pv;
    pv.lw = win + lane * 16;
    pv.gbase = p.slab + off;
    pv.shift = shift;
    uint32_t wend = (uint32_t)NCH * 16u - shift;
    pv.win_end = wend;
    pv.len = len;

    const pkt_out_t& out = p.out;
    const uint64_t n = p.n;
    auto push = [&](uint32_t slot, uint32_t t, uint32_t o) {
        if (out.hdr_type) out.hdr_type[(uint64_t)slot * n + i] = (uint8_t)t;
        if (out.hdr_off) out.hdr_off[(uint64_t)slot * n + i] = (uint16_t)o;
    };
    WalkResult r;
    walk(pv, entry_state(p.entry), active, push, r);
    if (!active) return;

    const bool ok = r.status == PKT_OK;
    if (out.status) out.status[i] = (uint8_t)r.status;
    if (out.n_hdrs) out.n_hdrs[i] = ok ? (uint8_t)r.n : (uint8_t)0;
    if (out.payload_off) out.payload_off[i] = ok ? (uint16_t)r.payload_off : (uint16_t)0;
    if (out.payload_len) out.payload_len[i] = ok ? (uint16_t)(len - r.payload_off) : (uint16_t)0;
    if (out.hdr_mask) out.hdr_mask[i] = ok ? r.mask : 0u;
    emit_fields(out, i, pv, r, ok);
}

// Batched `<Hdr>Slice::<field>()` (headers.rs:195-201 -> bit_range 252-263).
struct XParams {
    const uint8_t* slab;
    uint64_t slab_len;
    const uint64_t* offsets;
    const uint32_t* lens;
    uint32_t stride;
    uint64_t n;
    const uint8_t* n_hdrs;
    const uint8_t* hdr_type;
    const uint16_t* hdr_off;
    pkt_field_spec_t spec;
    uint64_t* values;
    uint8_t* found;
};

__global__ __launch_bounds__(256) void extract_kernel(XParams p) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= p.n) return;
    const uint32_t nh = p.n_hdrs[i];
    int hit = -1;
    uint32_t occ = 0;
    for (uint32_t j = 0; j < nh && j < PKT_MAX_HDRS; j++) {
        if (p.hdr_type[(uint64_t)j * p.n + i] == p.spec.hdr_type) {
            if (occ == p.spec.occurrence) { hit = (int)j; break; }
            occ++;
        }
    }
    uint64_t v = 0;
    if (hit >= 0) {
        uint64_t off;
        if (p.offsets) off = p.offsets[i];
        else off = i * (uint64_t)p.stride;
        const uint8_t* h = p.slab + off + p.hdr_off[(uint64_t)hit * p.n + i];
        const uint32_t start = p.spec.start, end = p.spec.end;
        const uint32_t w = end - start + 1;
        // bits [s2..end] hold the low 64 bits of the field; bit_range's release-build shifts
        // then keep the low (w mod 64, or 64) of them (headers.rs:262, Q8).
        const uint32_t s2 = w > 64 ? end - 63 : start;
        const uint32_t b0 = s2 >> 3, b1 = end >> 3;
        uint64_t acc = 0, top = 0;  // top = the byte shifted out when 9 bytes are spanned
        for (uint32_t b = b0; b <= b1; b++) {
            top = acc >> 56;
            acc = (acc << 8) | h[b];
        }
        const uint32_t r = 7 - (end & 7);
        uint64_t val = r ? ((acc >> r) | (top << (64 - r))) : acc;
        const uint32_t w2 = w > 64 ? (w & 63) : w;
        if (w2 != 0 && w2 < 64) val &= (1ull << w2) - 1;
        v = val;
    }
    p.values[i] = v;
    if (p.found) p.found[i] = hit >= 0 ? 1 : 0;
}

__global__ __launch_bounds__(256) void ipv4_csum_kernel(const uint8_t* hdrs, uint32_t stride, uint64_t n,
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

int fail(pkt_ctx* ctx, int code, const char* msg) {
    if (ctx) ctx->err = msg;
    return code;
}

int hip_fail(pkt_ctx* ctx, hipError_t e, const char* what) {
    if (ctx) ctx->err = std::string(what) + ": " + hipGetErrorString(e);
    return PKT_ERR_HIP;
}

template <int NCH>
hipError_t launch_parse(const KParams& kp, hipStream_t s) {
    dim3 grid((unsigned)((kp.n + kBlock - 1) / kBlock));
    hipLaunchKernelGGL(parse_kernel<NCH>, grid, dim3(kBlock), 0, s, kp);
    return hipGetLastError();
}

}  // namespace

extern "C" {

int pkt_ctx_create(int device, pkt_ctx_t** out) {
    if (!out) return PKT_ERR_INVALID_ARG;
    *out = nullptr;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count == 0) return PKT_ERR_NO_DEVICE;
    if (device < 0 || device >= count) return PKT_ERR_INVALID_ARG;
    pkt_ctx* c = new pkt_ctx();
    c->device = device;
    c->window = 0;
    *out = c;
    return PKT_SUCCESS;
}

int pkt_ctx_destroy(pkt_ctx_t* ctx) {
    delete ctx;
    return PKT_SUCCESS;
}

const char* pkt_ctx_last_error(const pkt_ctx_t* ctx) { return ctx ? ctx->err.c_str() : "null ctx"; }

int pkt_ctx_set_window(pkt_ctx_t* ctx, uint32_t w) {
    if (!ctx) return PKT_ERR_INVALID_ARG;
    ctx->window = w;
    return PKT_SUCCESS;
}

int pkt_parse_batch(pkt_ctx_t* ctx, const pkt_batch_t* b, int entry, const pkt_out_t* out,
                    void* stream) {
    if (!ctx || !b || !out) return fail(ctx, PKT_ERR_INVALID_ARG, "null argument");
    if (entry < 0 || entry >= PKT_ENTRY_COUNT) return fail(ctx, PKT_ERR_INVALID_ARG, "bad entry");
    if (b->n == 0) return PKT_SUCCESS;
    if (!b->slab) return fail(ctx, PKT_ERR_INVALID_ARG, "null slab");
    if (((uintptr_t)b->slab & 15) != 0) return fail(ctx, PKT_ERR_INVALID_ARG, "slab not 16-byte aligned");
    if (b->offsets && !b->lens) return fail(ctx, PKT_ERR_INVALID_ARG, "offsets without lens");
    if (!b->offsets && b->stride == 0) return fail(ctx, PKT_ERR_INVALID_ARG, "stride 0");
    if (out->ipv6_src && ((uintptr_t)out->ipv6_src & 15)) return fail(ctx, PKT_ERR_INVALID_ARG, "ipv6_src not 16-byte aligned");
    if (out->ipv6_dst && ((uintptr_t)out->ipv6_dst & 15)) return fail(ctx, PKT_ERR_INVALID_ARG, "ipv6_dst not 16-byte aligned");
    if (b->slab_len < 16) return fail(ctx, PKT_ERR_INVALID_ARG, "slab_len < 16");
    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) return hip_fail(ctx, e, "hipSetDevice");

    // Window: bytes of each packet staged in LDS.  Fixed stride: the slot (up to 128 B);
    // indexed: 128 B.  Unaligned packet starts need one more chunk.
    uint32_t w = ctx->window;
    if (w == 0) w = b->offsets ? 128u : std::min<uint32_t>(std::max<uint32_t>(b->stride, 16u), 128u);
    w = std::min<uint32_t>(std::max<uint32_t>((w + 15) & ~15u, 16u), 256u);
    bool aligned = !b->offsets && (b->stride % 16 == 0);
    int nch = (int)(w / 16) + (aligned ? 0 : 1);

    KParams kp;
    kp.slab = b->slab;
    kp.slab_len = b->slab_len;
    kp.offsets = b->offsets;
    kp.lens = b->lens;
    kp.stride = b->stride;
    kp.entry = entry;
    kp.n = b->n;
    kp.out = *out;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (nch <= 2) e = launch_parse<2>(kp, s);
    else if (nch <= 4) e = launch_parse<4>(kp, s);
    else if (nch <= 5) e = launch_parse<5>(kp, s);
    else if (nch <= 8) e = launch_parse<8>(kp, s);
    else if (nch <= 9) e = launch_parse<9>(kp, s);
    else if (nch <= 16) e = launch_parse<16>(kp, s);
    else e = launch_parse<17>(kp, s);
    if (e != hipSuccess) return hip_fail(ctx, e, "parse_kernel launch");
    return PKT_SUCCESS;
}

int pkt_extract_fields(pkt_ctx_t* ctx, const pkt_batch_t* b, const pkt_chain_t* chain,
                       const pkt_field_spec_t* specs, uint32_t nspec, uint64_t* const* values,
                       uint8_t* const* found, void* stream) {
    if (!ctx || !b || !chain || (nspec && (!specs || !values)))
        return fail(ctx, PKT_ERR_INVALID_ARG, "null argument");
    if (b->n == 0 || nspec == 0) return PKT_SUCCESS;
    if (!chain->n_hdrs || !chain->hdr_type || !chain->hdr_off || !b->slab)
        return fail(ctx, PKT_ERR_INVALID_ARG, "null chain column");
    if (b->offsets && !b->lens) return fail(ctx, PKT_ERR_INVALID_ARG, "offsets without lens");
    for (uint32_t s = 0; s < nspec; s++) {
        const pkt_field_spec_t& sp = specs[s];
        if (sp.hdr_type == 0 || sp.hdr_type >= PKT_HDR_COUNT || sp.end < sp.start ||
            sp.end >= 8 * pkt_hdr_size(sp.hdr_type) || !values[s])
            return fail(ctx, PKT_ERR_INVALID_ARG, "bad field spec");
    }
    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) return hip_fail(ctx, e, "hipSetDevice");
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    for (uint32_t s = 0; s < nspec; s++) {
        XParams xp;
        xp.slab = b->slab;
        xp.slab_len = b->slab_len;
        xp.offsets = b->offsets;
        xp.lens = b->lens;
        xp.stride = b->stride;
        xp.n = b->n;
        xp.n_hdrs = chain->n_hdrs;
        xp.hdr_type = chain->hdr_type;
        xp.hdr_off = chain->hdr_off;
        xp.spec = specs[s];
        xp.values = values[s];
        xp.found = found ? found[s] : nullptr;
        hipLaunchKernelGGL(extract_kernel, dim3((unsigned)((b->n + 255) / 256)), dim3(256), 0, st, xp);
        e = hipGetLastError();
        if (e != hipSuccess) return hip_fail(ctx, e, "extract_kernel launch");
    }
    return PKT_SUCCESS;
}

int pkt_ipv4_checksum_batch(pkt_ctx_t* ctx, const uint8_t* hdrs, uint32_t stride, uint64_t n,
                            uint16_t* out, void* stream) {
    if (!ctx || (n && (!hdrs || !out)) || (n && stride < 20)) return fail(ctx, PKT_ERR_INVALID_ARG, "bad argument");
    if (n == 0) return PKT_SUCCESS;
    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) return hip_fail(ctx, e, "hipSetDevice");
    hipLaunchKernelGGL(ipv4_csum_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), hdrs, stride, n, out);
    e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(ctx, e, "ipv4_csum_kernel launch");
    return PKT_SUCCESS;
}

}  // extern "C"
