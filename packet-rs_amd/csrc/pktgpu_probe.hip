// pktgpu_probe.hip — measurement probe for bench.py (lib/libpktprobe.so; NOT part of the product
// ABI and never called by it).
//
// pkt_probe_ceiling: the "ceiling" kernel of the roofline line.  Same launch shape as the C2
// parse launch (256-thread blocks, one packet per lane, grid = n / 256) and the SAME HBM traffic
// — each lane loads its packet's first 64 bytes with four 16-byte loads and stores the C2 bench
// tuple (chain with 3 slots + Ether + IPv4 + UDP = 69 B) into the same pkt_out_t columns with
// the same per-lane store widths — but no walk and no field logic: every stored value is a cheap
// mix of the loaded words.  Its launch time is what ANY kernel with C2's traffic shape costs in
// one launch on this box, so parse / ceiling says how much of the gap to the HBM peak is the
// parser's own.  pkt_probe_ceiling_groups: the same for the C3 column set (bench.py --config c3).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/pktgpu.h"

namespace {

template <class T>
__device__ __forceinline__ void put(T* base, uint32_t i, T v) { base[i] = v; }

__global__ __launch_bounds__(256) void ceiling_kernel(const uint8_t* slab, uint32_t n, uint32_t stride,
                                                      pkt_out_t o) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n) return;
    const uint4* p = reinterpret_cast<const uint4*>(slab + (uint64_t)i * stride);
    const uint4 a = p[0], b = p[1], c = p[2], d = p[3];
    const uint32_t v0 = a.x ^ d.w, v1 = a.y ^ c.z, v2 = a.z ^ b.y, v3 = a.w ^ c.x;
    const uint32_t v4 = b.x ^ d.x, v5 = b.z ^ c.y, v6 = b.w ^ d.y, v7 = c.w ^ d.z;
    // chain: status, n_hdrs, 3 header slots (type, offset), payload, mask
    put<uint8_t>(o.status, i, (uint8_t)(v0 & 1));
    put<uint8_t>(o.n_hdrs, i, (uint8_t)(3 + (v1 & 1)));
#pragma unroll
    for (uint32_t j = 0; j < 3; j++) {
        put<uint8_t>(o.hdr_type, j * n + i, (uint8_t)(v2 >> (8 * j)));
        put<uint16_t>(o.hdr_off, j * n + i, (uint16_t)(v3 >> (5 * j)));
    }
    put<uint16_t>(o.payload_off, i, (uint16_t)v4);
    put<uint16_t>(o.payload_len, i, (uint16_t)(v4 >> 16));
    put<uint32_t>(o.hdr_mask, i, v5);
    // Ether
    put<uint64_t>(o.eth_dst, i, ((uint64_t)a.x << 16) | (a.y >> 16));
    put<uint64_t>(o.eth_src, i, ((uint64_t)a.y << 32) | a.z);
    put<uint16_t>(o.eth_etype, i, (uint16_t)a.w);
    // IPv4
    put<uint8_t>(o.ipv4_version, i, (uint8_t)(v6 >> 4));
    put<uint8_t>(o.ipv4_ihl, i, (uint8_t)v6);
    put<uint8_t>(o.ipv4_diffserv, i, (uint8_t)(v6 >> 8));
    put<uint16_t>(o.ipv4_total_len, i, (uint16_t)(v6 >> 16));
    put<uint16_t>(o.ipv4_identification, i, (uint16_t)v7);
    put<uint8_t>(o.ipv4_flags, i, (uint8_t)(v7 >> 29));
    put<uint16_t>(o.ipv4_frag_startset, i, (uint16_t)(v7 >> 16));
    put<uint8_t>(o.ipv4_ttl, i, (uint8_t)(b.x >> 8));
    put<uint8_t>(o.ipv4_protocol, i, (uint8_t)b.x);
    put<uint16_t>(o.ipv4_header_checksum, i, (uint16_t)(b.y >> 16));
    put<uint32_t>(o.ipv4_src, i, b.z);
    put<uint32_t>(o.ipv4_dst, i, b.w);
    put<uint16_t>(o.ipv4_csum_calc, i, (uint16_t)(v0 + v1 + v2 + v3));
    // UDP
    put<uint16_t>(o.udp_src, i, (uint16_t)c.x);
    put<uint16_t>(o.udp_dst, i, (uint16_t)(c.x >> 16));
    put<uint16_t>(o.udp_length, i, (uint16_t)c.y);
    put<uint16_t>(o.udp_checksum, i, (uint16_t)(c.y >> 16));
}

// The C3 form (pkt_probe_ceiling_groups): the same loads, and stores into EVERY requested column of
// the chain (`slots` header slots), Ether, Vlan, IPv4, TCP and UDP groups with the parse's widths
// (a group is written when its first column is non-NULL; the parse writes absent groups as zeros).
__global__ __launch_bounds__(256) void ceiling_groups_kernel(const uint8_t* slab, uint32_t n, uint32_t stride,
                                                             uint32_t slots, pkt_out_t o) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n) return;
    const uint4* p = reinterpret_cast<const uint4*>(slab + (uint64_t)i * stride);
    const uint4 a = p[0], b = p[1], c = p[2], d = p[3];
    const uint32_t v0 = a.x ^ d.w, v1 = a.y ^ c.z, v2 = a.z ^ b.y, v3 = a.w ^ c.x;
    const uint32_t v4 = b.x ^ d.x, v5 = b.z ^ c.y, v6 = b.w ^ d.y, v7 = c.w ^ d.z;
    put<uint8_t>(o.status, i, (uint8_t)(v0 & 1));
    put<uint8_t>(o.n_hdrs, i, (uint8_t)(3 + (v1 & 1)));
    for (uint32_t j = 0; j < slots; j++) {
        put<uint8_t>(o.hdr_type, j * n + i, (uint8_t)(v2 >> (8 * (j & 3))));
        put<uint16_t>(o.hdr_off, j * n + i, (uint16_t)(v3 >> (5 * (j & 3))));
    }
    put<uint16_t>(o.payload_off, i, (uint16_t)v4);
    put<uint16_t>(o.payload_len, i, (uint16_t)(v4 >> 16));
    put<uint32_t>(o.hdr_mask, i, v5);
    if (o.eth_dst) {
        put<uint64_t>(o.eth_dst, i, ((uint64_t)a.x << 16) | (a.y >> 16));
        put<uint64_t>(o.eth_src, i, ((uint64_t)a.y << 32) | a.z);
        put<uint16_t>(o.eth_etype, i, (uint16_t)a.w);
    }
    if (o.vlan_pcp) {
        put<uint8_t>(o.vlan_pcp, i, (uint8_t)(b.x >> 29));
        put<uint8_t>(o.vlan_cfi, i, (uint8_t)(b.x >> 28));
        put<uint16_t>(o.vlan_vid, i, (uint16_t)(b.x >> 16));
        put<uint16_t>(o.vlan_etype, i, (uint16_t)b.x);
    }
    if (o.ipv4_version) {
        put<uint8_t>(o.ipv4_version, i, (uint8_t)(v6 >> 4));
        put<uint8_t>(o.ipv4_ihl, i, (uint8_t)v6);
        put<uint8_t>(o.ipv4_diffserv, i, (uint8_t)(v6 >> 8));
        put<uint16_t>(o.ipv4_total_len, i, (uint16_t)(v6 >> 16));
        put<uint16_t>(o.ipv4_identification, i, (uint16_t)v7);
        put<uint8_t>(o.ipv4_flags, i, (uint8_t)(v7 >> 29));
        put<uint16_t>(o.ipv4_frag_startset, i, (uint16_t)(v7 >> 16));
        put<uint8_t>(o.ipv4_ttl, i, (uint8_t)(b.x >> 8));
        put<uint8_t>(o.ipv4_protocol, i, (uint8_t)b.x);
        put<uint16_t>(o.ipv4_header_checksum, i, (uint16_t)(b.y >> 16));
        put<uint32_t>(o.ipv4_src, i, b.z);
        put<uint32_t>(o.ipv4_dst, i, b.w);
        put<uint16_t>(o.ipv4_csum_calc, i, (uint16_t)(v0 + v1 + v2 + v3));
    }
    if (o.tcp_src) {
        put<uint16_t>(o.tcp_src, i, (uint16_t)c.z);
        put<uint16_t>(o.tcp_dst, i, (uint16_t)(c.z >> 16));
        put<uint32_t>(o.tcp_seq_no, i, c.w ^ v0);
        put<uint32_t>(o.tcp_ack_no, i, d.x ^ v1);
        put<uint8_t>(o.tcp_data_startset, i, (uint8_t)(d.y >> 28));
        put<uint8_t>(o.tcp_res, i, (uint8_t)(d.y >> 24));
        put<uint8_t>(o.tcp_flags, i, (uint8_t)(d.y >> 16));
        put<uint16_t>(o.tcp_window, i, (uint16_t)d.y);
        put<uint16_t>(o.tcp_checksum, i, (uint16_t)(d.z >> 16));
        put<uint16_t>(o.tcp_urgent_ptr, i, (uint16_t)d.z);
    }
    if (o.udp_src) {
        put<uint16_t>(o.udp_src, i, (uint16_t)c.x);
        put<uint16_t>(o.udp_dst, i, (uint16_t)(c.x >> 16));
        put<uint16_t>(o.udp_length, i, (uint16_t)c.y);
        put<uint16_t>(o.udp_checksum, i, (uint16_t)(c.y >> 16));
    }
}

}  // namespace

extern "C" int pkt_probe_ceiling_groups(const uint8_t* slab, uint64_t n, uint32_t stride, uint32_t slots,
                                        const pkt_out_t* out, void* stream) {
    // every column of each written group present (chain always; a group by its first column)
    if (!slab || !out || n == 0 || n >= (1ull << 26) || stride < 64 || (stride & 15) || slots > PKT_MAX_HDRS)
        return PKT_ERR_INVALID_ARG;
    const void* const* cols = reinterpret_cast<const void* const*>(out);
    static const int lo[7] = {0, 7, 10, 14, 27, 35, 45}, hi[7] = {7, 10, 14, 27, 35, 45, 49};
    for (int g = 0; g < 7; g++) {
        if (g == 4 && cols[lo[g]]) return PKT_ERR_INVALID_ARG;  // IPv6: not part of any probe shape
        if (g > 0 && !cols[lo[g]]) continue;
        for (int c = lo[g]; c < hi[g]; c++)
            if (!cols[c]) return PKT_ERR_INVALID_ARG;
    }
    hipLaunchKernelGGL(ceiling_groups_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), slab, (uint32_t)n, stride, slots, *out);
    return hipGetLastError() == hipSuccess ? PKT_SUCCESS : PKT_ERR_HIP;
}

extern "C" int pkt_probe_ceiling(const uint8_t* slab, uint64_t n, uint32_t stride, const pkt_out_t* out,
                                 void* stream) {
    // The probe stores the C2 bench set only; every one of its columns must be present.
    if (!slab || !out || n == 0 || n >= (1ull << 26) || stride < 64 || (stride & 15)) return PKT_ERR_INVALID_ARG;
    // pkt_out_t members 0-9 (chain, Ether), 14-26 (IPv4) and 45-48 (UDP)
    const void* const* cols = reinterpret_cast<const void* const*>(out);
    for (int c = 0; c < 49; c++) {
        const bool need = c < 10 || (c >= 14 && c < 27) || c >= 45;
        if (need && !cols[c]) return PKT_ERR_INVALID_ARG;
    }
    hipLaunchKernelGGL(ceiling_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), slab, (uint32_t)n, stride, *out);
    return hipGetLastError() == hipSuccess ? PKT_SUCCESS : PKT_ERR_HIP;
}

// pkt_probe_fetch: FETCH_SIZE calibration for per-lane scattered reads (the access shape of the
// indexed-batch windows).  Item i (one lane) reads `width` bytes (16-byte loads) at
// buf + i * stride + phase and writes one word, so with stride >= 256 every item touches its own
// lines: FETCH_SIZE per item says at which granularity (64-B sector or 128-B line) the memory-side
// requests of this shape are counted.
namespace {
__global__ __launch_bounds__(256) void fetch_kernel(const uint8_t* buf, uint32_t n, uint32_t stride, uint32_t phase,
                                                    uint32_t width, uint32_t* out) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n) return;
    const uint4* p = reinterpret_cast<const uint4*>(buf + (uint64_t)i * stride + phase);
    uint32_t acc = 0;
    for (uint32_t c = 0; c < width / 16; c++) {
        const uint4 v = p[c];
        acc ^= v.x + v.y * 3u + v.z * 5u + v.w * 7u;
    }
    out[i] = acc;
}
}  // namespace

extern "C" int pkt_probe_fetch(const uint8_t* buf, uint64_t buf_len, uint32_t n, uint32_t stride, uint32_t phase,
                               uint32_t width, uint32_t* out, void* stream) {
    if (!buf || !out || !n || (phase & 15) || (width & 15) || width == 0 ||
        (uint64_t)(n - 1) * stride + phase + width > buf_len)
        return PKT_ERR_INVALID_ARG;
    hipLaunchKernelGGL(fetch_kernel, dim3((n + 255) / 256), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), buf,
                       n, stride, phase, width, out);
    return hipGetLastError() == hipSuccess ? PKT_SUCCESS : PKT_ERR_HIP;
}

// pkt_probe_c4load: the load shape of the indexed-batch parse without the walk.  Lane i loads `nch`
// 16-byte chunks from offsets[i] rounded down to 2^align_log2 bytes (clamped to the slab) and writes
// one byte.  Its time per launch is what the window loads alone cost for a given window placement.
namespace {
__global__ __launch_bounds__(256) void c4load_kernel(const uint8_t* slab, uint64_t slab_len, const uint64_t* offs,
                                                     uint32_t n, uint32_t nch, uint32_t align_log2, uint8_t* out) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n) return;
    const uint64_t last16 = ((slab_len + 15) & ~(uint64_t)15) - 16;
    const uint64_t a0 = offs[i] & ~((1ull << align_log2) - 1ull);
    uint32_t acc = 0;
    for (uint32_t c = 0; c < nch; c++) {
        uint64_t a = a0 + 16u * c;
        a = a > last16 ? last16 : a;
        const uint4 v = *reinterpret_cast<const uint4*>(slab + a);
        acc ^= v.x + v.y * 3u + v.z * 5u + v.w * 7u;
    }
    out[i] = (uint8_t)acc;
}
}  // namespace

extern "C" int pkt_probe_c4load(const uint8_t* slab, uint64_t slab_len, const uint64_t* offs, uint32_t n, uint32_t nch,
                                uint32_t align_log2, uint8_t* out, void* stream) {
    if (!slab || !offs || !out || !n || slab_len < 16 || align_log2 < 4 || align_log2 > 8 || nch == 0 || nch > 32)
        return PKT_ERR_INVALID_ARG;
    hipLaunchKernelGGL(c4load_kernel, dim3((n + 255) / 256), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), slab,
                       slab_len, offs, n, nch, align_log2, out);
    return hipGetLastError() == hipSuccess ? PKT_SUCCESS : PKT_ERR_HIP;
}

// pkt_probe_stream_copy: the streaming-copy ceiling of the C2 roofline (bench.py roofline.ceiling
// .stream_copy).  A hand-written copy with the parse's BYTES but the ideal access shape: batch b
// reads read_bytes from srcs[b] and writes write_bytes to dsts[b] (the chunks past read_bytes are
// derived from their index), every access a 16-byte global_load_dwordx4 / global_store_dwordx4 by
// consecutive lanes (1 KiB contiguous per wave instruction), four loads in flight per lane before
// the first store.  k batches in one launch (block j serves batch j / bpb), so the k = 1 launch and
// the k = 16 launch are the copy forms of the parse's one-batch and pkt_parse_batches launches.
namespace {
constexpr int kCopyMax = 16;
constexpr uint32_t kCopyU = 4;  // 16-byte chunks per lane
struct CopyArgs {
    const uint4* src[kCopyMax];
    uint4* dst[kCopyMax];
    uint64_t nr, nw;  // 16-byte chunks read / written per batch
    uint32_t bpb;     // blocks per batch
};
__global__ __launch_bounds__(256) void stream_copy_kernel(CopyArgs a) {
    const uint32_t b = blockIdx.x / a.bpb;
    const uint64_t c0 = (uint64_t)(blockIdx.x - b * a.bpb) * (256u * kCopyU) + threadIdx.x;
    const uint4* __restrict__ s = a.src[b];
    uint4* __restrict__ d = a.dst[b];
    uint4 v[kCopyU];
#pragma unroll
    for (uint32_t u = 0; u < kCopyU; u++) {
        const uint64_t c = c0 + 256u * u;
        v[u] = c < a.nr ? s[c] : make_uint4((uint32_t)c, (uint32_t)(c >> 32), 0u, 0u);
    }
#pragma unroll
    for (uint32_t u = 0; u < kCopyU; u++) {
        const uint64_t c = c0 + 256u * u;
        if (c < a.nw) d[c] = v[u];
    }
}
}  // namespace

extern "C" int pkt_probe_stream_copy(const uint8_t* const* srcs, uint8_t* const* dsts, uint32_t k, uint64_t read_bytes,
                                     uint64_t write_bytes, void* stream) {
    if (!srcs || !dsts || k == 0 || k > (uint32_t)kCopyMax || (read_bytes & 15) || (write_bytes & 15) ||
        (read_bytes == 0 && write_bytes == 0))
        return PKT_ERR_INVALID_ARG;
    CopyArgs a;
    for (uint32_t b = 0; b < (uint32_t)kCopyMax; b++) {
        const uint32_t q = b < k ? b : 0;
        if (((uintptr_t)srcs[q] & 15) || ((uintptr_t)dsts[q] & 15) || !srcs[q] || !dsts[q]) return PKT_ERR_INVALID_ARG;
        a.src[b] = reinterpret_cast<const uint4*>(srcs[q]);
        a.dst[b] = reinterpret_cast<uint4*>(dsts[q]);
    }
    a.nr = read_bytes / 16;
    a.nw = write_bytes / 16;
    const uint64_t nc = a.nr > a.nw ? a.nr : a.nw;
    const uint64_t bpb = (nc + 256u * kCopyU - 1) / (256u * kCopyU);
    if (bpb * k >= (1ull << 31)) return PKT_ERR_INVALID_ARG;
    a.bpb = (uint32_t)bpb;
    hipLaunchKernelGGL(stream_copy_kernel, dim3((unsigned)(bpb * k)), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), a);
    return hipGetLastError() == hipSuccess ? PKT_SUCCESS : PKT_ERR_HIP;
}
