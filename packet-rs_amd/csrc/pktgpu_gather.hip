// pktgpu_gather.hip — the root-side repack of the merged multi-GPU gather (pkt_mgpu_parse_gather with
// merge = 1, pktgpu_mgpu.cpp).
//
// The merged result is ONE packed output of the whole batch: column c of shard i lands at packets
// [lo_i, lo_i + n_i) of column c (each used slot row likewise).  Sent as such over RCCL that is one
// message per column and slot row per shard (C2 at 8 x 2^21: 248 messages).  Instead the shards send
// their packed buffers as they are (<= 2 messages each, the merge = 0 transfer) into a staging area
// on the root, and this kernel places every (shard, column | slot row) piece in the whole-batch
// layout: a device-side copy of pieces whose (src, dst, bytes) the host lists in a table.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "pktgpu_ctx.hpp"

namespace {

constexpr uint32_t kRepackChunks = 1024;  // 16-byte destination chunks per block (16 KiB)

// Block j copies destination chunks [q * 1024, (q + 1) * 1024) of the piece p whose block range
// holds j (q = j - first_block[p]); block 0 of a piece also copies its unaligned head and tail
// bytes.  Chunks are 16-byte aligned in the DESTINATION: 16-byte loads when the source has the
// same alignment (every piece of equal shards), dword or byte loads otherwise.
__global__ __launch_bounds__(256) void repack_kernel(const RepackPiece* __restrict__ tab, uint32_t np) {
    // the piece of this block: the last one whose first block is <= blockIdx.x (wave-uniform search)
    uint32_t lo = 0, hi = np;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (tab[mid].first_block <= blockIdx.x) lo = mid;
        else hi = mid;
    }
    const RepackPiece pc = tab[lo];
    const uint32_t q = blockIdx.x - pc.first_block;
    const uint8_t* s = reinterpret_cast<const uint8_t*>(pc.src);
    uint8_t* d = reinterpret_cast<uint8_t*>(pc.dst);
    const uint64_t lead = (uint64_t)(-(int64_t)pc.dst) & 15u;
    const uint64_t head = lead < pc.bytes ? lead : pc.bytes;
    const uint64_t nb = (pc.bytes - head) >> 4;
    const uint64_t body_end = head + 16u * nb;
    const uint32_t t = threadIdx.x;
    if (q == 0) {
        if (t < head) d[t] = s[t];
        if (t < pc.bytes - body_end) d[body_end + t] = s[body_end + t];
    }
    const uint64_t c0 = (uint64_t)q * kRepackChunks, c1 = c0 + kRepackChunks < nb ? c0 + kRepackChunks : nb;
    const uint8_t* sb = s + head;
    uint4* db = reinterpret_cast<uint4*>(d + head);
    const uint32_t sal = (uint32_t)(reinterpret_cast<uintptr_t>(sb) & 15u);
    if (sal == 0) {
        uint4 v[4];
#pragma unroll
        for (uint32_t u = 0; u < 4; u++) {
            const uint64_t c = c0 + t + 256u * u;
            if (c < c1) v[u] = reinterpret_cast<const uint4*>(sb)[c];
        }
#pragma unroll
        for (uint32_t u = 0; u < 4; u++) {
            const uint64_t c = c0 + t + 256u * u;
            if (c < c1) db[c] = v[u];
        }
    } else if ((sal & 3u) == 0) {
        for (uint64_t c = c0 + t; c < c1; c += 256u) {
            const uint32_t* w = reinterpret_cast<const uint32_t*>(sb + 16u * c);
            db[c] = make_uint4(w[0], w[1], w[2], w[3]);
        }
    } else {
        for (uint64_t c = c0 + t; c < c1; c += 256u) {
            uint32_t w[4];
            const uint8_t* b = sb + 16u * c;
#pragma unroll
            for (int k = 0; k < 4; k++)
                w[k] = (uint32_t)b[4 * k] | ((uint32_t)b[4 * k + 1] << 8) | ((uint32_t)b[4 * k + 2] << 16) |
                       ((uint32_t)b[4 * k + 3] << 24);
            db[c] = make_uint4(w[0], w[1], w[2], w[3]);
        }
    }
}

}  // namespace

uint32_t pktgpu_repack_blocks(uint64_t bytes) {
    const uint64_t b = (bytes + 16ull * kRepackChunks - 1) / (16ull * kRepackChunks);
    return (uint32_t)(b ? b : 1);
}

hipError_t pktgpu_repack_launch(const RepackPiece* tab_dev, uint32_t np, uint32_t nblocks, hipStream_t s) {
    if (!np || !nblocks) return hipSuccess;
    hipLaunchKernelGGL(repack_kernel, dim3(nblocks), dim3(256), 0, s, tab_dev, np);
    return hipGetLastError();
}

// ---- the capture-in-host-memory path's column export (pkt_parse_pcap_host, pktgpu.hip) ----
// A piece's records [lo, hi) (device words: the prefix counts) were parsed into DEVICE columns laid out
// like the caller's host columns (same element size, slot rows strided by cap); this kernel copies each
// column's range [lo, hi) — each slot row's below the piece's largest n_hdrs — into the caller's pinned
// host columns over the link.  16-byte chunks by consecutive lanes, so a wave instruction writes 1 KiB
// of one column: the parse's own per-lane stores to host memory (1-8 B per lane, 64-512 B per wave
// instruction) moved the columns at ~21 GB/s, a copy of wide chunks at the link's rate (~57 GB/s,
// profiles/host/r05b_pcap_host_pieces.jsonl).  Block (x, y): part x of column range y.
namespace {
__global__ __launch_bounds__(256) void export_kernel(ExportArgs a) {
    const ExportCol c = a.col[blockIdx.y];
    uint64_t hi = a.hi_dev ? *a.hi_dev : a.hi_h, lo = a.hi_dev ? (a.lo_dev ? *a.lo_dev : 0) : a.lo_h;
    hi = hi < a.cap ? hi : a.cap;
    lo = lo < hi ? lo : hi;
    const uint32_t t = threadIdx.x;
    if (c.row != kExportNoRow && a.nhw) {  // a slot row: only below the largest n_hdrs (256 spread words)
        __shared__ uint32_t s_max[4];
        uint32_t m = a.nhw[t];
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, d, 64));
        if ((t & 63u) == 0) s_max[t >> 6] = m;
        __syncthreads();
        m = max(max(s_max[0], s_max[1]), max(s_max[2], s_max[3]));
        if (c.row >= m) return;
    }
    const uint64_t bytes = (hi - lo) * c.sz;
    if (!bytes) return;
    const uint8_t* s = reinterpret_cast<const uint8_t*>(c.src) + lo * c.sz;
    uint8_t* d = reinterpret_cast<uint8_t*>(c.dst) + lo * c.sz;
    const uint64_t lead = (uint64_t)(-(int64_t)reinterpret_cast<uintptr_t>(d)) & 15u;
    const uint64_t head = lead < bytes ? lead : bytes;
    const uint64_t nb = (bytes - head) >> 4, body_end = head + 16u * nb;
    if (blockIdx.x == 0) {
        if (t < head) d[t] = s[t];
        if (t < bytes - body_end) d[body_end + t] = s[body_end + t];
    }
    const uint8_t* sb = s + head;
    uint4* db = reinterpret_cast<uint4*>(d + head);
    const uint64_t step = (uint64_t)gridDim.x * 256u;
    if ((reinterpret_cast<uintptr_t>(sb) & 15u) == 0) {
        for (uint64_t k = (uint64_t)blockIdx.x * 256u + t; k < nb; k += 2 * step) {
            const uint4 v0 = reinterpret_cast<const uint4*>(sb)[k];
            const bool two = k + step < nb;
            uint4 v1 = v0;
            if (two) v1 = reinterpret_cast<const uint4*>(sb)[k + step];
            db[k] = v0;
            if (two) db[k + step] = v1;
        }
    } else {
        for (uint64_t k = (uint64_t)blockIdx.x * 256u + t; k < nb; k += step) {
            uint32_t w[4];
            const uint8_t* b = sb + 16u * k;
#pragma unroll
            for (int q = 0; q < 4; q++)
                w[q] = (uint32_t)b[4 * q] | ((uint32_t)b[4 * q + 1] << 8) | ((uint32_t)b[4 * q + 2] << 16) |
                       ((uint32_t)b[4 * q + 3] << 24);
            db[k] = make_uint4(w[0], w[1], w[2], w[3]);
        }
    }
}
}  // namespace

hipError_t pktgpu_export_launch(const ExportArgs& a, hipStream_t s) {
    if (!a.ncol) return hipSuccess;
    hipLaunchKernelGGL(export_kernel, dim3(kExportParts, a.ncol), dim3(256), 0, s, a);
    return hipGetLastError();
}
