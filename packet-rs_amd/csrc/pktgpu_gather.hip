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
