// probe.hip — read-path probes for the 64-byte-packet slab (not part of the product).
// Each kernel reads n packets x 64 B and writes one u32 per packet (a checksum of its bytes),
// so that every variant moves the same bytes; they differ only in how the slab is read.
#include <hip/hip_runtime.h>
#include <stdint.h>

#define LDS_AS __attribute__((address_space(3)))

__device__ __forceinline__ uint32_t mix(uint4 a) { return a.x ^ (a.y * 3u) ^ (a.z * 5u) ^ (a.w * 7u); }

// A: LDS-DMA, per-lane gather (lane l loads chunk c of ITS packet): chunk-major LDS.
__global__ __launch_bounds__(256) void k_dma_gather(const uint8_t* slab, uint32_t n, uint32_t* out) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[4][5 * 1024];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    const uint8_t* p = slab + (uint64_t)min(i, n - 1) * 64;
    for (int c = 0; c < 4; c++)
        __builtin_amdgcn_global_load_lds((const void*)(p + 16 * c), (LDS_AS void*)(&lds[wv][c * 1024]), 16, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    uint32_t h = 0;
    for (int c = 0; c < 4; c++) h ^= mix(*(const uint4*)&lds[wv][c * 1024 + lane * 16]) + c;
    if (i < n) out[i] = h;
}

// B: LDS-DMA, contiguous 1 KiB per instruction: packet-major LDS.
__global__ __launch_bounds__(256) void k_dma_contig(const uint8_t* slab, uint32_t n, uint32_t* out) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[4][5 * 1024];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t wave0 = (blockIdx.x * 256u + wv * 64u);  // first packet of this wave
    const uint8_t* base = slab + (uint64_t)wave0 * 64;
    const uint64_t lim = (uint64_t)n * 64 - 16;
    for (int c = 0; c < 4; c++) {
        uint64_t o = (uint64_t)wave0 * 64 + c * 1024 + lane * 16;
        if (o > lim) o = lim;
        __builtin_amdgcn_global_load_lds((const void*)(slab + o), (LDS_AS void*)(&lds[wv][c * 1024]), 16, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    (void)base;
    const uint32_t i = wave0 + lane;
    uint32_t h = 0;
    for (int c = 0; c < 4; c++) h ^= mix(*(const uint4*)&lds[wv][lane * 64 + c * 16]) + c;
    if (i < n) out[i] = h;
}

// C: registers, per-lane strided dwordx4 (each lane reads its own 64 B).
__global__ __launch_bounds__(256) void k_reg_strided(const uint8_t* slab, uint32_t n, uint32_t* out) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    const uint4* p = (const uint4*)(slab + (uint64_t)min(i, n - 1) * 64);
    uint4 a = p[0], b = p[1], c = p[2], d = p[3];
    uint32_t h = mix(a) ^ (mix(b) + 1) ^ (mix(c) + 2) ^ (mix(d) + 3);
    if (i < n) out[i] = h;
}

// D: registers, coalesced (lane l reads 16 B at l*16 of each 1 KiB), no per-packet meaning.
__global__ __launch_bounds__(256) void k_reg_contig(const uint8_t* slab, uint32_t n, uint32_t* out) {
    const uint32_t wv = blockIdx.x * 4u + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    const uint4* p = (const uint4*)(slab + (uint64_t)wv * 4096);
    uint64_t lim = (uint64_t)n * 4;  // uint4 count
    uint32_t h = 0;
    for (int c = 0; c < 4; c++) {
        uint64_t k = (uint64_t)wv * 256 + c * 64 + lane;
        if (k < lim) h ^= mix(p[c * 64 + lane]) + c;
    }
    const uint32_t i = wv * 64 + lane;
    if (i < n) out[i] = h;
}

// E: persistent LDS-DMA gather, double-buffered, grid-stride over tiles of 64 packets.
__global__ __launch_bounds__(256) void k_dma_persist(const uint8_t* slab, uint32_t n, uint32_t* out) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[4][2][4 * 1024];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t ntiles = (n + 63) / 64;
    const uint32_t gw = blockIdx.x * 4 + wv, nw = gridDim.x * 4;
    uint32_t t = gw;
    int buf = 0;
    auto issue = [&](uint32_t tt, int b) {
        uint32_t i = tt * 64 + lane;
        const uint8_t* p = slab + (uint64_t)min(i, n - 1) * 64;
        for (int c = 0; c < 4; c++)
            __builtin_amdgcn_global_load_lds((const void*)(p + 16 * c), (LDS_AS void*)(&lds[wv][b][c * 1024]), 16, 0, 0);
    };
    if (t < ntiles) issue(t, 0);
    for (; t < ntiles; t += nw) {
        const uint32_t tn = t + nw;
        if (tn < ntiles) {
            issue(tn, buf ^ 1);
            asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        uint32_t h = 0;
        for (int c = 0; c < 4; c++) h ^= mix(*(const uint4*)&lds[wv][buf][c * 1024 + lane * 16]) + c;
        const uint32_t i = t * 64 + lane;
        if (i < n) out[i] = h;
        buf ^= 1;
    }
}

extern "C" int probe_launch(int which, const uint8_t* slab, uint32_t n, uint32_t* out, int grid_persist,
                            void* stream) {
    hipStream_t s = (hipStream_t)stream;
    unsigned grid = (n + 255) / 256;
    switch (which) {
        case 0: hipLaunchKernelGGL(k_dma_gather, dim3(grid), dim3(256), 0, s, slab, n, out); break;
        case 1: hipLaunchKernelGGL(k_dma_contig, dim3(grid), dim3(256), 0, s, slab, n, out); break;
        case 2: hipLaunchKernelGGL(k_reg_strided, dim3(grid), dim3(256), 0, s, slab, n, out); break;
        case 3: hipLaunchKernelGGL(k_reg_contig, dim3(grid), dim3(256), 0, s, slab, n, out); break;
        case 4: hipLaunchKernelGGL(k_dma_persist, dim3(grid_persist), dim3(256), 0, s, slab, n, out); break;
        default: return -1;
    }
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

// ---- write-path probes: read 64 B/packet (registers), write the C2 tuple layout (31 columns,
// 69 B/packet) either (F) with per-lane stores, or (G) staged through LDS and written as
// 16-byte chunks per lane.
struct Cols { void* p[31]; };
__constant__ int kColSize[31] = {1,1,1,1,1,1,1,1,1,1,1, 2,2,2,2,2,2,2,2,2,2,2,2,2,2,2, 4,4,4, 8,8};

__global__ __launch_bounds__(256) void k_write_lane(const uint8_t* slab, uint32_t n, Cols c) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    const uint4* p = (const uint4*)(slab + (uint64_t)min(i, n - 1) * 64);
    uint4 a = p[0], b = p[1], cc = p[2], d = p[3];
    uint32_t v[8] = {a.x, a.y ^ b.x, a.z ^ b.y, a.w ^ b.z, cc.x ^ b.w, cc.y ^ d.x, cc.z ^ d.y, cc.w ^ d.z};
    if (i >= n) return;
#pragma unroll
    for (int k = 0; k < 11; k++) ((uint8_t*)c.p[k])[i] = (uint8_t)(v[k & 7] >> k);
#pragma unroll
    for (int k = 11; k < 26; k++) ((uint16_t*)c.p[k])[i] = (uint16_t)(v[k & 7] >> (k & 15));
#pragma unroll
    for (int k = 26; k < 29; k++) ((uint32_t*)c.p[k])[i] = v[k & 7] + k;
#pragma unroll
    for (int k = 29; k < 31; k++) ((uint64_t*)c.p[k])[i] = ((uint64_t)v[k & 7] << 16) ^ v[(k + 1) & 7];
}

__global__ __launch_bounds__(256) void k_write_lds(const uint8_t* slab, uint32_t n, Cols c) {
    // per wave: 69 * 64 = 4416 B of column segments in LDS, column k at segoff[k]
    __shared__ __attribute__((aligned(16))) uint8_t st[4][4416];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    const uint32_t wave0 = i - lane;
    const uint4* p = (const uint4*)(slab + (uint64_t)min(i, n - 1) * 64);
    uint4 a = p[0], b = p[1], cc = p[2], d = p[3];
    uint32_t v[8] = {a.x, a.y ^ b.x, a.z ^ b.y, a.w ^ b.z, cc.x ^ b.w, cc.y ^ d.x, cc.z ^ d.y, cc.w ^ d.z};
    uint8_t* S = st[wv];
#pragma unroll
    for (int k = 0; k < 11; k++) S[k * 64 + lane] = (uint8_t)(v[k & 7] >> k);
#pragma unroll
    for (int k = 11; k < 26; k++) ((uint16_t*)(S + 704 + (k - 11) * 128))[lane] = (uint16_t)(v[k & 7] >> (k & 15));
#pragma unroll
    for (int k = 26; k < 29; k++) ((uint32_t*)(S + 2624 + (k - 26) * 256))[lane] = v[k & 7] + k;
#pragma unroll
    for (int k = 29; k < 31; k++) ((uint64_t*)(S + 3392 + (k - 29) * 512))[lane] = ((uint64_t)v[k & 7] << 16) ^ v[(k + 1) & 7];
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): own wave's LDS writes done
    __builtin_amdgcn_wave_barrier();
    // 276 16-byte chunks: lane j handles chunks j, j+64, ...
    for (int ch = lane; ch < 276; ch += 64) {
        int k, rel;
        uint32_t seg = ch * 16;
        if (seg < 704) { k = seg / 64; rel = seg - k * 64; }
        else if (seg < 2624) { k = 11 + (seg - 704) / 128; rel = (seg - 704) % 128; }
        else if (seg < 3392) { k = 26 + (seg - 2624) / 256; rel = (seg - 2624) % 256; }
        else { k = 29 + (seg - 3392) / 512; rel = (seg - 3392) % 512; }
        uint8_t* dst = (uint8_t*)c.p[k] + (uint64_t)wave0 * kColSize[k] + rel;
        if (wave0 + 64 <= n) *(uint4*)dst = *(const uint4*)(S + seg);
    }
}

extern "C" int probe_write(int which, const uint8_t* slab, uint32_t n, void* const* cols, void* stream) {
    Cols c;
    for (int k = 0; k < 31; k++) c.p[k] = cols[k];
    hipStream_t s = (hipStream_t)stream;
    unsigned grid = (n + 255) / 256;
    if (which == 0) hipLaunchKernelGGL(k_write_lane, dim3(grid), dim3(256), 0, s, slab, n, c);
    else hipLaunchKernelGGL(k_write_lds, dim3(grid), dim3(256), 0, s, slab, n, c);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

// H: read the first `rd` bytes (multiple of 16, <= 64) of each `stride`-byte slot.
__global__ __launch_bounds__(256) void k_read_prefix(const uint8_t* slab, uint32_t n, uint32_t stride, uint32_t rd, uint32_t* out) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    const uint4* p = (const uint4*)(slab + (uint64_t)min(i, n - 1) * stride);
    uint32_t h = 0;
    for (uint32_t c = 0; c < rd / 16; c++) h ^= mix(p[c]) + c;
    if (i < n) out[i] = h;
}
extern "C" int probe_prefix(const uint8_t* slab, uint32_t n, uint32_t stride, uint32_t rd, uint32_t* out, void* stream) {
    hipLaunchKernelGGL(k_read_prefix, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, slab, n, stride, rd, out);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
