// probe_store.hip — store-shape probes for the C2 tuple (not part of the product).
// Every kernel reads n packets x 64 B and writes 31 columns (11 u8, 15 u16, 3 u32, 2 u64 =
// 69 B/packet) of values derived from the packet bytes; they differ only in how many packets one
// lane handles (K = 1, 2, 4: a u8 column becomes one K-byte store per lane) — or (ideal) write
// 72 B/packet as four 1-KiB-per-instruction uint4 columns + one u64 column, or (copy) copy the
// 64-byte packets to a contiguous output.
#include <hip/hip_runtime.h>
#include <stdint.h>

struct Cols { void* p[31]; };

template <int K>
__global__ __launch_bounds__(256) void k_store(const uint8_t* slab, uint32_t n, Cols c) {
    const uint32_t g = blockIdx.x * 256u + threadIdx.x;  // lane group: packets g*K .. g*K+K-1
    const uint32_t i0 = g * K;
    if (i0 >= n) return;
    uint32_t v[K][8];
#pragma unroll
    for (int k = 0; k < K; k++) {
        const uint4* p = (const uint4*)(slab + (uint64_t)(i0 + k) * 64);
        uint4 a = p[0], b = p[1], cc = p[2], d = p[3];
        v[k][0] = a.x; v[k][1] = a.y ^ b.x; v[k][2] = a.z ^ b.y; v[k][3] = a.w ^ b.z;
        v[k][4] = cc.x ^ b.w; v[k][5] = cc.y ^ d.x; v[k][6] = cc.z ^ d.y; v[k][7] = cc.w ^ d.z;
    }
#pragma unroll
    for (int col = 0; col < 11; col++) {
        uint32_t w = 0;
#pragma unroll
        for (int k = 0; k < K; k++) w |= ((v[k][col & 7] >> col) & 0xFFu) << (8 * k);
        if constexpr (K == 1) ((uint8_t*)c.p[col])[i0] = (uint8_t)w;
        else if constexpr (K == 2) ((uint16_t*)c.p[col])[g] = (uint16_t)w;
        else ((uint32_t*)c.p[col])[g] = w;
    }
#pragma unroll
    for (int col = 11; col < 26; col++) {
        uint32_t h[K];
#pragma unroll
        for (int k = 0; k < K; k++) h[k] = (v[k][col & 7] >> (col & 15)) & 0xFFFFu;
        if constexpr (K == 1) ((uint16_t*)c.p[col])[i0] = (uint16_t)h[0];
        else if constexpr (K == 2) ((uint32_t*)c.p[col])[g] = h[0] | (h[1] << 16);
        else ((uint2*)c.p[col])[g] = make_uint2(h[0] | (h[1] << 16), h[2] | (h[3] << 16));
    }
#pragma unroll
    for (int col = 26; col < 29; col++) {
        if constexpr (K == 1) ((uint32_t*)c.p[col])[i0] = v[0][col & 7] + col;
        else if constexpr (K == 2) ((uint2*)c.p[col])[g] = make_uint2(v[0][col & 7] + col, v[1][col & 7] + col);
        else ((uint4*)c.p[col])[g] = make_uint4(v[0][col & 7] + col, v[1][col & 7] + col, v[2][col & 7] + col, v[3][col & 7] + col);
    }
#pragma unroll
    for (int col = 29; col < 31; col++) {
#pragma unroll
        for (int k = 0; k < K; k++)
            ((uint64_t*)c.p[col])[i0 + k] = ((uint64_t)v[k][col & 7] << 16) ^ v[k][(col + 1) & 7];
    }
}

// R packets per lane, packet g + r*(n/R) for r < R (all R loads issued first), each stored with
// the K=1 shape: a lane runs R rounds of the same per-packet stores, so the grid has 1/R the waves.
template <int R>
__global__ __launch_bounds__(256) void k_rounds(const uint8_t* slab, uint32_t n, Cols c) {
    const uint32_t g = blockIdx.x * 256u + threadIdx.x;
    const uint32_t part = n / R;
    if (g >= part) return;
    uint4 q[R][4];
#pragma unroll
    for (int r = 0; r < R; r++) {
        const uint4* p = (const uint4*)(slab + (uint64_t)(g + r * part) * 64);
        q[r][0] = p[0]; q[r][1] = p[1]; q[r][2] = p[2]; q[r][3] = p[3];
    }
#pragma unroll
    for (int r = 0; r < R; r++) {
        const uint32_t i = g + r * part;
        uint4 a = q[r][0], b = q[r][1], cc = q[r][2], d = q[r][3];
        uint32_t v[8] = {a.x, a.y ^ b.x, a.z ^ b.y, a.w ^ b.z, cc.x ^ b.w, cc.y ^ d.x, cc.z ^ d.y, cc.w ^ d.z};
#pragma unroll
        for (int k = 0; k < 11; k++) ((uint8_t*)c.p[k])[i] = (uint8_t)(v[k & 7] >> k);
#pragma unroll
        for (int k = 11; k < 26; k++) ((uint16_t*)c.p[k])[i] = (uint16_t)(v[k & 7] >> (k & 15));
#pragma unroll
        for (int k = 26; k < 29; k++) ((uint32_t*)c.p[k])[i] = v[k & 7] + k;
#pragma unroll
        for (int k = 29; k < 31; k++) ((uint64_t*)c.p[k])[i] = ((uint64_t)v[k & 7] << 16) ^ v[(k + 1) & 7];
    }
}

// ideal store shape: chunk q of packet i at out[q][i] (16 B), q = 0..3, plus one u64 column
__global__ __launch_bounds__(256) void k_ideal(const uint8_t* slab, uint32_t n, Cols c) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n) return;
    const uint4* p = (const uint4*)(slab + (uint64_t)i * 64);
    uint4 a = p[0], b = p[1], cc = p[2], d = p[3];
    ((uint4*)c.p[0])[i] = make_uint4(a.x ^ 1, a.y, a.z, a.w);
    ((uint4*)c.p[1])[i] = make_uint4(b.x ^ 2, b.y, b.z, b.w);
    ((uint4*)c.p[2])[i] = make_uint4(cc.x ^ 3, cc.y, cc.z, cc.w);
    ((uint4*)c.p[3])[i] = make_uint4(d.x ^ 4, d.y, d.z, d.w);
    ((uint64_t*)c.p[4])[i] = ((uint64_t)a.x << 32) | d.w;
}

extern "C" int probe_store(int which, const uint8_t* slab, uint32_t n, void* const* cols, void* stream) {
    Cols c;
    for (int k = 0; k < 31; k++) c.p[k] = cols[k];
    hipStream_t s = (hipStream_t)stream;
    switch (which) {
        case 0: hipLaunchKernelGGL(k_store<1>, dim3((n + 255) / 256), dim3(256), 0, s, slab, n, c); break;
        case 1: hipLaunchKernelGGL(k_store<2>, dim3((n / 2 + 255) / 256), dim3(256), 0, s, slab, n, c); break;
        case 2: hipLaunchKernelGGL(k_store<4>, dim3((n / 4 + 255) / 256), dim3(256), 0, s, slab, n, c); break;
        case 3: hipLaunchKernelGGL(k_ideal, dim3((n + 255) / 256), dim3(256), 0, s, slab, n, c); break;
        case 4: hipLaunchKernelGGL(k_rounds<2>, dim3((n / 2 + 255) / 256), dim3(256), 0, s, slab, n, c); break;
        case 5: hipLaunchKernelGGL(k_rounds<4>, dim3((n / 4 + 255) / 256), dim3(256), 0, s, slab, n, c); break;
        default: return -1;
    }
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
