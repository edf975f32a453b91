// probe_launch.hip — where does an isolated 2^20-packet launch lose time?  (not part of the product)
//
// Every kernel moves exactly C2's bytes: reads 64 B per packet (4 x dwordx4 per lane) and writes
// the C2 tuple layout (31 per-lane columns, 69 B per packet).  Variants differ only in how the
// grid is shaped.  Each figure = one HIP event pair around R back-to-back launches, each launch
// on a different slab/column set of a >= 1 GiB ring (same method as bench.py's roofline phase).
//
//   hipcc -O3 --offload-arch=gfx950 -o build/probe_launch scripts/probe_launch.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#define CK(x)                                                                            \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));    \
            exit(1);                                                                     \
        }                                                                                \
    } while (0)

struct Cols { void* p[31]; };

__device__ __forceinline__ void emit(const Cols& c, uint64_t i, const uint4& a, const uint4& b,
                                     const uint4& cc, const uint4& d) {
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

__global__ void k_empty(uint32_t n, uint32_t* out) {
    if (blockIdx.x * blockDim.x + threadIdx.x == 0xFFFFFFFFu) out[0] = n;
}

// one packet per lane, any block size
__global__ __launch_bounds__(1024) void k_lane(const uint8_t* slab, uint32_t n, Cols c) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint4* p = (const uint4*)(slab + (uint64_t)i * 64);
    emit(c, i, p[0], p[1], p[2], p[3]);
}

// one packet per lane, only the first `ncol` columns written (ncol = 1: status only)
__global__ __launch_bounds__(256) void k_lane_cols(const uint8_t* slab, uint32_t n, Cols c, int ncol) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint4* p = (const uint4*)(slab + (uint64_t)i * 64);
    uint4 a = p[0], b = p[1], cc = p[2], d = p[3];
    uint32_t v = a.x ^ b.y ^ cc.z ^ d.w;
    for (int k = 0; k < ncol; k++) ((uint8_t*)c.p[k])[i] = (uint8_t)(v >> k);
}

// status-only again, with a dynamic LDS allocation: mode 0 = allocated, unused; mode 1 = the
// parse kernel's staging (4 x ds_write_b128 chunk-major) and 4 dependent LDS reads back.
__global__ __launch_bounds__(256) void k_lane_lds(const uint8_t* slab, uint32_t n, Cols c, int mode) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const uint32_t t = threadIdx.x;
    const uint32_t i = blockIdx.x * blockDim.x + t;
    if (i >= n) return;
    const uint4* p = (const uint4*)(slab + (uint64_t)i * 64);
    uint4 a = p[0], b = p[1], cc = p[2], d = p[3];
    uint32_t v = a.x ^ b.y ^ cc.z ^ d.w;
    if (mode == 1) {
        *(uint4*)(lds + 0 * 4096 + t * 16) = a;
        *(uint4*)(lds + 1 * 4096 + t * 16) = b;
        *(uint4*)(lds + 2 * 4096 + t * 16) = cc;
        *(uint4*)(lds + 3 * 4096 + t * 16) = d;
        __builtin_amdgcn_wave_barrier();
        uint32_t k = v & 3;
        for (int s = 0; s < 4; s++) {  // dependent chain, like the walk's header-to-header reads
            v = *(const uint32_t*)(lds + ((k + s) & 3) * 4096 + t * 16 + (v & 12));
            k = v & 3;
        }
    }
    if (mode == 2) {  // packet-major, lane stride 17 dwords (odd: conflict-free b32 access)
        uint32_t* w = (uint32_t*)lds + t * 17;
        const uint32_t q[16] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, cc.x, cc.y, cc.z, cc.w, d.x, d.y, d.z, d.w};
#pragma unroll
        for (int k = 0; k < 16; k++) w[k] = q[k];
        __builtin_amdgcn_wave_barrier();
        for (int s = 0; s < 4; s++) v = w[(v + s) & 15];
    }
    if (mode == 3) {  // chunk-major, dependent b128 reads
        *(uint4*)(lds + 0 * 4096 + t * 16) = a;
        *(uint4*)(lds + 1 * 4096 + t * 16) = b;
        *(uint4*)(lds + 2 * 4096 + t * 16) = cc;
        *(uint4*)(lds + 3 * 4096 + t * 16) = d;
        __builtin_amdgcn_wave_barrier();
        for (int s = 0; s < 4; s++) {
            uint4 x = *(const uint4*)(lds + ((v + s) & 3) * 4096 + t * 16);
            v = x.x ^ x.y ^ x.z ^ x.w ^ v;
        }
    }
    ((uint8_t*)c.p[0])[i] = (uint8_t)v;
}

// P packets per lane: lane t of block b handles b*256*P + k*256 + t, all loads issued first
template <int P>
__global__ __launch_bounds__(256) void k_multi(const uint8_t* slab, uint32_t n, Cols c) {
    const uint32_t base = blockIdx.x * 256u * P + threadIdx.x;
    uint4 r[P][4];
#pragma unroll
    for (int k = 0; k < P; k++) {
        const uint32_t i = min(base + k * 256u, n - 1);
        const uint4* p = (const uint4*)(slab + (uint64_t)i * 64);
        r[k][0] = p[0]; r[k][1] = p[1]; r[k][2] = p[2]; r[k][3] = p[3];
    }
#pragma unroll
    for (int k = 0; k < P; k++) {
        const uint32_t i = base + k * 256u;
        if (i < n) emit(c, i, r[k][0], r[k][1], r[k][2], r[k][3]);
    }
}

// persistent: grid-stride over 256-packet tiles, next tile's loads issued before this tile's stores
__global__ __launch_bounds__(256) void k_persist(const uint8_t* slab, uint32_t n, Cols c) {
    const uint32_t tiles = (n + 255) / 256;
    uint32_t t = blockIdx.x;
    if (t >= tiles) return;
    uint32_t i = min(t * 256u + threadIdx.x, n - 1);
    const uint4* p = (const uint4*)(slab + (uint64_t)i * 64);
    uint4 a = p[0], b = p[1], cc = p[2], d = p[3];
    for (;;) {
        const uint32_t tn = t + gridDim.x;
        uint4 a2 = a, b2 = b, c2 = cc, d2 = d;
        if (tn < tiles) {
            const uint32_t in = min(tn * 256u + threadIdx.x, n - 1);
            const uint4* q = (const uint4*)(slab + (uint64_t)in * 64);
            a2 = q[0]; b2 = q[1]; c2 = q[2]; d2 = q[3];
        }
        const uint32_t ii = t * 256u + threadIdx.x;
        if (ii < n) emit(c, ii, a, b, cc, d);
        if (tn >= tiles) break;
        t = tn; a = a2; b = b2; cc = c2; d = d2;
    }
}

static const int kSizes[31] = {1,1,1,1,1,1,1,1,1,1,1, 2,2,2,2,2,2,2,2,2,2,2,2,2,2,2, 4,4,4, 8,8};

int main(int argc, char** argv) {
    const uint32_t n = argc > 1 ? (uint32_t)strtoul(argv[1], 0, 0) : (1u << 20);
    const int R = 50;
    const size_t slab_b = (size_t)n * 64;
    int ring = (int)((1ull << 30) / slab_b);
    if (ring < 2) ring = 2;
    std::vector<uint8_t*> slabs(ring);
    std::vector<Cols> cols(ring);
    for (int r = 0; r < ring; r++) {
        CK(hipMalloc(&slabs[r], slab_b));
        CK(hipMemset(slabs[r], r + 1, slab_b));
        for (int k = 0; k < 31; k++) CK(hipMalloc(&cols[r].p[k], (size_t)n * kSizes[k]));
    }
    uint32_t* dummy;
    CK(hipMalloc(&dummy, 4));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));

    auto run = [&](const char* name, auto launch) {
        for (int k = 0; k < 10; k++) launch(k % ring);
        CK(hipStreamSynchronize(s));
        float best = 1e30f;
        for (int rep = 0; rep < 3; rep++) {
            CK(hipEventRecord(e0, s));
            for (int k = 0; k < R; k++) launch(k % ring);
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (ms < best) best = ms;
        }
        CK(hipGetLastError());
        const double us = best * 1e3 / R;
        printf("%-28s n=%-9u %9.2f us/launch  %7.1f GB/s (133 B/pkt)  %6.2f us per 2^20\n", name, n, us,
               (double)n * 133 / us / 1e3, us * (1 << 20) / n);
    };
    const uint32_t b256 = (n + 255) / 256;
    run("empty 256-thr grid", [&](int r) { hipLaunchKernelGGL(k_empty, dim3(b256), dim3(256), 0, s, n, dummy); });
    for (int bs : {64, 128, 256, 512, 1024})
        run((std::string("lane bs=") + std::to_string(bs)).c_str(), [&](int r) {
            hipLaunchKernelGGL(k_lane, dim3((n + bs - 1) / bs), dim3(bs), 0, s, slabs[r], n, cols[r]);
        });
    for (int nc : {1, 4, 11})
        run((std::string("lane u8 cols=") + std::to_string(nc)).c_str(), [&](int r) {
            hipLaunchKernelGGL(k_lane_cols, dim3(b256), dim3(256), 0, s, slabs[r], n, cols[r], nc);
        });
    for (int lk : {0, 20480})
        for (int mode : {0, 1, 2, 3})
            run((std::string("status lds=") + std::to_string(lk) + " mode=" + std::to_string(mode)).c_str(), [&](int r) {
                hipLaunchKernelGGL(k_lane_lds, dim3(b256), dim3(256), lk, s, slabs[r], n, cols[r], lk ? mode : 0);
            });
    run("multi P=2", [&](int r) { hipLaunchKernelGGL(k_multi<2>, dim3((n + 511) / 512), dim3(256), 0, s, slabs[r], n, cols[r]); });
    run("multi P=4", [&](int r) { hipLaunchKernelGGL(k_multi<4>, dim3((n + 1023) / 1024), dim3(256), 0, s, slabs[r], n, cols[r]); });
    for (int g : {256, 512, 1024, 2048})
        run((std::string("persist g=") + std::to_string(g)).c_str(), [&](int r) {
            hipLaunchKernelGGL(k_persist, dim3(g), dim3(256), 0, s, slabs[r], n, cols[r]);
        });
    // plain copies of the same byte count for scale (read 64 B + write 69 B per packet)
    {
        uint8_t* dst;
        CK(hipMalloc(&dst, (size_t)n * 69 * 2));
        run("hipMemcpyAsync D2D 64B/pkt", [&](int r) { CK(hipMemcpyAsync(dst, slabs[r], slab_b, hipMemcpyDeviceToDevice, s)); });
        CK(hipFree(dst));
    }
    return 0;
}
