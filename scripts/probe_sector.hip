// Measurement probe (not part of libpktgpu): does a load that touches only half of each 128-B line
// fetch 64-B sectors from HBM when it carries cache-policy bits?  C3's parse reads the first ~64 B of
// each 128-B slot and its reads are whole lines (profiles/ab/r02calib_fetch_requests.txt: every
// memory-side request of plain loads is a 128-B line request).  Lane i reads `width` bytes at
// buf + i * stride (four 16-byte loads in flight per lane for width 64) with load kind `kind`:
//   0 plain global_load_dwordx4, 1 __builtin_nontemporal_load (nt), 2 glc slc (sc0 sc1), 3 nt sc0 sc1.
// Build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC -o scripts/_probe_sector.so scripts/probe_sector.hip
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {
template <int KIND>
__device__ __forceinline__ uint4 ld16(const uint4* p) {
    if constexpr (KIND == 0) {
        return *p;
    } else if constexpr (KIND == 1) {
        typedef uint32_t v4u __attribute__((ext_vector_type(4)));
        const v4u v = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p));
        return make_uint4(v.x, v.y, v.z, v.w);
    } else if constexpr (KIND == 2) {
        uint4 v;
        asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
        return v;
    } else {
        uint4 v;
        asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1 nt\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
        return v;
    }
}

template <int KIND>
__global__ __launch_bounds__(256) void sector_kernel(const uint8_t* buf, uint32_t n, uint32_t stride, uint32_t width,
                                                     uint32_t* out) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n) return;
    const uint4* p = reinterpret_cast<const uint4*>(buf + (uint64_t)i * stride);
    uint32_t acc = 0;
    uint4 v[8];
#pragma unroll
    for (uint32_t c = 0; c < 8; c++)
        if (c < width / 16) v[c] = ld16<KIND>(p + c);
#pragma unroll
    for (uint32_t c = 0; c < 8; c++)
        if (c < width / 16) acc ^= v[c].x + v[c].y * 3u + v[c].z * 5u + v[c].w * 7u;
    out[i] = acc;
}
}  // namespace

extern "C" int probe_sector(int kind, const uint8_t* buf, uint32_t n, uint32_t stride, uint32_t width, uint32_t* out,
                            void* stream) {
    if (width == 0 || width > 128 || (width & 15)) return -1;
    const dim3 g((n + 255) / 256), b(256);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    switch (kind) {
        case 0: hipLaunchKernelGGL(sector_kernel<0>, g, b, 0, s, buf, n, stride, width, out); break;
        case 1: hipLaunchKernelGGL(sector_kernel<1>, g, b, 0, s, buf, n, stride, width, out); break;
        case 2: hipLaunchKernelGGL(sector_kernel<2>, g, b, 0, s, buf, n, stride, width, out); break;
        default: hipLaunchKernelGGL(sector_kernel<3>, g, b, 0, s, buf, n, stride, width, out); break;
    }
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
