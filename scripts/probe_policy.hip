// probe_policy: do any load cache-policy bits make gfx950's L2 issue 64-B memory requests?
// Item i reads its first `width` bytes at buf + i*stride (C3's shape: 64 B of every 128-B slot), as
// `width`/16 consecutive lanes x 16 B (one wave instruction covers 64/(width/16) items).  One launch per
// (policy, width); run under rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum
// (request sizes per launch) and alone for the per-launch time (HIP events, printed).
//   hipcc -O3 --offload-arch=gfx950 -o probe_policy probe_policy.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                 \
    do {                                                                      \
        hipError_t e_ = (x);                                                  \
        if (e_ != hipSuccess) {                                               \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));           \
            exit(1);                                                          \
        }                                                                     \
    } while (0)

typedef int32_t i32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}

// AUX: buffer-load aux bits (gfx940+: 1 = sc0, 2 = nt, 16 = sc1)
template <int AUX>
__global__ __launch_bounds__(256) void probe(const uint8_t* buf, uint32_t bytes, uint32_t n, uint32_t stride,
                                             uint32_t cpi /* 16-B chunks per item */, uint32_t* out) {
    const uint32_t g = blockIdx.x * 256u + threadIdx.x;
    const uint32_t item = g / cpi, c = g % cpi;
    if (item >= n) return;
    const uint32_t off = item * stride + 16u * c;
    const i32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rsrc(buf, bytes), off, 0, AUX);
    const uint32_t acc = (uint32_t)(v.x + v.y * 3 + v.z * 5 + v.w * 7);
    if (acc == 0x12345678u) out[g] = acc;  // keep the load
}

template <int AUX>
float run(uint8_t* const* buf, uint32_t bytes, uint32_t n, uint32_t stride, uint32_t width, uint32_t* out, int reps) {
    const uint32_t cpi = width / 16, threads = n * cpi;
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventRecord(a, 0));
    for (int r = 0; r < reps; r++)
        hipLaunchKernelGGL(probe<AUX>, dim3((threads + 255) / 256), dim3(256), 0, 0, buf[r % 8], bytes, n, stride, cpi, out);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms * 1000.f / reps;
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 8;
    const uint32_t n = 1u << 20, stride = 128;
    const uint32_t bytes = n * stride;
    uint8_t* buf[8];  // a 1 GiB ring: no launch is served by the 256 MiB MALL
    uint32_t* out;
    for (auto& p : buf) {
        CK(hipMalloc(&p, bytes));
        CK(hipMemset(p, 1, bytes));
    }
    CK(hipMalloc(&out, (size_t)n * 8 * 4));
    // order: for width in {64, 128}: policies 0, sc0, nt, sc0|nt, sc1, sc1|nt, sc0|sc1
    for (uint32_t width : {64u, 128u}) {
        float t[7];
        t[0] = run<0>(buf, bytes, n, stride, width, out, reps);
        t[1] = run<1>(buf, bytes, n, stride, width, out, reps);
        t[2] = run<2>(buf, bytes, n, stride, width, out, reps);
        t[3] = run<3>(buf, bytes, n, stride, width, out, reps);
        t[4] = run<16>(buf, bytes, n, stride, width, out, reps);
        t[5] = run<18>(buf, bytes, n, stride, width, out, reps);
        t[6] = run<17>(buf, bytes, n, stride, width, out, reps);
        printf("width %3u of %u-B slots, us/launch: plain %.2f  sc0 %.2f  nt %.2f  sc0nt %.2f  sc1 %.2f  sc1nt %.2f  sc0sc1 %.2f\n",
               width, stride, t[0], t[1], t[2], t[3], t[4], t[5], t[6]);
    }
    for (auto& p : buf) CK(hipFree(p));
    CK(hipFree(out));
    return 0;
}
