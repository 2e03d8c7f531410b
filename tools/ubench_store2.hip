// ubench_store2.hip -- which streaming-store patterns reach torch's fill_ rate (~6.5 TB/s for
// 800 MB on MI355X) and which stop near 5.4 TB/s?  All variants write the same 800 MB of int64:
//   oneshot4   fill-like: 256-thread blocks, each thread 4 consecutive int64 (two dwordx4), one
//              pass, ~98K blocks (the dispatcher's frontier is compact)
//   oneshot1   the same with one int64 per thread (dwordx2)
//   persist_c  2048 one-wave blocks (8 per CU, LDS-capped), chunk c of 2 KB -> wave c % 2048
//              (grid-stride: all waves write inside a compact moving window)
//   persist_r  2048 one-wave blocks, each its own contiguous 390 KB run (the sampler kernels)
//   persist_r4 the same with dwordx4 stores (2 per 256 ids)
//   persist_r16 4096 / 8192 one-wave blocks (16 / 32 per CU), own runs
// Build: hipcc --offload-arch=gfx950 -O3 -o build/ubench_store2 tools/ubench_store2.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr uint64_t kIds = 100000000ull;

__global__ __launch_bounds__(256) void oneshot4(int64_t *o, uint64_t n, int64_t salt) {
    const uint64_t i = ((uint64_t)blockIdx.x * 256 + threadIdx.x) * 4;
    if (i + 3 < n) {
        longlong2 a, b;
        a.x = (int64_t)i + salt; a.y = (int64_t)i + 1 + salt;
        b.x = (int64_t)i + 2 + salt; b.y = (int64_t)i + 3 + salt;
        *(longlong2 *)(o + i) = a;
        *(longlong2 *)(o + i + 2) = b;
    }
}
__global__ __launch_bounds__(256) void oneshot1(int64_t *o, uint64_t n, int64_t salt) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) o[i] = (int64_t)i + salt;
}
__global__ __launch_bounds__(64) void persist_c(int64_t *o, uint64_t n, int64_t salt) {
    extern __shared__ uint32_t pad[];
    if (n == 0) pad[threadIdx.x] = 0;
    const uint64_t chunks = n / 256;
    for (uint64_t c = blockIdx.x; c < chunks; c += gridDim.x) {
        int64_t *p = o + c * 256;
#pragma unroll
        for (int j = 0; j < 4; j++) p[64 * j + threadIdx.x] = (int64_t)(c * 256 + 64 * j + threadIdx.x) + salt;
    }
}
template <int V4>
__global__ __launch_bounds__(64) void persist_r(int64_t *o, uint64_t n, int64_t salt) {
    extern __shared__ uint32_t pad[];
    if (n == 0) pad[threadIdx.x] = 0;
    const uint64_t per = n / gridDim.x;
    int64_t *p = o + blockIdx.x * per;
    for (uint64_t b = 0; b + 256 <= per; b += 256) {
        if (V4) {
#pragma unroll
            for (int j = 0; j < 2; j++) {
                const uint64_t s = b + 128 * j + 2 * threadIdx.x;
                longlong2 v; v.x = (int64_t)s + salt; v.y = (int64_t)s + 1 + salt;
                *(longlong2 *)(p + s) = v;
            }
        } else {
#pragma unroll
            for (int j = 0; j < 4; j++) p[b + 64 * j + threadIdx.x] = (int64_t)(b + 64 * j + threadIdx.x) + salt;
        }
    }
}

// one wave per 2 KB chunk-run of K chunks (K = 1: one-shot one-wave blocks)
template <int K>
__global__ __launch_bounds__(64) void short_runs(int64_t *o, uint64_t n, int64_t salt) {
    int64_t *p = o + (uint64_t)blockIdx.x * 256 * K;
#pragma unroll
    for (int c = 0; c < K; c++)
#pragma unroll
        for (int j = 0; j < 4; j++) p[256 * c + 64 * j + threadIdx.x] = (int64_t)(256 * c + 64 * j + threadIdx.x) + salt;
}
// one-shot blocks of NT threads, each lane S stores of 8 B (S x NT x 8 B per block)
template <int NT, int S>
__global__ __launch_bounds__(NT) void oneshot_ns(int64_t *o, uint64_t n, int64_t salt) {
    int64_t *p = o + (uint64_t)blockIdx.x * NT * S;
#pragma unroll
    for (int j = 0; j < S; j++) p[NT * j + threadIdx.x] = (int64_t)(NT * j + threadIdx.x) + salt;
}
// persistent own runs through a buffer descriptor (32-bit offsets, the k_g_emit store form);
// AUX = cache-policy bits of the store (1 glc/sc0, 2 slc/nt, 3 both)
template <int AUX = 0>
__global__ __launch_bounds__(64) void persist_rb(int64_t *o, uint64_t n, int64_t salt) {
    extern __shared__ uint32_t pad[];
    if (n == 0) pad[threadIdx.x] = 0;
    const uint64_t per = n / gridDim.x;
    int64_t *p = o + blockIdx.x * per;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(p, 0, (int)(per * 8), 0x00020000);
    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
    uint32_t voff = threadIdx.x * 8u;
    for (uint64_t b = 0; b + 256 <= per; b += 256) {
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const uint32_t v = (uint32_t)(b + 64 * j + threadIdx.x) + (uint32_t)salt;
            const u32x2 d = {v, 0u};
            __builtin_amdgcn_raw_buffer_store_b64(d, rs, (int)voff, 512 * j, AUX);
        }
        voff += 2048u;
    }
}

// canonical grid-stride fill: every iteration of the whole grid writes one contiguous band
__global__ __launch_bounds__(256) void gridstride(int64_t *o, uint64_t n, int64_t salt) {
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) o[i] = (int64_t)i + salt;
}
// persistent one-wave runs, but each wave's run split into KB-sized pieces dealt round-robin
// over the waves (wave w writes pieces w, w + G, ...), piece = P x 2 KB
template <int P>
__global__ __launch_bounds__(64) void persist_pieces(int64_t *o, uint64_t n, int64_t salt) {
    extern __shared__ uint32_t pad[];
    if (n == 0) pad[threadIdx.x] = 0;
    const uint64_t piece = 256ull * P, np = n / piece;
    for (uint64_t q = blockIdx.x; q < np; q += gridDim.x) {
        int64_t *p = o + q * piece;
        for (int c = 0; c < P; c++)
#pragma unroll
            for (int j = 0; j < 4; j++) p[256 * c + 64 * j + threadIdx.x] = (int64_t)(256 * c + 64 * j + threadIdx.x) + salt;
    }
}

template <class F>
void timeit(const char *name, F launch) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    launch(1);
    hipEventRecord(a);
    for (int r = 0; r < 20; r++) launch(2 + r);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    ms /= 20;
    printf("%-14s %7.1f us  %.2f TB/s\n", name, ms * 1e3, (double)kIds * 8 / (ms * 1e-3) / 1e12);
}

int main() {
    int64_t *o;
    hipMalloc(&o, kIds * 8 + 4096);
    const uint64_t n = kIds;
    for (auto fn : {(const void *)persist_c, (const void *)persist_r<0>, (const void *)persist_r<1>, (const void *)persist_rb<0>,
                    (const void *)persist_rb<1>, (const void *)persist_rb<2>, (const void *)persist_rb<3>,
                    (const void *)persist_pieces<16>, (const void *)persist_pieces<128>})
        (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    for (int rep = 0; rep < 2; rep++) {
        timeit("oneshot4", [&](int s) { hipLaunchKernelGGL(oneshot4, dim3((uint32_t)((n / 4 + 255) / 256)), dim3(256), 0, 0, o, n, (int64_t)s); });
        timeit("oneshot1", [&](int s) { hipLaunchKernelGGL(oneshot1, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, 0, o, n, (int64_t)s); });
        timeit("persist_c", [&](int s) { hipLaunchKernelGGL(persist_c, dim3(2048), dim3(64), 18220, 0, o, n, (int64_t)s); });
        timeit("persist_c16", [&](int s) { hipLaunchKernelGGL(persist_c, dim3(4096), dim3(64), 9000, 0, o, n, (int64_t)s); });
        timeit("persist_r", [&](int s) { hipLaunchKernelGGL(persist_r<0>, dim3(2048), dim3(64), 18220, 0, o, n, (int64_t)s); });
        timeit("persist_r4", [&](int s) { hipLaunchKernelGGL(persist_r<1>, dim3(2048), dim3(64), 18220, 0, o, n, (int64_t)s); });
        timeit("persist_r16", [&](int s) { hipLaunchKernelGGL(persist_r<0>, dim3(4096), dim3(64), 9000, 0, o, n, (int64_t)s); });
        timeit("persist_r32", [&](int s) { hipLaunchKernelGGL(persist_r<0>, dim3(8192), dim3(64), 4000, 0, o, n, (int64_t)s); });
        timeit("short1", [&](int s) { hipLaunchKernelGGL(short_runs<1>, dim3((uint32_t)(n / 256)), dim3(64), 0, 0, o, n, (int64_t)s); });
        timeit("short8", [&](int s) { hipLaunchKernelGGL(short_runs<8>, dim3((uint32_t)(n / 2048)), dim3(64), 0, 0, o, n, (int64_t)s); });
        timeit("short64", [&](int s) { hipLaunchKernelGGL(short_runs<64>, dim3((uint32_t)(n / 16384)), dim3(64), 0, 0, o, n, (int64_t)s); });
        timeit("persist_rb", [&](int s) { hipLaunchKernelGGL(persist_rb<0>, dim3(2048), dim3(64), 18220, 0, o, n, (int64_t)s); });
        timeit("persist_rb_sc0", [&](int s) { hipLaunchKernelGGL(persist_rb<1>, dim3(2048), dim3(64), 18220, 0, o, n, (int64_t)s); });
        timeit("persist_rb_nt", [&](int s) { hipLaunchKernelGGL(persist_rb<2>, dim3(2048), dim3(64), 18220, 0, o, n, (int64_t)s); });
        timeit("persist_rb_3", [&](int s) { hipLaunchKernelGGL(persist_rb<3>, dim3(2048), dim3(64), 18220, 0, o, n, (int64_t)s); });
        timeit("os_64x1", [&](int s) { hipLaunchKernelGGL((oneshot_ns<64, 1>), dim3((uint32_t)(n / 64)), dim3(64), 0, 0, o, n, (int64_t)s); });
        timeit("os_256x4", [&](int s) { hipLaunchKernelGGL((oneshot_ns<256, 4>), dim3((uint32_t)(n / 1024)), dim3(256), 0, 0, o, n, (int64_t)s); });
        timeit("os_256x16", [&](int s) { hipLaunchKernelGGL((oneshot_ns<256, 16>), dim3((uint32_t)(n / 4096)), dim3(256), 0, 0, o, n, (int64_t)s); });
        timeit("os_1024x4", [&](int s) { hipLaunchKernelGGL((oneshot_ns<1024, 4>), dim3((uint32_t)(n / 4096)), dim3(1024), 0, 0, o, n, (int64_t)s); });
        timeit("grid_2048", [&](int s) { hipLaunchKernelGGL(gridstride, dim3(2048), dim3(256), 0, 0, o, n, (int64_t)s); });
        timeit("grid_512", [&](int s) { hipLaunchKernelGGL(gridstride, dim3(512), dim3(256), 0, 0, o, n, (int64_t)s); });
        timeit("pieces_32K", [&](int s) { hipLaunchKernelGGL(persist_pieces<16>, dim3(2048), dim3(64), 18220, 0, o, n, (int64_t)s); });
        timeit("pieces_256K", [&](int s) { hipLaunchKernelGGL(persist_pieces<128>, dim3(2048), dim3(64), 18220, 0, o, n, (int64_t)s); });
        timeit("persist_r32x4", [&](int s) { hipLaunchKernelGGL(persist_r<1>, dim3(8192), dim3(64), 4000, 0, o, n, (int64_t)s); });
    }
    return 0;
}
