// ubench_store.hip -- streaming-store bandwidth in the V2 emit layouts: 2048 single-wave
// workgroups (LDS-padded to 8 per CU), each writing its own contiguous run of int64 ids,
// 512 B per store instruction (dwordx2 per lane) vs 1 KB (dwordx4: two ids per lane), with and
// without a little ALU work per id.  Build: hipcc --offload-arch=gfx950 -O3 -o build/ubench_store tools/ubench_store.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int MODE>
__global__ __launch_bounds__(64) void k(int64_t *out, uint32_t n, uint32_t salt) {
    extern __shared__ uint32_t pad[];
    if (n == 0) pad[threadIdx.x] = 0;
    int64_t *o = out + (size_t)blockIdx.x * n;
    const uint32_t lane = threadIdx.x;
    if (MODE == 0) {            // dwordx2, 4 per 256 steps
        for (uint32_t b = 0; b < n; b += 256)
#pragma unroll
            for (int j = 0; j < 4; j++) o[b + 64 * j + lane] = (int64_t)(b + 64 * j + lane + salt);
    } else if (MODE == 1) {     // dwordx4: lane writes ids 2l, 2l+1
        for (uint32_t b = 0; b < n; b += 256)
#pragma unroll
            for (int j = 0; j < 2; j++) {
                const uint32_t s = b + 128 * j + 2 * lane;
                longlong2 v; v.x = s + salt; v.y = s + 1 + salt;
                *(longlong2 *)(o + s) = v;
            }
    } else if (MODE == 3) {     // dwordx2, grid-interleaved: wave b writes 2 KB chunks b, b+grid, ...
        const uint32_t G = gridDim.x;
        for (uint32_t b = 0; b < n; b += 256)
#pragma unroll
            for (int j = 0; j < 4; j++)
                out[((size_t)(b >> 8) * G + blockIdx.x) * 256 + 64 * j + lane] = (int64_t)(b + 64 * j + lane + salt);
    } else if (MODE == 4) {     // dwordx2, contiguous runs at a padded stride (n + 512 ids)
        int64_t *op = out + (size_t)blockIdx.x * (n + 512);
        for (uint32_t b = 0; b < n; b += 256)
#pragma unroll
            for (int j = 0; j < 4; j++) op[b + 64 * j + lane] = (int64_t)(b + 64 * j + lane + salt);
    } else {                    // dwordx2 with nontemporal hint
        for (uint32_t b = 0; b < n; b += 256)
#pragma unroll
            for (int j = 0; j < 4; j++) __builtin_nontemporal_store((int64_t)(b + 64 * j + lane + salt), &o[b + 64 * j + lane]);
    }
}

// The grouped-pool (C5) layout: 8 ranks x G = 256 groups, one wave per (rank, group); a rank's
// step stream is cut into bursts of BL steps dealt round-robin to its groups, and each store
// instruction covers 64 / BL bursts of one group (lane l: burst l / BL, step l % BL of it).
template <int BL>
__global__ __launch_bounds__(64) void kg(int64_t *out, uint32_t n, uint32_t salt) {
    extern __shared__ uint32_t pad[];
    if (n == 0) pad[threadIdx.x] = 0;
    const uint32_t G = 256, lane = threadIdx.x;
    const uint32_t rank = blockIdx.x / G, g = blockIdx.x % G;
    int64_t *o = out + (size_t)rank * G * n + (size_t)g * BL;
    const uint32_t c_lane = (lane / BL) * BL * G + lane % BL;
    for (uint32_t u = 0; u < n; u += 256)
#pragma unroll
        for (int j = 0; j < 4; j++)
            o[(size_t)(u / BL) * BL * G + c_lane + j * 64u * G] = (int64_t)(u + 64 * j + lane + salt);
}

template <int BL>
void runsg(const char *name, int64_t *out, uint32_t n, int lds) {
    hipFuncSetAttribute((const void *)kg<BL>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    hipLaunchKernelGGL(kg<BL>, dim3(2048), dim3(64), lds, 0, out, n, 1u);
    hipEventRecord(a);
    for (int r = 0; r < 10; r++) hipLaunchKernelGGL(kg<BL>, dim3(2048), dim3(64), lds, 0, out, n, 2u + r);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    ms /= 10;
    printf("%-12s blocks= 2048 lds=%6d: %.1f us  %.2f TB/s\n", name, lds, ms * 1e3,
           (double)2048 * n * 8 / (ms * 1e-3) / 1e12);
}

template <int MODE>
void run(const char *name, int64_t *out, int blocks, uint32_t n, int lds) {
    hipFuncSetAttribute((const void *)k<MODE>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(64), lds, 0, out, n, 1u);
    hipEventRecord(a);
    for (int r = 0; r < 10; r++) hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(64), lds, 0, out, n, 2u + r);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    ms /= 10;
    printf("%-12s blocks=%5d lds=%6d: %.1f us  %.2f TB/s\n", name, blocks, lds, ms * 1e3,
           (double)blocks * n * 8 / (ms * 1e-3) / 1e12);
}

int main() {
    const uint32_t n = 48896;
    int64_t *out;
    hipMalloc(&out, (size_t)8192 * (n + 1024) * 8);
    run<0>("dwordx2", out, 2048, n, 18220);
    run<1>("dwordx4", out, 2048, n, 18220);
    run<2>("dwordx2-nt", out, 2048, n, 18220);
    run<3>("interleaved", out, 2048, n, 18220);
    run<4>("stride+4K", out, 2048, n, 18220);
    run<0>("dwordx2 49152", out, 2048, 49152, 18220);
    run<0>("dwordx2 48640", out, 2048, 48640, 18220);
    run<0>("dwordx2 4/CU", out, 1024, 2 * n, 36000);
    run<0>("dwordx2 2/CU", out, 512, 4 * n, 72000);
    run<0>("dwordx2", out, 4096, n / 2, 9000);
    run<1>("dwordx4", out, 4096, n / 2, 9000);
    run<0>("dwordx2", out, 8192, n / 4, 4000);
    runsg<16>("grouped b16", out, n, 18220);
    runsg<32>("grouped b32", out, n, 18220);
    runsg<64>("grouped b64", out, n, 18220);
    run<0>("dwordx2", out, 2048, n, 18220);
    runsg<16>("grouped b16", out, n, 18220);
    return 0;
}
