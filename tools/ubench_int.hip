// ubench_int.hip -- issue-rate micro-benchmark of the integer ops the sampler kernels lean on
// (v_mul_lo_u32, v_mad_u64_u32, v_mul_u32_u24, v_add_u32, v_xor_b32) on gfx950.
// Build: hipcc --offload-arch=gfx950 -O3 -o build/ubench_int tools/ubench_int.hip
// Each kernel runs 8 independent chains per lane so throughput, not latency, is measured.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define ITERS 4096

template <int OP>
__global__ __launch_bounds__(256) void k(uint32_t *out, uint32_t seed) {
    uint32_t x[8];
#pragma unroll
    for (int i = 0; i < 8; i++) x[i] = seed + threadIdx.x * 8 + i;
    const uint32_t c = seed | 1u;
    for (int it = 0; it < ITERS; it++) {
#pragma unroll
        for (int i = 0; i < 8; i++) {
            if (OP == 0) x[i] = x[i] + c;                                   // v_add_u32
            if (OP == 1) x[i] = x[i] * c;                                   // v_mul_lo_u32
            if (OP == 2) { uint64_t p = (uint64_t)x[i] * c; x[i] = (uint32_t)(p >> 32) ^ (uint32_t)p; }  // v_mad_u64_u32 (+xor)
            if (OP == 3) x[i] = __umul24(x[i], c) + i;                      // v_mul_u32_u24 (+add)
            if (OP == 4) x[i] = __umulhi(x[i], c);                          // v_mul_hi_u32
        }
    }
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) s ^= x[i];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int OP>
float run(uint32_t *out, int blocks) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, out, 7u);
    hipEventRecord(a);
    for (int r = 0; r < 5; r++) hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, out, 7u + r);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    return ms / 5;
}

int main() {
    const int blocks = 256 * 8;
    uint32_t *out;
    hipMalloc(&out, sizeof(uint32_t) * blocks * 256);
    const char *names[] = {"v_add_u32", "v_mul_lo_u32", "v_mad_u64_u32+xor", "v_mul_u32_u24", "v_mul_hi_u32"};
    float t[5] = {run<0>(out, blocks), run<1>(out, blocks), run<2>(out, blocks), run<3>(out, blocks), run<4>(out, blocks)};
    const double ops = (double)blocks * 256 * ITERS * 8;
    for (int i = 0; i < 5; i++)
        printf("%-20s %.3f ms  %.1f Gop/s  rel-to-add %.2fx\n", names[i], t[i], ops / (t[i] * 1e-3) / 1e9, t[i] / t[0]);
    hipFree(out);
    return 0;
}
