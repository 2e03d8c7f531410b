// ubench_int.hip -- issue-rate micro-benchmark of the integer ops the sampler kernels lean on
// (v_mul_lo_u32, v_mad_u64_u32, v_mul_u32_u24, v_mul_hi_u32 against v_add_u32) on gfx950.
// Build: hipcc --offload-arch=gfx950 -O3 -o build/ubench_int tools/ubench_int.hip
// Every op is followed by a shift-xor so the compiler cannot fold the loop; 8 independent
// chains per lane so throughput, not latency, is measured.  Reported: ns per op-pair per
// wave64 on one SIMD, relative to the add pair.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define ITERS 2048

template <int OP>
__global__ __launch_bounds__(256) void k(uint32_t *out, uint32_t seed) {
    uint32_t x[8];
#pragma unroll
    for (int i = 0; i < 8; i++) x[i] = seed + threadIdx.x * 8 + i;
    const uint32_t c = seed | 0x9E3779u;
    for (int it = 0; it < ITERS; it++) {
#pragma unroll
        for (int i = 0; i < 8; i++) {
            uint32_t y;
            if (OP == 0) y = x[i] + c;
            if (OP == 1) y = x[i] * c;
            if (OP == 2) { uint64_t p = (uint64_t)x[i] * c; y = (uint32_t)(p >> 32) + (uint32_t)p; }
            if (OP == 3) y = __umul24(x[i], c);
            if (OP == 4) y = __umulhi(x[i], c);
            x[i] = y ^ (x[i] >> 13);
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
    const char *names[] = {"add+shr+xor", "mul_lo+shr+xor", "mad_u64(+add)+shr+xor", "mul_u24+shr+xor", "mul_hi+shr+xor"};
    float t[5] = {run<0>(out, blocks), run<1>(out, blocks), run<2>(out, blocks), run<3>(out, blocks), run<4>(out, blocks)};
    const double iters = (double)blocks * 256 * ITERS * 8;   // lane-iterations
    for (int i = 0; i < 5; i++)
        printf("%-24s %.3f ms  %.2f T lane-iter/s  rel-to-add %.2fx\n", names[i], t[i], iters / (t[i] * 1e-3) / 1e12, t[i] / t[0]);
    hipFree(out);
    return 0;
}
