// ubench_lds.hip -- throughput of LDS ops at random word addresses over a 4096-word table (the
// V2 slot table shape): plain write, no-return max, returning max, exchange, read.  One
// 256-thread workgroup per CU slot; reports G lane-ops/s per CU.
// Build: hipcc --offload-arch=gfx950 -O3 -o build/ubench_lds tools/ubench_lds.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define ITERS 4096

template <int OP, int NT>
__global__ __launch_bounds__(NT) void k(uint32_t *out, uint32_t seed) {
    __shared__ uint32_t t[4096];
    for (int i = threadIdx.x; i < 4096; i += NT) t[i] = i;
    __syncthreads();
    uint32_t x = seed ^ (blockIdx.x * NT + threadIdx.x) * 0x9E3779B1u, acc = 0;
    for (int it = 0; it < ITERS; it += 4) {
        uint32_t a[4];
#pragma unroll
        for (int j = 0; j < 4; j++) { x = x * 1664525u + 1013904223u; a[j] = x >> 20; }
#pragma unroll
        for (int j = 0; j < 4; j++) {
            if (OP == 0) t[a[j]] = it + j;
            if (OP == 1) atomicMax(&t[a[j]], (uint32_t)(it + j));
            if (OP == 2) acc += atomicMax(&t[a[j]], (uint32_t)(it + j));
            if (OP == 3) acc += atomicExch(&t[a[j]], (uint32_t)(it + j));
            if (OP == 4) acc += t[a[j]];
        }
    }
    __syncthreads();
    out[blockIdx.x * NT + threadIdx.x] = acc + t[threadIdx.x];
}

template <int OP, int NT>
void run(const char *name, uint32_t *out, int blocks, int cus) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    hipLaunchKernelGGL((k<OP, NT>), dim3(blocks), dim3(NT), 0, 0, out, 7u);
    hipEventRecord(a);
    for (int r = 0; r < 5; r++) hipLaunchKernelGGL((k<OP, NT>), dim3(blocks), dim3(NT), 0, 0, out, 7u + r);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    ms /= 5;
    const double ops = (double)blocks * NT * ITERS;
    printf("%-12s NT=%4d blocks=%5d  %.3f ms  %.2f G lane-ops/s/CU  %.1f lanes/clk/CU@2.1GHz\n", name, NT,
           blocks, ms, ops / (ms * 1e-3) / 1e9 / cus, ops / (ms * 1e-3) / cus / 2.1e9);
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    uint32_t *out;
    hipMalloc(&out, sizeof(uint32_t) * 4096 * 1024);
    for (int wpc = 2; wpc <= 8; wpc *= 2) {
        const int blocks = cus * wpc;       // 256-thread WGs: 4 waves each
        run<0, 256>("write", out, blocks, cus);
        run<1, 256>("max", out, blocks, cus);
        run<2, 256>("max_rtn", out, blocks, cus);
        run<3, 256>("wrxchg_rtn", out, blocks, cus);
        run<4, 256>("read", out, blocks, cus);
    }
    run<0, 64>("write", out, cus * 8, cus);
    run<3, 64>("wrxchg_rtn", out, cus * 8, cus);
    hipFree(out);
    return 0;
}
