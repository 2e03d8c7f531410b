// ubench_lastocc.hip -- what bounds the V2 last-occurrence pass?  The kernel's loop shape
// (2048 workgroups x 256 threads, 16.8 KB LDS, 48,896 steps each) with: (a) slot hash + ds_max
// (the real loop), (b) hash only (xor-accumulated), (c) trivial address + ds_max.
// Build: hipcc --offload-arch=gfx950 -O3 -o build/ubench_lastocc tools/ubench_lastocc.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ uint32_t slot_hash(uint32_t t, uint32_t s0, uint32_t s1) {
    uint32_t x = t ^ s0; x ^= x >> 16; x *= 0x21F0AAADu; x ^= x >> 15; x ^= s1;
    x *= 0x735A2D97u; x ^= x >> 15; return x;
}

template <int MODE>
__global__ __launch_bounds__(256) void k(uint32_t *out, uint32_t n, uint32_t s0, uint32_t s1) {
    __shared__ uint32_t lastT[4096 + 128];
    for (int s = threadIdx.x; s < 4096; s += 256) lastT[s] = 0;
    __syncthreads();
    const uint32_t t0 = blockIdx.x * n;
    uint32_t acc = 0;
    if (MODE == 3) __builtin_amdgcn_s_setprio(3);
    for (uint32_t base = 0; base < n; base += 2048) {
        if (MODE == 3 && base == n / 2) __builtin_amdgcn_s_setprio(0);
        const uint32_t b = base + threadIdx.x;
        uint32_t k[8];
#pragma unroll
        for (int j = 0; j < 8; j++) {
            if (MODE == 2) k[j] = (b * 2654435761u + j * 977u) >> 20;
            else k[j] = (uint32_t)(((uint64_t)slot_hash(t0 + b + 256 * j, s0, s1) * 4096u) >> 32);
        }
#pragma unroll
        for (int j = 0; j < 8; j++) {
            if (MODE == 1) acc ^= k[j];
            else if (MODE == 4) acc += atomicMax(&lastT[k[j]], b + 256 * j + 1);
            else atomicMax(&lastT[k[j]], b + 256 * j + 1);
        }
    }
    __syncthreads();
    if (MODE == 5) {   // + the real epilogue shape: per slot a 6-round Feistel with LDS keys
        __shared__ uint32_t rk[8 * 16];
        if (threadIdx.x < 128) rk[threadIdx.x] = threadIdx.x * 0x9E3779B9u;
        __syncthreads();
        const float invB = 1.0f / 4096.0f;
        for (int s = threadIdx.x; s < 4096; s += 256) {
            const uint32_t lt = lastT[s];
            uint32_t p = 1000u + lt - 1u;
            uint32_t dw = (uint32_t)((float)p * invB);
            int32_t r = (int32_t)(p - dw * 4096u);
            if (r < 0) { dw--; r += 4096; }
            if (r >= 4096) { dw++; r -= 4096; }
            const uint32_t *k = rk + 8 * (dw & 15);
            uint32_t L = (uint32_t)r >> 6, R = (uint32_t)r & 63;
#pragma unroll
            for (int i = 0; i < 6; i++) { const uint32_t t = L ^ (((R ^ k[i]) * 0x9E3779B1u) >> 26); L = R; R = t; }
            out[blockIdx.x * 4096 + s] = lt ? (L << 6 | R) : 0xFFFFFFFFu;
        }
        return;
    }
    for (int s = threadIdx.x; s < 4096; s += 256) acc += lastT[s];
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

template <int MODE>
void run(const char *name, uint32_t *out) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    const uint32_t n = 48896 / 2048 * 2048;
    hipLaunchKernelGGL(k<MODE>, dim3(2048), dim3(256), 0, 0, out, n, 1u, 2u);
    hipEventRecord(a);
    for (int r = 0; r < 10; r++) hipLaunchKernelGGL(k<MODE>, dim3(2048), dim3(256), 0, 0, out, n, 1u + r, 2u);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    printf("%-16s %.1f us per launch (%u steps per WG, 2048 WGs)\n", name, ms * 100.0f, n);
}

int main() {
    uint32_t *out;
    hipMalloc(&out, 2048 * 4096 * 4);
    run<0>("hash+ds_max", out);
    run<1>("hash only", out);
    run<2>("trivial+ds_max", out);
    run<0>("hash+ds_max", out);
    run<3>("+setprio", out);
    run<4>("ds_max_rtn", out);
    run<5>("+epilogue", out);
    return 0;
}
