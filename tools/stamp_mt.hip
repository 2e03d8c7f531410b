// stamp_mt.hip -- diagnostic: the workgroup MT draws of pss_mt.h built with -DPSS_MT_STAMPS on
// C5-shaped V2 pool2 windows (W = P = 2^20, 88 streams); prints the per-round phase clocks.
// Build (from the repo root):
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DPSS_MT_STAMPS -Ipartiallyshuffledistributedsampler_amd/csrc \
//     -o build/stamp_mt tools/stamp_mt.hip
#include "../partiallyshuffledistributedsampler_amd/csrc/pss_mt.h"
#include <cstdio>
#include <vector>

using namespace pss;

__global__ __launch_bounds__(kMtWgThreads) void k_stamp(uint32_t W, uint32_t P, uint32_t *K1, uint32_t *K2) {
    __shared__ MtWgShared sh;
    if (threadIdx.x < 64) mt_seed_int(sh.mt[0], 7 + (int64_t)blockIdx.x * 10000);
    __syncthreads();
    uint32_t *k1 = K1 + (size_t)blockIdx.x * W, *k2 = K2 + (size_t)blockIdx.x * W;
    mt_draws_pair_wg(sh, 0, W, P, [&](bool second, uint32_t i, uint32_t r) {
        if (second) k2[i] = r;
        else k1[i] = r;
    });
}

__global__ __launch_bounds__(kMtWgThreads) void k_stamp_v1(uint32_t n, uint32_t *J) {
    __shared__ MtWgShared sh;
    if (threadIdx.x < 64) mt_seed_int(sh.mt[0], 9 + (int64_t)blockIdx.x * 10000);
    __syncthreads();
    uint32_t *jw = J + (size_t)blockIdx.x * n;
    mt_draws_wg(sh, 0, n - 1, [&](uint32_t d) { return n - d; }, [&](uint32_t d, uint32_t r) { jw[n - 1 - d] = r; });
}

int main() {
    const uint32_t W = 1u << 20, P = 1u << 20, nb = 88, nb1 = 96;
    uint32_t *K1, *K2;
    hipMalloc(&K1, (size_t)nb1 * W * 4);   // (the V1 run below takes 96 windows)
    hipMalloc(&K2, (size_t)nb * W * 4);
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    for (int it = 0; it < 2; it++) {
        std::vector<uint64_t> z((size_t)4096 * 8, 0);
        hipMemcpyToSymbol(HIP_SYMBOL(pss_mt_stamps), z.data(), z.size() * 8);
        hipEventRecord(a);
        hipLaunchKernelGGL(k_stamp, dim3(nb), dim3(kMtWgThreads), 0, 0, W, P, K1, K2);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms = 0;
        hipEventElapsedTime(&ms, a, b);
        std::vector<uint64_t> st((size_t)4096 * 8);
        hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(pss_mt_stamps), st.size() * 8);
        double sum[8] = {0};
        for (uint32_t k = 0; k < nb; k++)
            for (int i = 0; i < 8; i++) sum[i] += (double)st[(size_t)k * 8 + i];
        const double rounds = sum[7];
        printf("kernel %.3f ms, %d streams, %.1f rounds/stream; per round (clocks): summaries %.0f  combine %.0f  "
               "emit %.0f | generator %.0f %.0f %.0f | exact blocks %.2f\n",
               ms, nb, rounds / nb, sum[0] / rounds, sum[1] / rounds, sum[2] / rounds, sum[3] / rounds,
               sum[4] / rounds, sum[5] / rounds, sum[6] / rounds);
    }
    {   // V1 windows: 96 streams of 2^20 - 1 draws
        hipEventRecord(a);
        hipLaunchKernelGGL(k_stamp_v1, dim3(nb1), dim3(kMtWgThreads), 0, 0, W, K1);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms = 0;
        hipEventElapsedTime(&ms, a, b);
        printf("v1 draws: kernel %.3f ms, 96 streams of 2^20\n", ms);
    }
    return 0;
}
