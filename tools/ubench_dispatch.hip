// ubench_dispatch.hip -- how do one-round grids actually land on MI355X?  Each workgroup spins
// for a fixed amount of VALU work and records s_memrealtime at start/end plus its hardware
// placement (XCC / SE / CU / SIMD via HW_ID).  Prints concurrency and per-CU counts.
// Build: hipcc --offload-arch=gfx950 -O3 -o build/ubench_dispatch tools/ubench_dispatch.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>
#include <map>

__global__ void k(uint64_t *rec, int work, int lds_words) {
    extern __shared__ uint32_t sm[];
    uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    uint32_t x = threadIdx.x;
    for (int i = threadIdx.x; i < lds_words; i += blockDim.x) sm[i] = i;
    __syncthreads();
    for (int i = 0; i < work; i++) x = x * 1664525u + sm[(x >> 20) % (lds_words ? lds_words : 1)];
    uint64_t t1 = __builtin_amdgcn_s_memrealtime();
    uint32_t hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));     // HW_REG_HW_ID (id 4), 32 bits
    uint32_t xcc = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (15 << 11));   // HW_REG_XCC_ID (id 20)
    if (threadIdx.x == 0) {
        rec[blockIdx.x * 4 + 0] = t0;
        rec[blockIdx.x * 4 + 1] = t1;
        rec[blockIdx.x * 4 + 2] = hw;
        rec[blockIdx.x * 4 + 3] = xcc;
    }
    if (x == 0x12345678u) rec[0] = x;
}

void run(const char *name, int blocks, int threads, int lds_bytes, int work) {
    uint64_t *d;
    hipMalloc(&d, (size_t)blocks * 32);
    hipFuncSetAttribute((const void *)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), lds_bytes, 0, d, work, lds_bytes / 4);
    hipDeviceSynchronize();
    hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), lds_bytes, 0, d, work, lds_bytes / 4);
    hipDeviceSynchronize();
    std::vector<uint64_t> h((size_t)blocks * 4);
    hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost);
    uint64_t t0 = ~0ull, t1 = 0;
    double dur = 0;
    std::map<uint32_t, int> percu;
    for (int b = 0; b < blocks; b++) {
        t0 = std::min(t0, h[b * 4]); t1 = std::max(t1, h[b * 4 + 1]);
        dur += (double)(h[b * 4 + 1] - h[b * 4]);
        uint32_t hw = (uint32_t)h[b * 4 + 2];
        uint32_t cu = (hw >> 8) & 15, sh = (hw >> 12) & 1, se = (hw >> 13) & 7, xcc = (uint32_t)h[b * 4 + 3] & 15;
        percu[(xcc << 16) | (se << 8) | (sh << 4) | cu]++;
    }
    // start-time spread
    std::vector<uint64_t> st(blocks);
    for (int b = 0; b < blocks; b++) st[b] = h[b * 4] - t0;
    std::sort(st.begin(), st.end());
    int mn = 1 << 30, mx = 0;
    for (auto &kv : percu) { mn = std::min(mn, kv.second); mx = std::max(mx, kv.second); }
    printf("%-10s blocks=%5d thr=%4d lds=%6d: span %.1f us, mean WG life %.1f us, start p50 %.1f p90 %.1f p99 %.1f max %.1f us; CUs used %zu, WGs/CU min %d max %d\n",
           name, blocks, threads, lds_bytes, (t1 - t0) / 100.0, dur / blocks / 100.0,
           st[blocks / 2] / 100.0, st[blocks * 9 / 10] / 100.0, st[blocks * 99 / 100] / 100.0, st[blocks - 1] / 100.0,
           percu.size(), mn, mx);
    hipFree(d);
}

int main() {
    run("lastocc", 2048, 256, 16832, 20000);
    run("emit64", 2048, 64, 18220, 20000);
    run("emit64nl", 2048, 64, 18220, 20000);
    run("emit256", 512, 256, 4 * 18220 / 4 * 4, 20000);
    run("small", 256, 256, 0, 20000);
    return 0;
}
