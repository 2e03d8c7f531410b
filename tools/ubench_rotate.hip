// ubench_rotate.hip -- does a persistent per-wave store stream (the C2 replay's store pattern:
// 2048 waves, each writing its own contiguous run of 800 MB / 2048) gain when each launch's runs
// start where the previous launch's waves wrote last (those lines still dirty in the Infinity
// Cache)?  Mode A: the same runs every launch.  Mode B: runs shifted by T - D each launch, so a
// wave's first D ids land on the previous launch's last D ids of a run.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

constexpr uint64_t N = 100000000ull;   // ids (800 MB)
constexpr uint32_t WAVES = 2048;

__global__ __launch_bounds__(256) void k_runs(uint64_t *out, uint64_t T, uint64_t off, uint64_t v, uint64_t late) {
    // late > 0: the run's first `late` ids are written after the rest (held back, written last)
    const uint32_t lane = threadIdx.x & 63, w = blockIdx.x * 4u + (threadIdx.x >> 6);
    const uint64_t base = off + (uint64_t)w * T;
    for (uint64_t i = late; i < T; i += 64) {
        const uint64_t p = (base + i + lane) % N;
        if (i + lane < T) out[p] = v + p;
    }
    for (uint64_t i = 0; i < late; i += 64) {
        const uint64_t p = (base + i + lane) % N;
        if (i + lane < late) out[p] = v + p;
    }
}

int main() {
    uint64_t *out;
    (void)hipMalloc(&out, N * sizeof(uint64_t));
    (void)hipMemset(out, 0, N * sizeof(uint64_t));
    const uint64_t T = (N + WAVES - 1) / WAVES;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    const uint64_t Ds[] = {0, 4096, 8192, 16384, 24576};
    for (int rep = 0; rep < 2; rep++)
        for (uint64_t D : Ds) {
            uint64_t off = 0;
            std::vector<float> ms;
            for (int e = 0; e < 30; e++) {
                (void)hipEventRecord(a, 0);
                hipLaunchKernelGGL(k_runs, dim3(WAVES / 4), dim3(256), 0, 0, out, T, off, (uint64_t)e, (uint64_t)0);
                (void)hipEventRecord(b, 0);
                (void)hipEventSynchronize(b);
                float t = 0;
                (void)hipEventElapsedTime(&t, a, b);
                ms.push_back(t);
                if (D) off = (off + T - D) % N;
            }
            double s = 0;
            for (int e = 5; e < 30; e++) s += ms[e];
            printf("D %6lu ids (%s): mean %.1f us over launches 5..29 (first %.1f)\n", (unsigned long)D,
                   D ? "runs start on the last writes" : "same runs", s / 25 * 1e3, ms[0] * 1e3);
        }
    // alternate launches hold back their runs' first D ids (even: late, odd: in order)
    for (int rep = 0; rep < 2; rep++)
        for (uint64_t D : Ds) {
            std::vector<float> ms;
            for (int e = 0; e < 30; e++) {
                (void)hipEventRecord(a, 0);
                hipLaunchKernelGGL(k_runs, dim3(WAVES / 4), dim3(256), 0, 0, out, T, (uint64_t)0, (uint64_t)e,
                                   (e & 1) ? (uint64_t)0 : D);
                (void)hipEventRecord(b, 0);
                (void)hipEventSynchronize(b);
                float t = 0;
                (void)hipEventElapsedTime(&t, a, b);
                ms.push_back(t);
            }
            double se = 0, so = 0;
            for (int e = 6; e < 30; e += 2) { se += ms[e]; so += ms[e + 1]; }
            printf("alternate, D %6lu: held-back launches %.1f us, in-order launches after them %.1f us, mean %.1f\n",
                   (unsigned long)D, se / 12 * 1e3, so / 12 * 1e3, (se + so) / 24 * 1e3);
        }
    return 0;
}
