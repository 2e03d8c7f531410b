// ubench_balance.hip -- is the persistent-kernel write gap (own runs ~5.3 TB/s against one-shot
// ~6.3 TB/s for the same 800 MB) a per-XCD imbalance that dynamic work claiming removes?
//   oneshot4      fill-like reference: 256-thread blocks, 4 int64 per thread, one pass
//   persist_r     2048 one-wave blocks, each its own contiguous run (the replay's layout)
//   queue_<C>     2048 one-wave blocks claiming chunks of C x 2 KB from one agent-scope counter
//                 (vector atomic from lane 0, readfirstlane of the result) until none is left
//   guided        2048 one-wave blocks: chunk = max(2 KB, remaining / (2 x 2048)) (guided
//                 self-scheduling: big chunks first, small ones at the end)
// Each variant also reports the bytes every XCC wrote (per-wave XCC_ID) and the spread of wave
// end times (s_memrealtime, 100 MHz).
// Build: hipcc --offload-arch=gfx950 -O3 -o build/ubench_balance tools/ubench_balance.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>

constexpr uint64_t kIds = 100000000ull;
constexpr int kWaves = 2048;
constexpr int kMaxWaves = 8192;

struct Stats { unsigned long long xcc_bytes[8]; unsigned long long end[kMaxWaves]; unsigned long long t0; unsigned int xcc[kMaxWaves]; };

__device__ __forceinline__ uint32_t xcc_id() { return __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (15 << 11)) & 7u; }

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

__device__ __forceinline__ void fill_chunk(int64_t *o, uint64_t c0, uint64_t c1, int64_t salt) {
    for (uint64_t c = c0; c < c1; c++) {
        int64_t *p = o + c * 256;
#pragma unroll
        for (int j = 0; j < 4; j++) p[64 * j + threadIdx.x] = (int64_t)(c * 256 + 64 * j + threadIdx.x) + salt;
    }
}

__device__ __forceinline__ void record(Stats *st, uint64_t chunks_done) {
    if (threadIdx.x == 0) {
        atomicAdd(&st->xcc_bytes[xcc_id()], (unsigned long long)chunks_done * 2048ull);
        const uint32_t w = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
        st->end[w] = __builtin_amdgcn_s_memrealtime();
        st->xcc[w] = xcc_id();
    }
}
__device__ __forceinline__ void record_w(Stats *st, uint64_t chunks_done) {   // every wave of a block
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(&st->xcc_bytes[xcc_id()], (unsigned long long)chunks_done * 2048ull);
        const uint32_t w = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
        st->end[w] = __builtin_amdgcn_s_memrealtime();
        st->xcc[w] = xcc_id();
    }
}

__global__ __launch_bounds__(64) void persist_r(int64_t *o, uint64_t n, int64_t salt, Stats *st) {
    extern __shared__ uint32_t pad[];
    if (n == 0) pad[threadIdx.x] = 0;
    const uint64_t chunks = n / 256, per = chunks / gridDim.x;
    fill_chunk(o, blockIdx.x * per, blockIdx.x * per + per, salt);
    record(st, per);
}

// claim `k` chunks; returns the first (>= total: nothing left)
__device__ __forceinline__ uint64_t claim(unsigned long long *ctr, uint64_t k) {
    unsigned long long got = 0;
    if (threadIdx.x == 0) got = atomicAdd(ctr, (unsigned long long)k);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)got);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(got >> 32));
    return ((uint64_t)hi << 32) | lo;
}

template <int C>
__global__ __launch_bounds__(64) void queue(int64_t *o, uint64_t n, int64_t salt, Stats *st,
                                            unsigned long long *ctr) {
    extern __shared__ uint32_t pad[];
    if (n == 0) pad[threadIdx.x] = 0;
    const uint64_t chunks = n / 256;
    uint64_t done = 0;
    for (;;) {
        const uint64_t c0 = claim(ctr, C);
        if (c0 >= chunks) break;
        const uint64_t c1 = c0 + C < chunks ? c0 + C : chunks;
        fill_chunk(o, c0, c1, salt);
        done += c1 - c0;
    }
    record(st, done);
}

__global__ __launch_bounds__(64) void guided(int64_t *o, uint64_t n, int64_t salt, Stats *st,
                                             unsigned long long *ctr) {
    extern __shared__ uint32_t pad[];
    if (n == 0) pad[threadIdx.x] = 0;
    const uint64_t chunks = n / 256;
    uint64_t done = 0;
    for (;;) {
        // guess of what is left from a plain read (racy but only a size hint), then claim
        unsigned long long seen = 0;
        if (threadIdx.x == 0) seen = __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint64_t s = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(seen >> 32)) << 32) |
                           __builtin_amdgcn_readfirstlane((uint32_t)seen);
        const uint64_t left = s < chunks ? chunks - s : 0;
        uint64_t k = left / (2 * kWaves);
        if (k < 1) k = 1;
        const uint64_t c0 = claim(ctr, k);
        if (c0 >= chunks) break;
        const uint64_t c1 = c0 + k < chunks ? c0 + k : chunks;
        fill_chunk(o, c0, c1, salt);
        done += c1 - c0;
    }
    record(st, done);
}

// NW waves per block, each its own contiguous run; the block's waves re-align every K chunks
// (s_barrier), so no wave of a CU runs ahead of its partners
template <int NW, int K>
__global__ __launch_bounds__(64 * NW) void persist_bar(int64_t *o, uint64_t n, int64_t salt, Stats *st) {
    const uint64_t chunks = n / 256, nwaves = (uint64_t)gridDim.x * NW, per = chunks / nwaves;
    const uint64_t w = (uint64_t)blockIdx.x * NW + threadIdx.x / 64;
    const int lane = threadIdx.x & 63;
    int64_t *p = o + w * per * 256;
    for (uint64_t c = 0; c < per; c++) {
#pragma unroll
        for (int j = 0; j < 4; j++) p[c * 256 + 64 * j + lane] = (int64_t)(c * 256 + 64 * j + lane) + salt;
        if (K && (c % K) == K - 1) __syncthreads();
    }
    record_w(st, per);
}

// own runs sized by block parity: the blocks dispatched to the slow XCCs (block b on XCC
// (b + 7) mod 8 on every box seen: even b -> odd XCC) get F/16 of the others' share.  The
// partition depends on blockIdx only (always a partition); the balance on that mapping.
template <int F>
__global__ __launch_bounds__(64) void persist_x(int64_t *o, uint64_t n, int64_t salt, Stats *st) {
    extern __shared__ uint32_t pad[];
    if (n == 0) pad[threadIdx.x] = 0;
    const uint64_t chunks = n / 256, pairs = gridDim.x / 2;
    const uint64_t per2 = chunks / pairs;                       // chunks per (even, odd) pair
    const uint64_t short_ = per2 * F / (16 + F), long_ = per2 - short_;
    const uint64_t pr = blockIdx.x / 2;
    const bool slow = (blockIdx.x & 1) == 0;
    const uint64_t c0 = pr * per2 + (slow ? 0 : short_);
    const uint64_t c1 = slow ? c0 + short_ : pr * per2 + per2;
    fill_chunk(o, c0, c1, salt);
    record(st, c1 - c0);
}

// own runs with 16-byte stores: lane l writes ids 2l, 2l + 1 of each 128-id half chunk (each
// store instruction 1 KB contiguous, the shape of oneshot4)
__global__ __launch_bounds__(64) void persist_r16(int64_t *o, uint64_t n, int64_t salt, Stats *st) {
    extern __shared__ uint32_t pad[];
    if (n == 0) pad[threadIdx.x] = 0;
    const uint64_t chunks = n / 256, per = chunks / gridDim.x;
    for (uint64_t c = blockIdx.x * per; c < blockIdx.x * per + per; c++) {
        int64_t *p = o + c * 256;
#pragma unroll
        for (int j = 0; j < 2; j++) {
            const uint64_t i = 128 * j + 2 * threadIdx.x;
            longlong2 a;
            a.x = (int64_t)(c * 256 + i) + salt; a.y = (int64_t)(c * 256 + i + 1) + salt;
            *(longlong2 *)(p + i) = a;
        }
    }
    record(st, per);
}

// own runs with 16-byte stores after a lane exchange: the values come out as the replay makes
// them (lane l holds ids l + 64 j, j < 4) and two ds_bpermute-style shuffles per pair of
// registers move them to lane order 2l, 2l + 1
__global__ __launch_bounds__(64) void persist_r16x(int64_t *o, uint64_t n, int64_t salt, Stats *st) {
    extern __shared__ uint32_t pad[];
    if (n == 0) pad[threadIdx.x] = 0;
    const uint64_t chunks = n / 256, per = chunks / gridDim.x;
    const int l = threadIdx.x;
    for (uint64_t c = blockIdx.x * per; c < blockIdx.x * per + per; c++) {
        int64_t *p = o + c * 256;
        int64_t v[4];
#pragma unroll
        for (int j = 0; j < 4; j++) v[j] = (int64_t)(c * 256 + 64 * j + l) + salt;
#pragma unroll
        for (int h = 0; h < 2; h++) {   // ids [128 h, 128 h + 128): registers 2h, 2h + 1
            const int s0 = (2 * l) & 63, s1 = (2 * l + 1) & 63;
            const bool hi = l >= 32;
            const int64_t a0 = __shfl(v[2 * h], s0), b0 = __shfl(v[2 * h + 1], s0);
            const int64_t a1 = __shfl(v[2 * h], s1), b1 = __shfl(v[2 * h + 1], s1);
            longlong2 a;
            a.x = hi ? b0 : a0; a.y = hi ? b1 : a1;
            *(longlong2 *)(p + 128 * h + 2 * l) = a;
        }
    }
    record(st, per);
}

// the same bytes per wave, chunk-interleaved over groups of IL waves: wave w = IL a + b writes
// chunks base_a + c IL + b, so the waves of a group write adjacent 2 KB chunks at any moment
// (IL = gridDim: the whole grid sweeps the output together, like a one-shot grid)
template <int IL>
__global__ __launch_bounds__(64) void persist_il(int64_t *o, uint64_t n, int64_t salt, Stats *st) {
    extern __shared__ uint32_t pad[];
    if (n == 0) pad[threadIdx.x] = 0;
    const uint64_t chunks = n / 256, per = chunks / gridDim.x;
    const uint64_t il = IL ? IL : gridDim.x;
    const uint64_t a = blockIdx.x / il, b = blockIdx.x % il;
    const uint64_t base = a * il * per;
    for (uint64_t c = 0; c < per; c++) {
        const uint64_t ch = base + c * il + b;
        int64_t *p = o + ch * 256;
#pragma unroll
        for (int j = 0; j < 4; j++) p[64 * j + threadIdx.x] = (int64_t)(ch * 256 + 64 * j + threadIdx.x) + salt;
    }
    record(st, per);
}

// own runs, each wave starting inside its run at a wave-dependent chunk and wrapping (ROT: chunk
// (w * 37) mod per), or its run shifted by (w mod 16) chunks of 2 KB (SKEW: neighbouring runs
// overlap by up to 30 KB, timing only): are equal-phase runs conflicting in the HBM channels?
template <int MODE>
__global__ __launch_bounds__(64) void persist_phase(int64_t *o, uint64_t n, int64_t salt, Stats *st) {
    extern __shared__ uint32_t pad[];
    if (n == 0) pad[threadIdx.x] = 0;
    const uint64_t chunks = n / 256, per = chunks / gridDim.x - 16;
    const uint64_t w = blockIdx.x;
    const uint64_t base = w * (per + 16) + (MODE == 1 ? (w % 16) : 0);
    const uint64_t rot = MODE == 0 ? (w * 37) % per : 0;
    for (uint64_t c = 0; c < per; c++) {
        uint64_t cc = c + rot;
        if (cc >= per) cc -= per;
        const uint64_t ch = base + cc;
        int64_t *p = o + ch * 256;
#pragma unroll
        for (int j = 0; j < 4; j++) p[64 * j + threadIdx.x] = (int64_t)(ch * 256 + 64 * j + threadIdx.x) + salt;
    }
    record(st, per);
}

// own runs with non-temporal stores (global_store ... nt): does the L2's write allocation of
// 2048 concurrent runs cost the persistent streams their rate?
__global__ __launch_bounds__(64) void persist_nt(int64_t *o, uint64_t n, int64_t salt, Stats *st) {
    extern __shared__ uint32_t pad[];
    if (n == 0) pad[threadIdx.x] = 0;
    const uint64_t chunks = n / 256, per = chunks / gridDim.x;
    for (uint64_t c = blockIdx.x * per; c < blockIdx.x * per + per; c++) {
        int64_t *p = o + c * 256;
#pragma unroll
        for (int j = 0; j < 4; j++)
            __builtin_nontemporal_store((int64_t)(c * 256 + 64 * j + threadIdx.x) + salt, p + 64 * j + threadIdx.x);
    }
    record(st, per);
}

// one-shot with non-temporal stores
__global__ __launch_bounds__(256) void oneshot_nt(int64_t *o, uint64_t n, int64_t salt) {
    const uint64_t i = ((uint64_t)blockIdx.x * 256 + threadIdx.x) * 4;
    if (i + 3 < n) {
#pragma unroll
        for (int k = 0; k < 4; k++) __builtin_nontemporal_store((int64_t)(i + k) + salt, o + i + k);
    }
}

__global__ void stamp_t0(Stats *st) { if (threadIdx.x == 0) st->t0 = __builtin_amdgcn_s_memrealtime(); }

template <class F>
void timeit(const char *name, Stats *st, unsigned long long *ctr, F launch) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    hipMemset(ctr, 0, 8);
    launch(1);
    float best = 1e9, sum = 0;
    Stats h{};
    for (int r = 0; r < 10; r++) {
        hipMemset(st, 0, sizeof(Stats));
        hipMemset(ctr, 0, 8);
        hipLaunchKernelGGL(stamp_t0, dim3(1), dim3(64), 0, 0, st);
        hipEventRecord(a);
        launch(2 + r);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms = 0;
        hipEventElapsedTime(&ms, a, b);
        sum += ms;
        if (ms < best) { best = ms; hipMemcpy(&h, st, sizeof(Stats), hipMemcpyDeviceToHost); }
    }
    printf("%-12s mean %7.1f us best %7.1f us  %.2f TB/s (mean)", name, sum / 10 * 1e3, best * 1e3,
           (double)kIds * 8 / (sum / 10 * 1e-3) / 1e12);
    if (h.t0) {
        std::vector<double> e, ex[8];
        for (int i = 0; i < kMaxWaves; i++) if (h.end[i]) {
            e.push_back((h.end[i] - h.t0) / 100.0);
            ex[h.xcc[i] & 7].push_back((h.end[i] - h.t0) / 100.0);
        }
        std::sort(e.begin(), e.end());
        if (!e.empty())
            printf("  wave end us p10 %.1f p50 %.1f p90 %.1f max %.1f", e[e.size() / 10], e[e.size() / 2],
                   e[e.size() * 9 / 10], e.back());
        printf("\n   XCC MB:");
        for (int x = 0; x < 8; x++) printf(" %6.1f", h.xcc_bytes[x] / 1e6);
        printf("\n   XCC p50 end us:");
        for (int x = 0; x < 8; x++) {
            std::sort(ex[x].begin(), ex[x].end());
            printf(" %6.1f", ex[x].empty() ? 0.0 : ex[x][ex[x].size() / 2]);
        }
    }
    printf("\n");
}

int main() {
    int64_t *o;
    Stats *st;
    unsigned long long *ctr;
    hipMalloc(&o, kIds * 8 + 4096);
    hipMalloc(&st, sizeof(Stats));
    hipMalloc(&ctr, 64);
    const uint64_t n = kIds;
    for (auto fn : {(const void *)persist_r, (const void *)queue<8>, (const void *)queue<32>, (const void *)queue<128>,
                    (const void *)guided, (const void *)persist_bar<4, 8>, (const void *)persist_bar<8, 8>,
                    (const void *)persist_bar<8, 1>, (const void *)persist_bar<8, 0>, (const void *)persist_x<14>,
                    (const void *)persist_x<13>, (const void *)persist_x<12>, (const void *)persist_r16,
                    (const void *)persist_r16x, (const void *)persist_il<0>, (const void *)persist_il<8>,
                    (const void *)persist_il<64>, (const void *)persist_il<256>, (const void *)persist_phase<0>,
                    (const void *)persist_phase<1>, (const void *)persist_phase<2>, (const void *)persist_nt})
        (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    const size_t lds = 18220;   // 8 one-wave blocks per CU, as the replay
    for (int rep = 0; rep < 2; rep++) {
        timeit("oneshot4", st, ctr, [&](int s) { hipLaunchKernelGGL(oneshot4, dim3((uint32_t)((n / 4 + 255) / 256)), dim3(256), 0, 0, o, n, (int64_t)s); });
        timeit("persist_r", st, ctr, [&](int s) { hipLaunchKernelGGL(persist_r, dim3(kWaves), dim3(64), lds, 0, o, n, (int64_t)s, st); });
        timeit("persist_nt", st, ctr, [&](int s) { hipLaunchKernelGGL(persist_nt, dim3(kWaves), dim3(64), lds, 0, o, n, (int64_t)s, st); });
        timeit("oneshot_nt", st, ctr, [&](int s) { hipLaunchKernelGGL(oneshot_nt, dim3((uint32_t)((n / 4 + 255) / 256)), dim3(256), 0, 0, o, n, (int64_t)s); });
        timeit("phase_none", st, ctr, [&](int s) { hipLaunchKernelGGL(persist_phase<2>, dim3(kWaves), dim3(64), lds, 0, o, n, (int64_t)s, st); });
        timeit("phase_rot", st, ctr, [&](int s) { hipLaunchKernelGGL(persist_phase<0>, dim3(kWaves), dim3(64), lds, 0, o, n, (int64_t)s, st); });
        timeit("phase_skew", st, ctr, [&](int s) { hipLaunchKernelGGL(persist_phase<1>, dim3(kWaves), dim3(64), lds, 0, o, n, (int64_t)s, st); });
        if (rep == 0) continue;
        timeit("il_all", st, ctr, [&](int s) { hipLaunchKernelGGL(persist_il<0>, dim3(kWaves), dim3(64), lds, 0, o, n, (int64_t)s, st); });
        timeit("il_8", st, ctr, [&](int s) { hipLaunchKernelGGL(persist_il<8>, dim3(kWaves), dim3(64), lds, 0, o, n, (int64_t)s, st); });
        timeit("il_64", st, ctr, [&](int s) { hipLaunchKernelGGL(persist_il<64>, dim3(kWaves), dim3(64), lds, 0, o, n, (int64_t)s, st); });
        timeit("il_256", st, ctr, [&](int s) { hipLaunchKernelGGL(persist_il<256>, dim3(kWaves), dim3(64), lds, 0, o, n, (int64_t)s, st); });
        if (rep == 0) continue;
        timeit("persist_r16", st, ctr, [&](int s) { hipLaunchKernelGGL(persist_r16, dim3(kWaves), dim3(64), lds, 0, o, n, (int64_t)s, st); });
        timeit("persist_r16x", st, ctr, [&](int s) { hipLaunchKernelGGL(persist_r16x, dim3(kWaves), dim3(64), lds, 0, o, n, (int64_t)s, st); });
        timeit("persist_4096", st, ctr, [&](int s) { hipLaunchKernelGGL(persist_r, dim3(4096), dim3(64), lds, 0, o, n, (int64_t)s, st); });
        timeit("persist_8192", st, ctr, [&](int s) { hipLaunchKernelGGL(persist_r, dim3(8192), dim3(64), lds, 0, o, n, (int64_t)s, st); });
        timeit("r16_8192", st, ctr, [&](int s) { hipLaunchKernelGGL(persist_r16, dim3(8192), dim3(64), lds, 0, o, n, (int64_t)s, st); });
        if (rep == 0) continue;
        timeit("queue_256K", st, ctr, [&](int s) { hipLaunchKernelGGL(queue<128>, dim3(kWaves), dim3(64), lds, 0, o, n, (int64_t)s, st, ctr); });
        timeit("xsplit_14", st, ctr, [&](int s) { hipLaunchKernelGGL(persist_x<14>, dim3(kWaves), dim3(64), lds, 0, o, n, (int64_t)s, st); });
        timeit("xsplit_13", st, ctr, [&](int s) { hipLaunchKernelGGL(persist_x<13>, dim3(kWaves), dim3(64), lds, 0, o, n, (int64_t)s, st); });
        timeit("xsplit_12", st, ctr, [&](int s) { hipLaunchKernelGGL(persist_x<12>, dim3(kWaves), dim3(64), lds, 0, o, n, (int64_t)s, st); });
        timeit("bar4_k8", st, ctr, [&](int s) { hipLaunchKernelGGL((persist_bar<4, 8>), dim3(kWaves / 4), dim3(256), lds * 4, 0, o, n, (int64_t)s, st); });
        timeit("bar8_k8", st, ctr, [&](int s) { hipLaunchKernelGGL((persist_bar<8, 8>), dim3(kWaves / 8), dim3(512), lds * 8, 0, o, n, (int64_t)s, st); });
        timeit("bar8_k1", st, ctr, [&](int s) { hipLaunchKernelGGL((persist_bar<8, 1>), dim3(kWaves / 8), dim3(512), lds * 8, 0, o, n, (int64_t)s, st); });
        timeit("bar8_k0", st, ctr, [&](int s) { hipLaunchKernelGGL((persist_bar<8, 0>), dim3(kWaves / 8), dim3(512), lds * 8, 0, o, n, (int64_t)s, st); });
    }
    hipError_t e = hipDeviceSynchronize();
    printf("status %s\n", hipGetErrorString(e));
    return 0;
}
