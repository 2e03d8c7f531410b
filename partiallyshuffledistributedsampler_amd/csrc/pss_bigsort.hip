// pss_bigsort.hip -- pool permutations too large for one workgroup's LDS (n > 16384; e.g.
// shuffle_buffer = 2^20).  Same definition as the LDS path: perm = stable
// argsort of 32-bit Philox keys (ties by index), evaluated as an HBM multi-pass:
//
//   k_bs_count    per 16K-element chunk: LDS histogram of the top hb key bits -> global counts
//   k_bs_scan     per job: exclusive scan of the 2^hb bucket counts (wave64 DPP scan)
//   k_bs_scatter  per chunk: reserve a range per bucket (one global atomic per bucket and
//                 chunk), scatter (key << 32 | index) into bucket order
//   k_bs_bucket   per bucket (~512..1024 entries): LDS bitonic sort of the 64-bit pairs
//
// hb = ceil(log2 nmax) - 10, so buckets average <= 1024 entries and hold at most kBucketCap
// (8192) -- exceeding that flags error 2 (probability ~e^-5000 for Philox keys).
#include "pss_device.h"

namespace pss {


constexpr int BS_QPT = 16;                      // quads per thread
constexpr int BS_CHUNK = 256 * BS_QPT * 4;      // elements per chunk (16384)

__host__ __device__ static inline int64_t cdivl(int64_t a, int64_t b) { return (a + b - 1) / b; }

static int bs_hb(int64_t nmax) {
    int hb = ceil_log2_u64((uint64_t)nmax) - 10;
    if (hb < 0) hb = 0;
    if (hb > 14) hb = 14;                       // LDS histogram of the chunk kernels
    return hb;
}

static inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

__device__ __forceinline__ uint32_t bucket_of(uint32_t key, int hb) {
    return hb ? key >> (32 - hb) : 0u;
}

__global__ __launch_bounds__(256) void k_bs_count(Geometry g, SortJobs J, int64_t job_lo,
                                                  BigSortWS ws) {
    extern __shared__ __attribute__((aligned(16))) uint32_t h[];
    const int64_t jj = blockIdx.y;
    uint32_t rank, c1;
    int64_t n;
    sort_job(J, job_lo + jj, rank, c1, n);
    const int64_t e0 = (int64_t)blockIdx.x * BS_CHUNK;
    for (int i = threadIdx.x; i < ws.nb; i += 256) h[i] = 0;
    __syncthreads();
    if (e0 < n) {
        for (int q = 0; q < BS_QPT; q++) {
            const int64_t quad = e0 / 4 + q * 256 + threadIdx.x;
            if (quad * 4 >= n) break;
            uint32_t c0 = (uint32_t)quad, cc1 = c1, c2 = rank, c3 = J.dom;
            philox4x32_10(c0, cc1, c2, c3, g.key0, g.key1);
            const uint32_t k[4] = {c0, cc1, c2, c3};
#pragma unroll
            for (int w = 0; w < 4; w++)
                if (quad * 4 + w < n) atomicAdd(&h[bucket_of(k[w], ws.hb)], 1u);
        }
    }
    __syncthreads();
    uint32_t *cnt = ws.start + jj * (ws.nb + 1);
    for (int i = threadIdx.x; i < ws.nb; i += 256)
        if (h[i]) atomicAdd(&cnt[i], h[i]);
}

__global__ __launch_bounds__(1024) void k_bs_scan(SortJobs J, int64_t job_lo, BigSortWS ws) {
    __shared__ uint32_t tot[16];
    const int64_t jj = blockIdx.x;
    uint32_t rank, c1;
    int64_t n;
    sort_job(J, job_lo + jj, rank, c1, n);
    uint32_t *st = ws.start + jj * (ws.nb + 1);
    uint32_t *cu = ws.cur + jj * ws.nb;
    const int64_t per = cdivl(ws.nb, 1024);
    int64_t lo = (int64_t)threadIdx.x * per;
    if (lo > ws.nb) lo = ws.nb;
    const int64_t hi = lo + per < ws.nb ? lo + per : ws.nb;
    uint32_t s = 0;
    for (int64_t i = lo; i < hi; i++) s += st[i];
    uint32_t total;
    uint32_t run = block_excl_scan<1024>(s, tot, total);
    for (int64_t i = lo; i < hi; i++) { const uint32_t c = st[i]; st[i] = run; cu[i] = run; run += c; }
    if (threadIdx.x == 0) st[ws.nb] = (uint32_t)n;
}

__global__ __launch_bounds__(256) void k_bs_scatter(Geometry g, SortJobs J, int64_t job_lo,
                                                    BigSortWS ws) {
    extern __shared__ __attribute__((aligned(16))) uint32_t h[];
    uint32_t *base = h + ws.nb;
    const int64_t jj = blockIdx.y;
    uint32_t rank, c1;
    int64_t n;
    sort_job(J, job_lo + jj, rank, c1, n);
    const int64_t e0 = (int64_t)blockIdx.x * BS_CHUNK;
    if (e0 >= n) return;                        // uniform per block
    for (int i = threadIdx.x; i < ws.nb; i += 256) h[i] = 0;
    __syncthreads();
    uint32_t key[BS_QPT][4];
#pragma unroll
    for (int q = 0; q < BS_QPT; q++) {
        const int64_t quad = e0 / 4 + q * 256 + threadIdx.x;
        uint32_t c0 = (uint32_t)quad, cc1 = c1, c2 = rank, c3 = J.dom;
        philox4x32_10(c0, cc1, c2, c3, g.key0, g.key1);
        key[q][0] = c0; key[q][1] = cc1; key[q][2] = c2; key[q][3] = c3;
#pragma unroll
        for (int w = 0; w < 4; w++)
            if (quad * 4 + w < n) atomicAdd(&h[bucket_of(key[q][w], ws.hb)], 1u);
    }
    __syncthreads();
    uint32_t *cu = ws.cur + jj * ws.nb;
    for (int i = threadIdx.x; i < ws.nb; i += 256) {
        const uint32_t c = h[i];
        if (c) base[i] = atomicAdd(&cu[i], c);
        h[i] = 0;
    }
    __syncthreads();
    uint64_t *tmp = ws.tmp + jj * ws.nmax;
#pragma unroll
    for (int q = 0; q < BS_QPT; q++) {
        const int64_t quad = e0 / 4 + q * 256 + threadIdx.x;
#pragma unroll
        for (int w = 0; w < 4; w++) {
            const int64_t i = quad * 4 + w;
            if (i < n) {
                const uint32_t b = bucket_of(key[q][w], ws.hb);
                const uint32_t pos = base[b] + atomicAdd(&h[b], 1u);
                tmp[pos] = ((uint64_t)key[q][w] << 32) | (uint64_t)(uint32_t)i;
            }
        }
    }
}

__global__ __launch_bounds__(256) void k_bs_bucket(SortJobs J, int64_t job_lo, BigSortWS ws,
                                                   int32_t *err) {
    __shared__ uint64_t v[kBucketCap];
    const int64_t jj = blockIdx.y;
    const int64_t b = blockIdx.x;
    const uint32_t *st = ws.start + jj * (ws.nb + 1);
    const uint32_t s0 = st[b], s1 = st[b + 1];
    const int m = (int)(s1 - s0);
    if (m <= 0) return;
    if (m > kBucketCap) {
        if (threadIdx.x == 0) atomicOr(err, 2);
        return;
    }
    int P = 1;
    while (P < m) P <<= 1;
    const uint64_t *src = ws.tmp + jj * ws.nmax + s0;
    for (int i = threadIdx.x; i < P; i += 256) v[i] = i < m ? src[i] : ~0ull;
    __syncthreads();
    for (int k = 2; k <= P; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < P; i += 256) {
                const int ixj = i ^ j;
                if (ixj > i) {
                    const uint64_t a = v[i], c = v[ixj];
                    const bool up = (i & k) == 0;
                    if ((a > c) == up) { v[i] = c; v[ixj] = a; }
                }
            }
            __syncthreads();
        }
    }
    uint32_t *dst = ws.perm + jj * ws.nmax + s0;
    for (int i = threadIdx.x; i < m; i += 256) dst[i] = (uint32_t)v[i];
}


size_t big_sort_bytes(int64_t nmax, int64_t nj) {
    const int64_t nb = (int64_t)1 << bs_hb(nmax);
    return align256((size_t)nj * (nb + 1) * 4) + align256((size_t)nj * nb * 4) +
           align256((size_t)nj * nmax * 8) + align256((size_t)nj * nmax * 4);
}

BigSortWS big_sort_ws(void *base, int64_t nmax, int64_t nj) {
    BigSortWS w{};
    w.hb = bs_hb(nmax);
    w.nb = (int64_t)1 << w.hb;
    w.nmax = nmax;
    char *p = (char *)base;
    w.start = (uint32_t *)p; p += align256((size_t)nj * (w.nb + 1) * 4);
    w.cur = (uint32_t *)p;   p += align256((size_t)nj * w.nb * 4);
    w.tmp = (uint64_t *)p;   p += align256((size_t)nj * nmax * 8);
    w.perm = (uint32_t *)p;
    return w;
}

int64_t big_sort_batch(int64_t nmax, int64_t njobs, size_t budget) {
    const size_t per = big_sort_bytes(nmax, 1);
    int64_t j = (int64_t)(budget / (per ? per : 1));
    if (j < 1) j = 1;
    return j < njobs ? j : njobs;
}

hipError_t launch_big_sort(const Geometry &g, const SortJobs &J, int64_t job_lo, int64_t nj,
                           const BigSortWS &ws, int32_t *err, hipStream_t s) {
    if (nj <= 0) return hipSuccess;
    if (J.nmax > ((int64_t)1 << 26)) return hipErrorNotSupported;
    hipError_t e = hipMemsetAsync(ws.start, 0, (size_t)nj * (ws.nb + 1) * 4, s);
    if (e != hipSuccess) return e;
    const dim3 chunks((uint32_t)cdivl(J.nmax, BS_CHUNK), (uint32_t)nj);
    hipLaunchKernelGGL(k_bs_count, chunks, dim3(256), (size_t)ws.nb * 4, s, g, J, job_lo, ws);
    hipLaunchKernelGGL(k_bs_scan, dim3((uint32_t)nj), dim3(1024), 0, s, J, job_lo, ws);
    hipLaunchKernelGGL(k_bs_scatter, chunks, dim3(256), (size_t)ws.nb * 8, s, g, J, job_lo, ws);
    hipLaunchKernelGGL(k_bs_bucket, dim3((uint32_t)ws.nb, (uint32_t)nj), dim3(256), 0, s, J, job_lo, ws, err);
    return hipGetLastError();
}

hipError_t init_kernel_attributes_bigsort() {
    const int big = 160 * 1024;
    hipError_t e = hipFuncSetAttribute((const void *)k_bs_scatter, hipFuncAttributeMaxDynamicSharedMemorySize, big);
    hipError_t e2 = hipFuncSetAttribute((const void *)k_bs_count, hipFuncAttributeMaxDynamicSharedMemorySize, big);
    return e != hipSuccess ? e : e2;
}

}  // namespace pss
