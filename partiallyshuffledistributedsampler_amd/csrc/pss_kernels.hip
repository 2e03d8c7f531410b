// pss_kernels.hip -- gfx950 (MI355X / CDNA4) kernels of the partial-shuffle sampler:
// prologue (scan + partition), V1 generation, id -> (file, offset) map, coverage digest.
// V2 lives in pss_v2.hip, pools beyond LDS in pss_bigsort.hip, primitives in pss_device.h.
//
// The hot path of the reference (index generation, V1:157-172 / V2:96-116, and the id ->
// (file, offset) scan, V1:181-221) is restated as integer, HBM-write-bound kernels:
//
//   k_scan_partial/_final  exclusive scan of files_len over the shuffled file order (wave64 DPP)
//   k_part_*           balanced file -> rank partition (segments of each rank's id block)
//   k_v1_lds<EPT>      V1: one workgroup per (rank, window); pool permutation = stable sort
//                      of Philox keys in LDS (bucket pass on the top key bits + fix-up)
//   k_v1_write_big     V1 windows > 16384: ids from the HBM multi-pass sort
//   k_map, k_digest    id -> (file position, offset); coverage digest for the RCCL check
//
// Schedule definitions: DESIGN.md §3, restated on the CPU in oracle/pss_oracle.c
// (orc_v1_philox_stream / orc_v2_philox_stream); both must agree bit for bit.  No MFMA
// anywhere -- this is integer, memory/latency-bound work.
#include <cstdlib>

#include "pss_device.h"

namespace pss {

// ------------------------------------------------------------------------------------------
// scan + partition (V1:27-53,181-190 / V2:27-49,184-193)
// ------------------------------------------------------------------------------------------
// Two passes over chunks of 4096 files (256 threads x 16, coalesced order reads):
// k_scan_partial sums each chunk; k_scan_final adds the sums of the chunks before its own and
// scans its chunk with 16 workgroup DPP scans.  One chunk (F <= 4096) skips the first pass.
constexpr int kScanChunk = 4096;

__device__ __forceinline__ uint64_t block_sum256(uint64_t x, uint64_t *tot) {
    uint64_t total;
    (void)block_excl_scan<256>(x, tot, total);
    return total;
}

__global__ __launch_bounds__(256) void k_scan_partial(const int64_t *__restrict__ lens,
                                                      const int32_t *__restrict__ order,
                                                      int64_t F, uint64_t *__restrict__ part) {
    __shared__ uint64_t tot[4];
    const int64_t base = (int64_t)blockIdx.x * kScanChunk;
    uint64_t s = 0;
#pragma unroll
    for (int j = 0; j < kScanChunk / 256; j++) {
        const int64_t f = base + j * 256 + threadIdx.x;
        if (f < F) s += (uint64_t)lens[order[f]];
    }
    const uint64_t total = block_sum256(s, tot);
    if (threadIdx.x == 0) part[blockIdx.x] = total;
}

__global__ __launch_bounds__(256) void k_scan_final(const int64_t *__restrict__ lens,
                                                    const int32_t *__restrict__ order, int64_t F,
                                                    const uint64_t *__restrict__ part,
                                                    int64_t *__restrict__ prefix) {
    __shared__ uint64_t tot[4];
    const int64_t c = blockIdx.x;
    const int64_t base = c * kScanChunk;
    uint64_t x[kScanChunk / 256];
#pragma unroll
    for (int j = 0; j < kScanChunk / 256; j++) {       // all 16 gathers in flight
        const int64_t f = base + j * 256 + threadIdx.x;
        x[j] = f < F ? (uint64_t)lens[order[f]] : 0;
    }
    uint64_t cs = 0;
    for (int64_t i = threadIdx.x; i < c; i += 256) cs += part[i];
    uint64_t carry = block_sum256(cs, tot);
#pragma unroll
    for (int j = 0; j < kScanChunk / 256; j++) {
        const int64_t f = base + j * 256 + threadIdx.x;
        uint64_t total;
        const uint64_t ex = block_excl_scan<256>(x[j], tot, total);
        if (f < F) prefix[f] = (int64_t)(carry + ex);
        carry += total;
    }
    if (c == gridDim.x - 1 && threadIdx.x == 0) prefix[F] = (int64_t)carry;
}

// largest f in [0, F) with prefix[f] <= id  (the file holding id; empty files are skipped
// because an empty file shares its prefix with the next one)
__device__ __forceinline__ int64_t file_of(const int64_t *prefix, int64_t F, int64_t id) {
    int64_t lo = 0, hi = F;
    while (hi - lo > 1) {
        const int64_t mid = (lo + hi) >> 1;
        if (prefix[mid] <= id) lo = mid; else hi = mid;
    }
    return lo;
}

// The id ranges a rank reads in one epoch, in stream order, wrapped at N and clipped to the
// scanned total T = prefix[F] (ids >= T are reflected, V1:191-196).
struct Ranges { int64_t lo[4], hi[4]; int n; };

__device__ void rank_ranges(const Geometry &g, const RankDesc &rd, int64_t T, Ranges &r) {
    int64_t plo[2], plen[2];
    int np = 0;
    if (g.version == 1) {
        plo[0] = rd.new_start; plen[0] = g.ns; np = 1;
    } else {
        const int64_t a = 2 * g.B < g.ns ? 2 * g.B : g.ns;
        plo[0] = rd.old_start; plen[0] = a; np = 1;
        if (g.ns > a) { plo[1] = rd.new_start + a; plen[1] = g.ns - a; np = 2; }
    }
    r.n = 0;
    for (int i = 0; i < np; i++) {
        int64_t lo = plo[i] % g.N, len = plen[i];
        while (len > 0) {
            const int64_t take = (g.N - lo) < len ? (g.N - lo) : len;
            int64_t h = lo + take;
            const int64_t l = lo;
            if (h > T) h = T;
            if (l < h) { r.lo[r.n] = l; r.hi[r.n] = h; r.n++; }
            len -= take;
            lo = 0;
        }
    }
}

__global__ void k_part_count(Geometry g, const RankDesc *ranks, int32_t rank_lo, int32_t nr,
                             const int64_t *prefix, int64_t F, int64_t *seg_off) {
    const int64_t T = prefix[F];
    for (int32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nr; i += gridDim.x * blockDim.x) {
        Ranges rr;
        rank_ranges(g, ranks[rank_lo + i], T, rr);
        int64_t c = 0;
        for (int k = 0; k < rr.n; k++) {
            const int64_t f0 = file_of(prefix, F, rr.lo[k]);
            const int64_t f1 = file_of(prefix, F, rr.hi[k] - 1);
            for (int64_t f = f0; f <= f1; f++) c += prefix[f + 1] > prefix[f];
        }
        seg_off[i + 1] = c;
    }
}

__global__ __launch_bounds__(1024) void k_excl_scan_inplace(int64_t *a, int64_t n) {
    // a[0] := 0, a[1..n] := inclusive scan of counts stored in a[1..n]
    __shared__ uint64_t tot[16];
    const int64_t per = (n + 1023) / 1024;
    int64_t lo = (int64_t)threadIdx.x * per;
    if (lo > n) lo = n;
    const int64_t hi = lo + per < n ? lo + per : n;
    uint64_t s = 0;
    for (int64_t i = lo; i < hi; i++) s += (uint64_t)a[i + 1];
    uint64_t total;
    uint64_t run = block_excl_scan<1024>(s, tot, total);
    for (int64_t i = lo; i < hi; i++) { run += (uint64_t)a[i + 1]; a[i + 1] = (int64_t)run; }
    if (threadIdx.x == 0) a[0] = 0;
}

__global__ void k_part_emit(Geometry g, const RankDesc *ranks, int32_t rank_lo, int32_t nr,
                            const int64_t *prefix, int64_t F, const int64_t *seg_off,
                            int32_t *seg_file, int64_t *seg_lo, int64_t *seg_hi,
                            int64_t seg_cap, int32_t *err) {
    const int64_t T = prefix[F];
    for (int32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nr; i += gridDim.x * blockDim.x) {
        Ranges rr;
        rank_ranges(g, ranks[rank_lo + i], T, rr);
        int64_t o = seg_off[i];
        if (seg_off[i + 1] > seg_cap) { atomicOr(err, 1); continue; }
        for (int k = 0; k < rr.n; k++) {
            const int64_t f0 = file_of(prefix, F, rr.lo[k]);
            const int64_t f1 = file_of(prefix, F, rr.hi[k] - 1);
            for (int64_t f = f0; f <= f1; f++) {
                if (prefix[f + 1] <= prefix[f]) continue;
                const int64_t a = rr.lo[k] > prefix[f] ? rr.lo[k] : prefix[f];
                const int64_t b = rr.hi[k] < prefix[f + 1] ? rr.hi[k] : prefix[f + 1];
                seg_file[o] = (int32_t)f;
                seg_lo[o] = a - prefix[f];
                seg_hi[o] = b - prefix[f];
                o++;
            }
        }
    }
}

// id -> (file position, offset) over the shuffled order (V1:181-221).  Ids at or past the
// scanned total are reflected exactly as V1:191-196 does; the host moves those to the end of
// their batch (they are flagged by a negative file position: fpos = -1 - f).
__global__ void k_map(const int64_t *__restrict__ prefix, int64_t F,
                      const int64_t *__restrict__ ids, int64_t n, int32_t *__restrict__ fpos,
                      int64_t *__restrict__ off) {
    const int64_t T = prefix[F];
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        int64_t id = ids[i];
        bool refl = false;
        if (id >= T) {
            id = 2 * T - id;
            if (id == T) id = T - 1;
            refl = true;
        }
        if (id < 0) { fpos[i] = INT32_MIN; off[i] = ids[i]; continue; }
        const int64_t f = file_of(prefix, F, id);
        fpos[i] = refl ? (int32_t)(-1 - f) : (int32_t)f;
        off[i] = id - prefix[f];
    }
}

__global__ void k_digest(const int64_t *__restrict__ ids, int64_t n, uint64_t *acc) {
    uint64_t s = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        s += mix64((uint64_t)ids[i]);
    s = wave_sum(s);
    if ((threadIdx.x & 63) == 0) atomicAdd((unsigned long long *)acc, (unsigned long long)s);
}

__global__ void k_digest_range(int64_t lo, int64_t hi, uint64_t *acc) {
    uint64_t s = 0;
    for (int64_t i = lo + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < hi;
         i += (int64_t)gridDim.x * blockDim.x)
        s += mix64((uint64_t)i);
    s = wave_sum(s);
    if ((threadIdx.x & 63) == 0) atomicAdd((unsigned long long *)acc, (unsigned long long)s);
}

__global__ void k_debug_wave_scan(const uint64_t *in, uint64_t *out, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t x = i < n ? in[i] : 0;
    const uint64_t y = wave_incl_scan(x);
    const uint32_t y32 = wave_incl_scan((uint32_t)x);
    if (i < n) { out[2 * i] = y; out[2 * i + 1] = y32; }
}

// ------------------------------------------------------------------------------------------
// V1 (V1:157-172): window w of rank r -> ids start + w*B + perm_w[p], wrap at N
// ------------------------------------------------------------------------------------------
template <int EPT, int NT>
__global__ __launch_bounds__(NT) void k_v1_lds(Geometry g, const RankDesc *__restrict__ ranks,
                                               int32_t rank_lo, int64_t w_lo, int64_t nw,
                                               int64_t pos_lo, int64_t count,
                                               int64_t *__restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    uint32_t *S = smem, *hist = smem + NT * EPT, *tot = hist + bpad_size(NT * EPT);
    const int32_t rl = (int32_t)(blockIdx.x / nw);
    const int64_t w = w_lo + (int64_t)(blockIdx.x % nw);
    const int32_t rank = rank_lo + rl;
    const int64_t wb = w * g.B;
    const int64_t n = g.ns - wb < g.B ? g.ns - wb : g.B;
    const int64_t base = ranks[rank].new_start + wb;
    int hb = 0;
    if (g.shuffle) hb = block_sort_keys<EPT, NT>(g.key0, g.key1, (uint32_t)w, (uint32_t)rank, DOM_V1_WIN, (int)n, S, hist, tot);
    const uint32_t mask = (1u << hb) - 1u;
    int64_t *o = out + (int64_t)rl * count - pos_lo;
    int64_t p0 = 0, p1 = n;
    if (wb < pos_lo) p0 = pos_lo - wb;
    if (wb + n > pos_lo + count) p1 = pos_lo + count - wb;
    for (int64_t p = p0 + threadIdx.x; p < p1; p += NT) {
        const uint32_t idx = g.shuffle ? (S[p] & mask) : (uint32_t)p;
        o[wb + p] = wrap_id(base + idx, g.N);
    }
}

__global__ __launch_bounds__(256) void k_v1_write_big(Geometry g, const RankDesc *__restrict__ ranks,
                                                     SortJobs J, int64_t job_lo, BigSortWS ws,
                                                     int64_t pos_lo, int64_t count,
                                                     int64_t *__restrict__ out) {
    const int64_t jj = blockIdx.y;
    uint32_t rank, w;
    int64_t n;
    sort_job(J, job_lo + jj, rank, w, n);
    const int64_t rl = (int64_t)rank - J.rank_lo;
    const int64_t wb = (int64_t)w * g.B;
    const int64_t base = ranks[rank].new_start + wb;
    const uint32_t *perm = ws.perm + jj * ws.nmax;
    int64_t *o = out + rl * count - pos_lo;
    const int64_t pos_hi = pos_lo + count;
    for (int64_t p = (int64_t)blockIdx.x * 1024 + threadIdx.x; p < n && p < (int64_t)(blockIdx.x + 1) * 1024; p += 256) {
        const int64_t pos = wb + p;
        if (pos >= pos_lo && pos < pos_hi) o[pos] = wrap_id(base + perm[p], g.N);
    }
}

// ------------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------------
static inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

struct RankArgs { RankDesc r[kArgRanks]; };

__global__ __launch_bounds__(kArgRanks) void k_put_ranks(RankArgs a, int32_t n, RankDesc *dst) {
    if ((int32_t)threadIdx.x < n) dst[threadIdx.x] = a.r[threadIdx.x];
}

hipError_t launch_put_ranks(const RankDesc *host, int32_t R, RankDesc *dst, hipStream_t s) {
    for (int32_t r0 = 0; r0 < R; r0 += kArgRanks) {
        RankArgs a;
        const int32_t n = R - r0 < kArgRanks ? R - r0 : kArgRanks;
        for (int32_t i = 0; i < n; i++) a.r[i] = host[r0 + i];
        hipLaunchKernelGGL(k_put_ranks, dim3(1), dim3(kArgRanks), 0, s, a, n, dst + r0);
    }
    return hipGetLastError();
}

size_t scan_scratch_words(int64_t F) { return (size_t)cdiv(F > 0 ? F : 1, kScanChunk); }

hipError_t launch_scan_prefix(const int64_t *lens, const int32_t *order, int64_t F,
                              int64_t *prefix, uint64_t *scratch, hipStream_t s) {
    const int64_t nc = cdiv(F > 0 ? F : 1, kScanChunk);
    if (nc > 1)
        hipLaunchKernelGGL(k_scan_partial, dim3((uint32_t)nc), dim3(256), 0, s, lens, order, F, scratch);
    hipLaunchKernelGGL(k_scan_final, dim3((uint32_t)nc), dim3(256), 0, s, lens, order, F,
                       (const uint64_t *)scratch, prefix);
    return hipGetLastError();
}

hipError_t launch_partition(const Geometry &g, const RankDesc *ranks, int32_t rank_lo,
                            int32_t nr, const int64_t *prefix, int64_t F, int64_t *seg_off,
                            int32_t *seg_file, int64_t *seg_lo, int64_t *seg_hi,
                            int64_t seg_cap, int32_t *err, hipStream_t s) {
    if (nr <= 0) return hipSuccess;
    const int blocks = (int)cdiv(nr, 256);
    hipLaunchKernelGGL(k_part_count, dim3(blocks), dim3(256), 0, s, g, ranks, rank_lo, nr, prefix, F, seg_off);
    hipLaunchKernelGGL(k_excl_scan_inplace, dim3(1), dim3(1024), 0, s, seg_off, (int64_t)nr);
    if (seg_cap > 0)
        hipLaunchKernelGGL(k_part_emit, dim3(blocks), dim3(256), 0, s, g, ranks, rank_lo, nr, prefix, F,
                           (const int64_t *)seg_off, seg_file, seg_lo, seg_hi, seg_cap, err);
    return hipGetLastError();
}

static inline int grid_for(int64_t n, int bs) {
    int64_t b = cdiv(n, bs);
    if (b > 8192) b = 8192;
    if (b < 1) b = 1;
    return (int)b;
}

hipError_t launch_map(const int64_t *prefix, int64_t F, const int64_t *ids, int64_t n,
                      int32_t *fpos, int64_t *off, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_map, dim3(grid_for(n, 256)), dim3(256), 0, s, prefix, F, ids, n, fpos, off);
    return hipGetLastError();
}

hipError_t launch_digest(const int64_t *ids, int64_t n, uint64_t *acc, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_digest, dim3(grid_for(n, 256)), dim3(256), 0, s, ids, n, acc);
    return hipGetLastError();
}

hipError_t launch_digest_range(int64_t lo, int64_t hi, uint64_t *acc, hipStream_t s) {
    if (hi <= lo) return hipSuccess;
    hipLaunchKernelGGL(k_digest_range, dim3(grid_for(hi - lo, 256)), dim3(256), 0, s, lo, hi, acc);
    return hipGetLastError();
}

hipError_t launch_debug_wave_scan(const uint64_t *in, uint64_t *out, int64_t n, hipStream_t s) {
    hipLaunchKernelGGL(k_debug_wave_scan, dim3(cdiv(n, 256)), dim3(256), 0, s, in, out, n);
    return hipGetLastError();
}

template <int EPT, int NT = 256>
static void launch_v1_ept(const Geometry &g, const RankDesc *ranks, int32_t rank_lo, int32_t nr,
                          int64_t w_lo, int64_t nw, int64_t pos_lo, int64_t count, int64_t *out,
                          hipStream_t s) {
    const size_t lds = g.shuffle ? sort_lds_bytes<EPT, NT>() : 16;
    hipLaunchKernelGGL(HIP_KERNEL_NAME(k_v1_lds<EPT, NT>), dim3((uint32_t)(nr * nw)), dim3(NT), lds, s,
                       g, ranks, rank_lo, w_lo, nw, pos_lo, count, out);
}

static bool v1_window_range(const Geometry &g, int64_t pos_lo, int64_t count, int64_t &w_lo,
                            int64_t &nw) {
    const int64_t pos_hi = pos_lo + count < g.ns ? pos_lo + count : g.ns;
    if (pos_hi <= pos_lo) return false;
    w_lo = pos_lo / g.B;
    nw = (pos_hi - 1) / g.B - w_lo + 1;
    return true;
}

static SortJobs v1_jobs(const Geometry &g, int32_t rank_lo, int64_t w_lo, int64_t nw) {
    SortJobs J{};
    J.kind = 0; J.rank_lo = rank_lo; J.nw = nw; J.w_lo = w_lo;
    J.B = g.B; J.ns = g.ns; J.P1 = 0; J.dom = DOM_V1_WIN;
    J.nmax = g.B < g.ns ? g.B : g.ns;
    return J;
}

size_t v1_workspace_bytes(const Geometry &g, int32_t nr, int64_t pos_lo, int64_t count) {
    int64_t w_lo, nw;
    const int64_t nmax = g.B < g.ns ? g.B : g.ns;
    if (!g.shuffle || nmax <= kLdsSortMax || nr <= 0 || !v1_window_range(g, pos_lo, count, w_lo, nw))
        return 0;
    const int64_t jb = big_sort_batch(nmax, (int64_t)nr * nw, kBigSortBudget);
    return big_sort_bytes(nmax, jb);
}

hipError_t launch_v1(const Geometry &g, const RankDesc *ranks, int32_t rank_lo, int32_t nr,
                     int64_t pos_lo, int64_t count, int64_t *out, uint32_t *sort_ws,
                     int32_t *err, hipStream_t s, const Marker &mk) {
    int64_t w_lo, nw;
    if (nr <= 0 || !v1_window_range(g, pos_lo, count, w_lo, nw)) return hipSuccess;
    const int64_t nmax = g.B < g.ns ? g.B : g.ns;
    mk(K_V1, s);
    static const int v1_nt = [] {   // experiment knob: threads per window workgroup
        const char *e = getenv("PSS_V1_NT");   // 512 measured fastest at B = 4096 (C2 V1: 0.39 ms
        return e ? atoi(e) : 512;              // vs 0.51 ms at 256 and 1024 threads)
    }();
    if (!g.shuffle || nmax <= 1024) launch_v1_ept<4>(g, ranks, rank_lo, nr, w_lo, nw, pos_lo, count, out, s);
    else if (nmax <= 4096 && v1_nt == 1024) launch_v1_ept<4, 1024>(g, ranks, rank_lo, nr, w_lo, nw, pos_lo, count, out, s);
    else if (nmax <= 4096 && v1_nt == 512) launch_v1_ept<8, 512>(g, ranks, rank_lo, nr, w_lo, nw, pos_lo, count, out, s);
    else if (nmax <= 4096) launch_v1_ept<16>(g, ranks, rank_lo, nr, w_lo, nw, pos_lo, count, out, s);
    else if (nmax <= 8192 && v1_nt == 512) launch_v1_ept<16, 512>(g, ranks, rank_lo, nr, w_lo, nw, pos_lo, count, out, s);
    else if (nmax <= 8192) launch_v1_ept<32>(g, ranks, rank_lo, nr, w_lo, nw, pos_lo, count, out, s);
    else if (nmax <= kLdsSortMax) launch_v1_ept<64>(g, ranks, rank_lo, nr, w_lo, nw, pos_lo, count, out, s);
    else {
        // pools beyond LDS: HBM multi-pass sort, batches of jobs bounded by kBigSortBudget
        const SortJobs J = v1_jobs(g, rank_lo, w_lo, nw);
        const int64_t njobs = (int64_t)nr * nw;
        const int64_t jb = big_sort_batch(nmax, njobs, kBigSortBudget);
        const BigSortWS ws = big_sort_ws(sort_ws, nmax, jb);
        for (int64_t j0 = 0; j0 < njobs; j0 += jb) {
            const int64_t nj = njobs - j0 < jb ? njobs - j0 : jb;
            hipError_t e = launch_big_sort(g, J, j0, nj, ws, err, s);
            if (e != hipSuccess) return e;
            hipLaunchKernelGGL(k_v1_write_big, dim3((uint32_t)cdiv(nmax, 1024), (uint32_t)nj), dim3(256), 0, s,
                               g, ranks, J, j0, ws, pos_lo, count, out);
        }
    }
    mk(-1, s);
    return hipGetLastError();
}

hipError_t init_kernel_attributes() {
    const int big = 160 * 1024;
    hipError_t e = hipSuccess;
#define PSS_ATTR(fn) { hipError_t x = hipFuncSetAttribute((const void *)(fn), hipFuncAttributeMaxDynamicSharedMemorySize, big); if (x != hipSuccess) e = x; }
    PSS_ATTR((k_v1_lds<32, 256>));
    PSS_ATTR((k_v1_lds<64, 256>));
    PSS_ATTR((k_v1_lds<16, 512>));
#undef PSS_ATTR
    hipError_t e2 = init_kernel_attributes_v2();
    hipError_t e3 = init_kernel_attributes_bigsort();
    return e != hipSuccess ? e : (e2 != hipSuccess ? e2 : e3);
}

}  // namespace pss
