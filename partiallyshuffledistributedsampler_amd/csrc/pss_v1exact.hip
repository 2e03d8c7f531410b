// pss_v1exact.hip -- V1 window permutations in the reference's EXACT order (order mode
// PSS_ORDER_EXACT): window 0 is `seed(epoch); shuffle(range(len))` (V1:102,114-115), window
// b >= 1 is `seed(epoch + b*10000); shuffle(range(len))` (V1:165-171), both with CPython
// 3.10's MT19937 (`random.py:128-168` seeding, `:239-249` _randbelow, `:380-396` shuffle).
// Every window reseeds, so windows are independent: one 256-thread workgroup per
// (rank, window), three phases, for windows up to kV1ExactMaxB entries (LDS-resident); larger
// windows run the same three phases through HBM (k_v1x_*, below).
//
//   1. seeding (wave 0, uniform/scalar code): init_by_array over the compile-time
//      init_genrand(19650218) table -- two serial chains of 624 + 623 steps.
//   2. draws (wave 0): the state is twisted in LDS 64 words at a time and tempered on the
//      fly; the Fisher-Yates draws j_i = _randbelow(i + 1), i = n-1 .. 1, come out of a
//      64-word speculative block: lane l assumes the state i - (l - R_l), R_l = rejections
//      among lower lanes, and the block iterates R <- popc(ballot(reject) below l) to the
//      fixed point, which is the sequential answer (lane l is final after l passes; a
//      block settles in ~5).  j_i lands in LDS as u16.
//   3. permutation (all threads): the swap sequence is resolved without replaying it.  With
//      A_i(p) = value at position p just before the swap of step i,
//        x[i] = A_i(j_i);  A_i(p) = R(k) for the smallest k > i with j_k = p, else p;
//        R(k) = A_k(k)   = R(parent(k)), parent(k) = smallest k' > k with j_k' = k, else k.
//      Bucket the steps by j (count, scan, scatter), take parents from the buckets, pointer-
//      jump to the roots, and read each x[i] off its bucket.  tests/test_gpu_parity.py checks
//      the streams against oracle/pss_oracle.c's exact V1 (CPython restatement, pinned by the
//      reference's golden streams).
#include <cstdlib>

#include "pss_mt.h"

namespace pss {

namespace {
constexpr int kExactNT = 256;
}  // namespace

// Phases 1-2 alone, one wave per window (2.5 KB of LDS, so a CU holds 32 of them): the draws
// j_i of every window go to HBM (u16, B per window) for k_v1_exact's resolution.
__global__ __launch_bounds__(64) void k_v1x_draws(Geometry g, int64_t w_lo, int64_t nw, int64_t epoch,
                                                  uint16_t *__restrict__ J) {
    __shared__ uint32_t mt[kMtN];
    const int64_t w = w_lo + (int64_t)(blockIdx.x % nw);
    const int64_t wb = w * g.B;
    const int n = (int)(g.ns - wb < g.B ? g.ns - wb : g.B);
    if (n <= 1) return;
    uint16_t *jw = J + (size_t)blockIdx.x * (size_t)(g.B < g.ns ? g.B : g.ns);
    mt_seed_int(mt, w == 0 ? epoch : epoch + w * 10000);
    mt_draws(mt, (uint32_t)(n - 1), [&](uint32_t d) { return (uint32_t)n - d; },
             [&](uint32_t d, uint32_t r) { jw[n - 1 - (int)d] = (uint16_t)r; });
}

// One workgroup per (local rank, window) of [w_lo, w_lo + nw).
__global__ __launch_bounds__(kExactNT) void k_v1_exact(Geometry g, const RankDesc *__restrict__ ranks,
                                                       int32_t rank_lo, int64_t w_lo, int64_t nw,
                                                       int64_t pos_lo, int64_t count, int64_t epoch,
                                                       const uint16_t *__restrict__ J,
                                                       int64_t *__restrict__ out, MapArgs ma) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    const int32_t rl = (int32_t)(blockIdx.x / nw);
    const int64_t w = w_lo + (int64_t)(blockIdx.x % nw);
    const int32_t rank = rank_lo + rl;
    const int64_t wb = w * g.B;
    const int n = (int)(g.ns - wb < g.B ? g.ns - wb : g.B);
    const int tid = threadIdx.x, wid = tid >> 6;
    uint32_t *mt = smem;                                   // [624]
    uint32_t *cnt = smem + kMtN;                           // [n + 1] bucket counts -> ends
    uint16_t *jv = (uint16_t *)(cnt + n + 1);              // [n] j_i
    uint16_t *lst = jv + n;                                // [n] steps bucketed by j
    uint16_t *nxt = lst + n;                               // [n] parent -> root
    __shared__ uint32_t tot[kExactNT / 64];

    if (J) {                 // draws already made by k_v1x_draws
        const uint16_t *jw = J + (size_t)blockIdx.x * (size_t)(g.B < g.ns ? g.B : g.ns);
        for (int i = tid; i < n; i += kExactNT) jv[i] = jw[i];
    } else if (wid == 0 && n > 1) {
        // ---- 1. seed(a): key = 32-bit words of abs(a) (random_seed) ----
        mt_seed_int(mt, w == 0 ? epoch : epoch + w * 10000);
        // ---- 2. the draws of shuffle(range(n)): draw d is j_i = _randbelow(i + 1), i = n-1-d
        mt_draws(mt, (uint32_t)(n - 1), [&](uint32_t d) { return (uint32_t)n - d; },
                 [&](uint32_t d, uint32_t r) { jv[n - 1 - (int)d] = (uint16_t)r; });
    }
    // ---- 3. resolve the swap sequence (all threads) ----
    for (int p = tid; p <= n; p += kExactNT) cnt[p] = 0;
    __syncthreads();
    for (int k = 1 + tid; k < n; k += kExactNT) atomicAdd(&cnt[jv[k]], 1u);
    __syncthreads();
    {   // exclusive scan of cnt[0, n): contiguous chunks per thread
        const int per = (n + kExactNT - 1) / kExactNT;
        const int lo = tid * per, hi = lo + per < n ? lo + per : n;
        uint32_t sum = 0;
        for (int p = lo; p < hi; p++) sum += cnt[p];
        uint32_t total;
        uint32_t run = block_excl_scan<kExactNT>(sum, tot, total);
        for (int p = lo; p < hi; p++) { const uint32_t c = cnt[p]; cnt[p] = run; run += c; }
    }
    __syncthreads();
    for (int k = 1 + tid; k < n; k += kExactNT) lst[atomicAdd(&cnt[jv[k]], 1u)] = (uint16_t)k;
    __syncthreads();   // bucket p is lst[p ? cnt[p-1] : 0, cnt[p])
    auto succ = [&](int p, int above) -> int {   // smallest k > above in bucket p, or -1
        const int b0 = p ? (int)cnt[p - 1] : 0, b1 = (int)cnt[p];
        int best = -1;
        for (int x = b0; x < b1; x++) {
            const int k = lst[x];
            if (k > above && (best < 0 || k < best)) best = k;
        }
        return best;
    };
    for (int k = tid; k < n; k += kExactNT) {
        const int pk = succ(k, k);
        nxt[k] = (uint16_t)(pk < 0 ? k : pk);
    }
    __syncthreads();
    for (int round = 0; (1 << round) < n; round++) {   // pointer jumping to the chain roots
        for (int k = tid; k < n; k += kExactNT) nxt[k] = nxt[nxt[k]];
        __syncthreads();
    }
    // ---- output: x[i] for the positions of this window inside [pos_lo, pos_lo + count) ----
    const int64_t base = ranks[rank].new_start + wb;
    const int64_t ebase = (int64_t)rl * count - pos_lo;   // element of stream position 0
    int64_t p0 = 0, p1 = n;
    if (wb < pos_lo) p0 = pos_lo - wb;
    if (wb + n > pos_lo + count) p1 = pos_lo + count - wb;
    for (int64_t p = p0 + tid; p < p1; p += kExactNT) {
        const int i = (int)p;
        int x;
        if (n <= 1) {
            x = 0;
        } else if (i == 0) {
            const int k = succ(0, 0);
            x = k < 0 ? 0 : nxt[k];
        } else {
            const int pj = jv[i];
            if (pj == i) {
                x = nxt[i];
            } else {
                const int k = succ(pj, i);
                x = k < 0 ? pj : nxt[k];
            }
        }
        put_id_or_pair(out, ma, ebase + wb + p, wrap_id(base + x, g.N));
    }
}

// ---- windows beyond LDS (n > kV1ExactMaxB): the same resolution through HBM ----------------
// One pass covers `nj` jobs (rank, window) of the launch, jobs j0 .. j0 + nj - 1 (job -> local
// rank job / nw, window w_lo + job % nw), each with B-entry slices of four u32 arrays:
//   J   the draws j_i (k_v1x_draws32, one wave per window: the MT stream is serial)
//   CNT bucket counts of j -> exclusive offsets -> bucket ends (count, scan, scatter)
//   LST the steps bucketed by j
//   NXT parent(k) = the smallest k' > k with j_k' = k, else k
// and the output walks each x[i]'s parent chain to its root (expected length O(1): parent(k)
// is about k * U^-1 for a uniform U, so chains climb geometrically towards n).
struct V1xBig {
    int64_t w_lo, nw;       // windows of the launch
    uint64_t j0;            // first job of the pass
    uint32_t nj;            // jobs in the pass
    uint32_t B;             // slice length: min(shuffle_buffer, num_samples)
    uint32_t *J, *CNT, *LST, *NXT;
    uint32_t xb;            // 256-entry blocks per window (the flat kernels' x extent)
    uint32_t xcd;           // 1: XCD-major flat grid (v1x_block)
};

// The flat kernels (count, scatter, parent, out) make random accesses inside one window's
// slices.  XCD-major grid: workgroup L runs on XCD L mod 8 (round-robin dispatch), so block L is
// given window slot 8 (L / 8 / xb) + L mod 8 and entry block (L / 8) mod xb -- every window's
// blocks then run on one XCD, which keeps its slices' lines in that XCD's L2 instead of
// bouncing the atomics and reads of one window across all eight.  xcd = 0: blockIdx.y = slot.
__device__ __forceinline__ bool v1x_block(const V1xBig &b, uint32_t &slot, uint32_t &xblk) {
    if (!b.xcd) { slot = blockIdx.y; xblk = blockIdx.x; return true; }
    const uint32_t L = blockIdx.x, q = L >> 3;
    slot = 8u * (q / b.xb) + (L & 7u);
    xblk = q % b.xb;
    return slot < b.nj;
}

__device__ __forceinline__ int v1x_len(const Geometry &g, int64_t w) {
    const int64_t wb = w * g.B;
    return (int)(g.ns - wb < g.B ? g.ns - wb : g.B);
}

// Each draw also counts its bucket (CNT[j]++, a fire-and-forget atomic beside the latency-bound
// draws), so no counting pass re-reads J: C5 V1 exact 17.3 -> 15.4 ms (round 4, same box,
// profiles/r04/ab_v1x_fcount/)
__global__ __launch_bounds__(64) void k_v1x_draws32(Geometry g, V1xBig b, int64_t epoch) {
    __shared__ uint32_t mt[kMtN];
    const uint64_t job = b.j0 + blockIdx.x;
    const int64_t w = b.w_lo + (int64_t)(job % (uint64_t)b.nw);
    const int n = v1x_len(g, w);
    if (n <= 1) return;
    uint32_t *jw = b.J + (size_t)blockIdx.x * b.B;
    uint32_t *cnt = b.CNT + (size_t)blockIdx.x * ((size_t)b.B + 1);
    mt_seed_int(mt, w == 0 ? epoch : epoch + w * 10000);
    mt_draws(mt, (uint32_t)(n - 1), [&](uint32_t d) { return (uint32_t)n - d; },
             [&](uint32_t d, uint32_t r) {
                 jw[n - 1 - (int)d] = r;
                 atomicAdd(&cnt[r], 1u);
             });
}

// The same draws with a workgroup per window (pss_mt.h mt_draws_wg): few, long windows (C5: 2^20
// entries, ~12 per rank)
__global__ __launch_bounds__(kMtWgThreads) void k_v1x_draws32_wg(Geometry g, V1xBig b, int64_t epoch) {
    __shared__ MtWgShared sh;
    const uint64_t job = b.j0 + blockIdx.x;
    const int64_t w = b.w_lo + (int64_t)(job % (uint64_t)b.nw);
    const int n = v1x_len(g, w);
    if (n <= 1) return;
    uint32_t *jw = b.J + (size_t)blockIdx.x * b.B;
    uint32_t *cnt = b.CNT + (size_t)blockIdx.x * ((size_t)b.B + 1);
    if (threadIdx.x < 64) mt_seed_int(sh.mt[0], w == 0 ? epoch : epoch + w * 10000);
    __syncthreads();
    mt_draws_wg(sh, 0, (uint32_t)(n - 1), [&](uint32_t d) { return (uint32_t)n - d; },
                [&](uint32_t d, uint32_t r) {
                    jw[n - 1 - (int)d] = r;
                    atomicAdd(&cnt[r], 1u);
                });
}

// slot of the pass and block of the window's entries (v1x_block)
#define V1X_SLOT_PROLOGUE                                                          \
    uint32_t slot, xblk;                                                           \
    if (!v1x_block(b, slot, xblk)) return;                                         \
    const uint64_t job = b.j0 + slot;                                              \
    const int64_t w = b.w_lo + (int64_t)(job % (uint64_t)b.nw);                    \
    const int n = v1x_len(g, w);                                                   \
    const uint32_t *J = b.J + (size_t)slot * b.B;                                  \
    uint32_t *CNT = b.CNT + (size_t)slot * ((size_t)b.B + 1);                      \
    (void)J; (void)CNT;

// exclusive scan of CNT[0, n) in place, one workgroup per window, in tiles of kV1xScanNT x 8
// counts: coalesced loads into LDS (skewed one word per 32), each thread scans 8 consecutive
// counts, one block scan, coalesced stores.  (A thread per 1/1024 of the window, reading its
// stretch serially, had every load of a wave touch 64 cache lines: 2.2 ms at C5's windows.)
constexpr int kV1xScanNT = 1024, kV1xScanPer = 8, kV1xScanTile = kV1xScanNT * kV1xScanPer;
__global__ __launch_bounds__(kV1xScanNT) void k_v1x_scan(Geometry g, V1xBig b) {
    const uint32_t slot = blockIdx.x;
    const uint64_t job = b.j0 + slot;
    const int64_t w = b.w_lo + (int64_t)(job % (uint64_t)b.nw);
    const int n = v1x_len(g, w);
    uint32_t *CNT = b.CNT + (size_t)slot * ((size_t)b.B + 1);
    __shared__ uint32_t tot[kV1xScanNT / 64];
    __shared__ uint32_t st[kV1xScanTile + kV1xScanTile / 32];
    auto ix = [](int e) { return e + (e >> 5); };
    const int t = (int)threadIdx.x;
    uint32_t carry = 0;
    for (int base = 0; base < n; base += kV1xScanTile) {
#pragma unroll
        for (int i = 0; i < kV1xScanPer; i++) {
            const int e = i * kV1xScanNT + t;
            st[ix(e)] = base + e < n ? CNT[base + e] : 0u;
        }
        __syncthreads();
        uint32_t v[kV1xScanPer], sum = 0;
#pragma unroll
        for (int i = 0; i < kV1xScanPer; i++) { v[i] = st[ix(t * kV1xScanPer + i)]; sum += v[i]; }
        uint32_t total;
        uint32_t run = carry + block_excl_scan<kV1xScanNT>(sum, tot, total);
#pragma unroll
        for (int i = 0; i < kV1xScanPer; i++) { st[ix(t * kV1xScanPer + i)] = run; run += v[i]; }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < kV1xScanPer; i++) {
            const int e = i * kV1xScanNT + t;
            if (base + e < n) CNT[base + e] = st[ix(e)];
        }
        carry += total;
        __syncthreads();
    }
}

__global__ __launch_bounds__(256) void k_v1x_scatter(Geometry g, V1xBig b) {
    V1X_SLOT_PROLOGUE
    const int k = (int)(xblk * 256 + threadIdx.x);
    if (k >= 1 && k < n) b.LST[(size_t)slot * b.B + atomicAdd(&CNT[J[k]], 1u)] = (uint32_t)k;
}

// smallest k > above in bucket p (bucket p = LST[p ? CNT[p-1] : 0, CNT[p])), or -1
__device__ __forceinline__ int v1x_succ(const uint32_t *CNT, const uint32_t *LST, int p, int above) {
    const int b0 = p ? (int)CNT[p - 1] : 0, b1 = (int)CNT[p];
    int best = -1;
    for (int x = b0; x < b1; x++) {
        const int k = (int)LST[x];
        if (k > above && (best < 0 || k < best)) best = k;
    }
    return best;
}

__global__ __launch_bounds__(256) void k_v1x_parent(Geometry g, V1xBig b) {
    V1X_SLOT_PROLOGUE
    const int k = (int)(xblk * 256 + threadIdx.x);
    if (k >= n) return;
    const int pk = v1x_succ(CNT, b.LST + (size_t)slot * b.B, k, k);
    b.NXT[(size_t)slot * b.B + k] = (uint32_t)(pk < 0 ? k : pk);
}

__global__ __launch_bounds__(256) void k_v1x_out(Geometry g, V1xBig b, const RankDesc *__restrict__ ranks,
                                                 int32_t rank_lo, int64_t pos_lo, int64_t count,
                                                 int64_t *__restrict__ out, MapArgs ma) {
    V1X_SLOT_PROLOGUE
    const int64_t wb = w * g.B;
    const int64_t p = wb + (int64_t)(xblk * 256 + threadIdx.x);
    const int i = (int)(p - wb);
    if (i >= n || p < pos_lo || p >= pos_lo + count) return;
    const uint32_t *LST = b.LST + (size_t)slot * b.B, *NXT = b.NXT + (size_t)slot * b.B;
    auto root = [&](int k) {
        for (;;) {
            const int nk = (int)NXT[k];
            if (nk == k) return k;
            k = nk;
        }
    };
    int x;
    if (n <= 1) {
        x = 0;
    } else if (i == 0) {
        const int k = v1x_succ(CNT, LST, 0, 0);
        x = k < 0 ? 0 : root(k);
    } else {
        const int pj = (int)J[i];
        if (pj == i) {
            x = root(i);
        } else {
            const int k = v1x_succ(CNT, LST, pj, i);
            x = k < 0 ? pj : root(k);
        }
    }
    const int32_t rl = (int32_t)(job / (uint64_t)b.nw);
    put_id_or_pair(out, ma, (int64_t)rl * count + (p - pos_lo), wrap_id(ranks[rank_lo + rl].new_start + wb + x, g.N));
}

namespace {
// entries per pass of the HBM path (16 B each: a pass's workspace is <= 2 GB while windows have
// at most 2^27 entries; a longer window is one job of ~16 B per entry, up to ~32 GB near 2^31 --
// pss.h states the cost, and a workspace the device cannot hold fails pss_generate with PSS_EHIP)
constexpr int64_t kV1xPassEntries = (int64_t)1 << 27;
int64_t v1x_jobs_per_pass(int64_t B) {
    const int64_t j = kV1xPassEntries / B;
    return j < 1 ? 1 : (j > 65535 ? 65535 : j);
}
}  // namespace

size_t v1_exact_lds_bytes(int64_t n) {
    return (size_t)(kMtN + n + 1) * sizeof(uint32_t) + (size_t)3 * n * sizeof(uint16_t) + 16;
}

bool v1_exact_supported(const Geometry &g) { return g.B < ((int64_t)1 << 31); }

size_t v1_exact_ws_bytes(const Geometry &g, int32_t nr, int64_t pos_lo, int64_t count) {
    const int64_t pos_hi = pos_lo + count < g.ns ? pos_lo + count : g.ns;
    if (nr <= 0 || pos_hi <= pos_lo || !v1_exact_supported(g)) return 0;
    const int64_t nw = (pos_hi - 1) / g.B - pos_lo / g.B + 1;
    const int64_t jobs = (int64_t)nr * nw;
    const int64_t W = g.B < g.ns ? g.B : g.ns;   // the longest window
    if (W <= kV1ExactMaxB) return (size_t)jobs * (size_t)W * sizeof(uint16_t);
    const int64_t pj = jobs < v1x_jobs_per_pass(W) ? jobs : v1x_jobs_per_pass(W);
    return (size_t)pj * ((size_t)4 * W + 1) * sizeof(uint32_t);
}

static hipError_t launch_v1_exact_big(const Geometry &g, const RankDesc *ranks, int32_t rank_lo, int32_t nr,
                                      int64_t pos_lo, int64_t count, int64_t epoch, int64_t *out,
                                      uint32_t *ws, hipStream_t s, const MapArgs &ma) {
    const int64_t pos_hi = pos_lo + count < g.ns ? pos_lo + count : g.ns;
    const int64_t w_lo = pos_lo / g.B, w_hi = (pos_hi - 1) / g.B;
    const int64_t nw = w_hi - w_lo + 1;
    const uint64_t jobs = (uint64_t)nr * (uint64_t)nw;
    const int64_t W = g.B < g.ns ? g.B : g.ns;   // the longest window: the slice length
    const uint64_t per = (uint64_t)v1x_jobs_per_pass(W);
    const uint32_t B = (uint32_t)W;
    for (uint64_t j0 = 0; j0 < jobs; j0 += per) {
        V1xBig b{};
        b.w_lo = w_lo; b.nw = nw; b.j0 = j0; b.B = B;
        b.nj = (uint32_t)(jobs - j0 < per ? jobs - j0 : per);
        b.J = ws;
        b.CNT = b.J + (size_t)b.nj * B;
        b.LST = b.CNT + (size_t)b.nj * ((size_t)B + 1);
        b.NXT = b.LST + (size_t)b.nj * B;
        hipError_t e = hipMemsetAsync(b.CNT, 0, sizeof(uint32_t) * (size_t)b.nj * ((size_t)B + 1), s);
        if (e != hipSuccess) return e;
        b.xb = (B + 255) / 256;
        // XCD-major only while the 1-D grid stays below 2^32 threads (round 3: the scatter's
        // random LST writes 8.2 -> 5.2 ms at C5 against the (x, slot) grid)
        b.xcd = (uint64_t)b.xb * (((uint64_t)b.nj + 7) / 8) * 8 < ((uint64_t)1 << 24) ? 1u : 0u;
        const dim3 flat = b.xcd ? dim3((uint32_t)((uint64_t)b.xb * (((uint64_t)b.nj + 7) / 8) * 8))
                                : dim3(b.xb, b.nj);
        // few windows: a workgroup per window's MT stream (PSS_V1X_DRAWS_WG=0 / 1 forces a form)
        static const int wg_env = [] {
            const char *e = getenv("PSS_V1X_DRAWS_WG");
            return e ? atoi(e) : -1;
        }();
        const bool wg = wg_env == 0 || wg_env == 1 ? wg_env == 1 : b.nj < 1024;
        if (wg) hipLaunchKernelGGL(k_v1x_draws32_wg, dim3(b.nj), dim3(kMtWgThreads), 0, s, g, b, epoch);
        else hipLaunchKernelGGL(k_v1x_draws32, dim3(b.nj), dim3(64), 0, s, g, b, epoch);
        hipLaunchKernelGGL(k_v1x_scan, dim3(b.nj), dim3(kV1xScanNT), 0, s, g, b);
        hipLaunchKernelGGL(k_v1x_scatter, flat, dim3(256), 0, s, g, b);
        hipLaunchKernelGGL(k_v1x_parent, flat, dim3(256), 0, s, g, b);
        hipLaunchKernelGGL(k_v1x_out, flat, dim3(256), 0, s, g, b, ranks, rank_lo, pos_lo, count, out, ma);
        e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t launch_v1_exact(const Geometry &g, const RankDesc *ranks, int32_t rank_lo, int32_t nr,
                           int64_t pos_lo, int64_t count, int64_t epoch, int64_t *out, void *ws,
                           hipStream_t s, const MapArgs *mapped) {
    const MapArgs ma = mapped ? *mapped : MapArgs{};
    const int64_t pos_hi = pos_lo + count < g.ns ? pos_lo + count : g.ns;
    if (nr <= 0 || pos_hi <= pos_lo) return hipSuccess;
    if (!v1_exact_supported(g)) return hipErrorInvalidValue;
    if ((g.B < g.ns ? g.B : g.ns) > kV1ExactMaxB) {
        if (!ws) return hipErrorInvalidValue;
        return launch_v1_exact_big(g, ranks, rank_lo, nr, pos_lo, count, epoch, out, (uint32_t *)ws, s, ma);
    }
    const int64_t w_lo = pos_lo / g.B, w_hi = (pos_hi - 1) / g.B;
    const int64_t nw = w_hi - w_lo + 1;
    const size_t lds = v1_exact_lds_bytes(g.B < g.ns ? g.B : g.ns);
    static const hipError_t attr = hipFuncSetAttribute(
        (const void *)k_v1_exact, hipFuncAttributeMaxDynamicSharedMemorySize,
        (int)v1_exact_lds_bytes(kV1ExactMaxB));
    if (attr != hipSuccess) return attr;
    const dim3 grid((uint32_t)(nr * nw));
    // with a workspace, the serial MT phases run one wave per window (many windows in flight)
    // ahead of the resolution; without one, each workgroup's first wave does them in place
    if (ws) hipLaunchKernelGGL(k_v1x_draws, grid, dim3(64), 0, s, g, w_lo, nw, epoch, (uint16_t *)ws);
    hipLaunchKernelGGL(k_v1_exact, grid, dim3(kExactNT), lds, s, g, ranks, rank_lo, w_lo, nw, pos_lo,
                       count, epoch, (const uint16_t *)ws, out, ma);
    return hipGetLastError();
}

}  // namespace pss
