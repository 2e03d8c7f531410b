// pss_v1exact.hip -- V1 window permutations in the reference's EXACT order (order mode
// PSS_ORDER_EXACT): window 0 is `seed(epoch); shuffle(range(len))` (V1:102,114-115), window
// b >= 1 is `seed(epoch + b*10000); shuffle(range(len))` (V1:165-171), both with CPython
// 3.10's MT19937 (`random.py:128-168` seeding, `:239-249` _randbelow, `:380-396` shuffle).
// Every window reseeds, so windows are independent: one 256-thread workgroup per
// (rank, window), three phases.
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
    uint16_t *jw = J + (size_t)blockIdx.x * (size_t)g.B;
    mt_seed_int(mt, w == 0 ? epoch : epoch + w * 10000);
    mt_draws(mt, (uint32_t)(n - 1), [&](uint32_t d) { return (uint32_t)n - d; },
             [&](uint32_t d, uint32_t r) { jw[n - 1 - (int)d] = (uint16_t)r; });
}

// One workgroup per (local rank, window) of [w_lo, w_lo + nw).
__global__ __launch_bounds__(kExactNT) void k_v1_exact(Geometry g, const RankDesc *__restrict__ ranks,
                                                       int32_t rank_lo, int64_t w_lo, int64_t nw,
                                                       int64_t pos_lo, int64_t count, int64_t epoch,
                                                       const uint16_t *__restrict__ J,
                                                       int64_t *__restrict__ out) {
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
        const uint16_t *jw = J + (size_t)blockIdx.x * (size_t)g.B;
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
    int64_t *o = out + (int64_t)rl * count - pos_lo;
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
        o[wb + p] = wrap_id(base + x, g.N);
    }
}

size_t v1_exact_lds_bytes(int64_t n) {
    return (size_t)(kMtN + n + 1) * sizeof(uint32_t) + (size_t)3 * n * sizeof(uint16_t) + 16;
}

bool v1_exact_supported(const Geometry &g) { return g.B <= kV1ExactMaxB; }

size_t v1_exact_ws_bytes(const Geometry &g, int32_t nr, int64_t pos_lo, int64_t count) {
    const int64_t pos_hi = pos_lo + count < g.ns ? pos_lo + count : g.ns;
    if (nr <= 0 || pos_hi <= pos_lo || !v1_exact_supported(g)) return 0;
    const int64_t nw = (pos_hi - 1) / g.B - pos_lo / g.B + 1;
    return (size_t)nr * (size_t)nw * (size_t)g.B * sizeof(uint16_t);
}

hipError_t launch_v1_exact(const Geometry &g, const RankDesc *ranks, int32_t rank_lo, int32_t nr,
                           int64_t pos_lo, int64_t count, int64_t epoch, int64_t *out, uint16_t *ws,
                           hipStream_t s) {
    const int64_t pos_hi = pos_lo + count < g.ns ? pos_lo + count : g.ns;
    if (nr <= 0 || pos_hi <= pos_lo) return hipSuccess;
    if (!v1_exact_supported(g)) return hipErrorInvalidValue;
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
    if (ws) hipLaunchKernelGGL(k_v1x_draws, grid, dim3(64), 0, s, g, w_lo, nw, epoch, ws);
    hipLaunchKernelGGL(k_v1_exact, grid, dim3(kExactNT), lds, s, g, ranks, rank_lo, w_lo, nw, pos_lo,
                       count, epoch, (const uint16_t *)ws, out);
    return hipGetLastError();
}

}  // namespace pss
