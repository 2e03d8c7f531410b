// pss_v1exact.hip -- V1 window permutations in the reference's EXACT order (order mode
// PSS_ORDER_EXACT): window 0 is `seed(epoch); shuffle(range(len))` (V1:102,114-115), window
// b >= 1 is `seed(epoch + b*10000); shuffle(range(len))` (V1:165-171), both with CPython
// 3.10's MT19937 (`random.py:128-168` seeding, `:239-249` _randbelow, `:380-396` shuffle).
// Every window reseeds, so windows are independent -- and the same for every rank: the seed is
// the epoch and the window index, the shuffled list range(len) (V1:165-171), and every rank has
// num_samples positions.  A window's permutation is resolved once per call; its output stage
// writes id = new_start + w B + x for each rank of the call (kV1FanRanks per workgroup row).
// One 256-thread workgroup per window, three phases, for windows up to kV1ExactMaxB entries
// (LDS-resident); larger windows run the same three phases through HBM (k_v1x_*, below).
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
//      Bucket the steps by j (count, scan, scatter), take parents from the buckets, climb to
//      the roots (in place, one pass), and read each x[i] off its bucket.  tests/test_gpu_parity.py checks
//      the streams against oracle/pss_oracle.c's exact V1 (CPython restatement, pinned by the
//      reference's golden streams).
#include <cstdlib>

#include "pss_mt.h"

namespace pss {

namespace {
constexpr int kExactNT = 256;
constexpr int32_t kV1FanRanks = 8;   // ranks whose ids one workgroup writes
}  // namespace

// Phases 1-2 alone, one wave per window (2.5 KB of LDS, so a CU holds 32 of them): the draws
// j_i of every window go to HBM (u16, B per window) for k_v1_exact's resolution.  Grid: nw.
// The windows' MT states come seeded by k_mt_seed_streams (ST: [window slot][624]).
__global__ __launch_bounds__(64) void k_v1x_draws(Geometry g, int64_t w_lo, int64_t nw, int64_t epoch,
                                                  const uint32_t *__restrict__ ST, uint16_t *__restrict__ J) {
    __shared__ uint32_t mt[kMtN];
    const int64_t w = w_lo + (int64_t)(blockIdx.x % nw);
    const int64_t wb = w * g.B;
    const int n = (int)(g.ns - wb < g.B ? g.ns - wb : g.B);
    if (n <= 1) return;
    uint16_t *jw = J + (size_t)blockIdx.x * (size_t)(g.B < g.ns ? g.B : g.ns);
    mt_load(mt, ST + (size_t)blockIdx.x * kMtN);
    mt_draws(mt, (uint32_t)(n - 1), [&](uint32_t d) { return (uint32_t)n - d; },
             [&](uint32_t d, uint32_t r) { jw[n - 1 - (int)d] = (uint16_t)r; });
}

// One workgroup per (rank group, window) of [w_lo, w_lo + nw): the window's permutation, then
// the ids of ranks [group * kV1FanRanks, ...) of the call (nout ranks from rank_lo).  (Writing
// the window offsets once for a one-shot fan-out grid instead, as the exact V2 does, measured
// slower at C2: 0.42 -> 0.48 ms -- the resolution, not the stores, sets this kernel's time.)
__global__ __launch_bounds__(kExactNT) void k_v1_exact(Geometry g, const RankDesc *__restrict__ ranks,
                                                       int32_t rank_lo, int32_t nout, int64_t w_lo, int64_t nw,
                                                       int64_t pos_lo, int64_t count, int64_t epoch,
                                                       const uint16_t *__restrict__ J,
                                                       int64_t *__restrict__ out, MapArgs ma) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    const int32_t r_a = (int32_t)(blockIdx.x / nw) * kV1FanRanks;
    const int32_t r_b = r_a + kV1FanRanks < nout ? r_a + kV1FanRanks : nout;
    const uint32_t wslot = (uint32_t)(blockIdx.x % nw);
    const int64_t w = w_lo + (int64_t)wslot;
    const int64_t wb = w * g.B;
    const int n = (int)(g.ns - wb < g.B ? g.ns - wb : g.B);
    const int tid = threadIdx.x, wid = tid >> 6;
    // LDS (v1_exact_lds_bytes): [624] MT state only when this block draws itself, then 10 B per
    // entry -- 40 KB at n = 4096, four workgroups per CU
    uint32_t *mt = smem;                                   // [624] (no J)
    uint32_t *cnt = J ? smem : smem + kMtN;                // [n] bucket counts -> ends
    uint16_t *jv = (uint16_t *)(cnt + n);                  // [n] j_i
    uint16_t *lst = jv + n;                                // [n] steps bucketed by j
    uint16_t *nxt = lst + n;                               // [n] parent -> root
    // the block scan's wave totals in nxt, unused until after the scan (n >= 8; tiny windows:
    // the 16 bytes after the arrays)
    uint32_t *tot = n >= 8 ? (uint32_t *)nxt : (uint32_t *)(((uintptr_t)(nxt + n) + 3u) & ~(uintptr_t)3u);

    if (J) {                 // draws already made by k_v1x_draws
        const uint16_t *jw = J + (size_t)wslot * (size_t)(g.B < g.ns ? g.B : g.ns);
        for (int i = tid; i < n; i += kExactNT) jv[i] = jw[i];
    } else if (wid == 0 && n > 1) {
        // ---- 1. seed(a): key = 32-bit words of abs(a) (random_seed) ----
        mt_seed_int(mt, w == 0 ? epoch : epoch + w * 10000);
        // ---- 2. the draws of shuffle(range(n)): draw d is j_i = _randbelow(i + 1), i = n-1-d
        mt_draws(mt, (uint32_t)(n - 1), [&](uint32_t d) { return (uint32_t)n - d; },
                 [&](uint32_t d, uint32_t r) { jv[n - 1 - (int)d] = (uint16_t)r; });
    }
    // ---- 3. resolve the swap sequence (all threads) ----
    for (int p = tid; p < n; p += kExactNT) cnt[p] = 0;
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
    // the chain roots: each thread climbs from its k (the chains are short -- they climb
    // geometrically, ~1-2 steps -- where log2(n) rounds of pointer jumping with a barrier each took
    // 54 of this kernel's ~180 us at C2) and writes the root in place.  Threads race on nxt, but
    // every value written is an ancestor of its entry and a root is never changed, so a climb that
    // reads an already compressed entry only gets there sooner.
    {
        volatile uint16_t *vn = nxt;
        for (int k = tid; k < n; k += kExactNT) {
            int r = vn[k];
            for (int q = vn[r]; q != r; q = vn[r]) r = q;
            vn[k] = (uint16_t)r;
        }
    }
    __syncthreads();
    // ---- output: x[i] for the positions of this window inside [pos_lo, pos_lo + count) ----
    int64_t p0 = 0, p1 = n;
    if (wb < pos_lo) p0 = pos_lo - wb;
    if (wb + n > pos_lo + count) p1 = pos_lo + count - wb;
    auto x_of = [&](int i) -> int {
        if (n <= 1) return 0;
        if (i == 0) {
            const int k = succ(0, 0);
            return k < 0 ? 0 : nxt[k];
        }
        const int pj = jv[i];
        if (pj == i) return nxt[i];
        const int k = succ(pj, i);
        return k < 0 ? pj : nxt[k];
    };
    // two consecutive positions per thread, one 16-byte store per rank where the rows allow it
    // (an even first element and a 16-byte aligned output), else one id at a time
    const int64_t e0 = -pos_lo + wb + p0;   // element of position p0 in rank row 0
    const bool pairs = !ma.fpos && ((count | e0) & 1) == 0 && (((uintptr_t)out) & 15u) == 0;
    if (pairs) {
        for (int64_t p = p0 + 2 * tid; p < p1; p += 2 * kExactNT) {
            const int x0 = x_of((int)p);
            const bool two = p + 1 < p1;
            const int x1 = two ? x_of((int)p + 1) : 0;
            for (int32_t r = r_a; r < r_b; r++) {   // (wave-uniform rank: scalar descriptor loads)
                const int64_t ns0 = ranks[rank_lo + r].new_start + wb;
                int64_t *o = out + (int64_t)r * count - pos_lo + wb + p;
                if (two) *(longlong2 *)o = make_longlong2(wrap_id(ns0 + x0, g.N), wrap_id(ns0 + x1, g.N));
                else o[0] = wrap_id(ns0 + x0, g.N);
            }
        }
        return;
    }
    for (int64_t p = p0 + tid; p < p1; p += kExactNT) {
        const int x = x_of((int)p);
        for (int32_t r = r_a; r < r_b; r++)   // (wave-uniform rank: scalar descriptor loads)
            put_id_or_pair(out, ma, (int64_t)r * count - pos_lo + wb + p, wrap_id(ranks[rank_lo + r].new_start + wb + x, g.N));
    }
}

// ---- windows beyond LDS (n > kV1ExactMaxB): the same resolution through HBM ----------------
// One pass covers `nj` jobs (windows) of the launch, jobs j0 .. j0 + nj - 1 (job -> window
// w_lo + job % nw: every rank of the call shares it), each with slices of the window length W:
//   J      the draws j_k, k = 1 .. n-1 (k_v1x_draws32[_wg]: the MT stream is serial); each draw
//          also counts its bucket, j >> 11, in BCNT (nbk = ceil(W / 2048) counters per window)
//   PART   the steps k partitioned by bucket (k_v1x_part: counts -> offsets by k_v1x_bscan, then
//          per 8192-step chunk a local LDS sort and one coalesced run per bucket), PARTP their
//          j & 2047
//   S, H   per bucket in LDS (k_v1x_solve): the lists {k : j_k = p} of its 2048 values p,
//          sorted; S[k] = the next element of k's list (none: ~0), H[p] = the first element of
//          list p above p -- with x[0]'s list 0 taking 0 as its smallest element
// and the output x[i] = S[i] ? root(S[i]) : j_i (x[0]: 0), root(k) = H[k] ? root(H[k]) : k
// (k_v1x_out; the chains climb geometrically towards n, ~1-2 steps on average).  The resolution
// of round 3 bucketed the steps by j with one random HBM atomic and one random store per step
// (5.2 ms at C5) and read every answer back through them (3.3 ms).
constexpr uint32_t kV1bShift = 11, kV1bBW = 1u << kV1bShift;   // bucket width in values of j
constexpr uint32_t kV1bNone = 0xFFFFFFFFu;
struct V1xBig {
    int64_t w_lo, nw;       // windows of the launch
    uint64_t j0;            // first job of the pass
    uint32_t nj;            // jobs in the pass
    uint32_t B;             // slice length W: min(shuffle_buffer, num_samples)
    uint32_t nbk;           // buckets per window: ceil(W / 2048)
    uint32_t *J, *S, *H, *PART, *BCNT;   // BCNT: nbk counts -> offsets -> bucket ends per window
    uint16_t *PARTP;
    uint32_t xb;            // the flat kernel's x extent (blocks per window)
    uint32_t xcd;           // 1: XCD-major flat grid (v1x_block)
};

// The flat kernels make random accesses inside one window's slices.  XCD-major grid: workgroup
// L runs on XCD L mod 8 (round-robin dispatch), so block L is given window slot 8 (L / 8 / xb) +
// L mod 8 and block (L / 8) mod xb -- every window's blocks then run on one XCD, one window after
// another, which keeps its slices' lines in that XCD's L2.  xcd = 0: blockIdx.y = slot.
__device__ __forceinline__ bool v1x_block(const V1xBig &b, uint32_t &slot, uint32_t &xblk) {
    if (!b.xcd) { slot = blockIdx.y; xblk = blockIdx.x; return true; }
    const uint32_t L = blockIdx.x, q = L >> 3;
    slot = 8u * (q / b.xb) + (L & 7u);
    xblk = q % b.xb;
    return slot < b.nj;
}

__host__ __device__ __forceinline__ int v1x_len(const Geometry &g, int64_t w) {
    const int64_t wb = w * g.B;
    return (int)(g.ns - wb < g.B ? g.ns - wb : g.B);
}

// Each draw also counts its bucket (a fire-and-forget atomic on a small, L2-resident table beside
// the latency-bound draws)
__global__ __launch_bounds__(64) void k_v1x_draws32(Geometry g, V1xBig b, int64_t epoch) {
    __shared__ uint32_t mt[kMtN];
    const uint64_t job = b.j0 + blockIdx.x;
    const int64_t w = b.w_lo + (int64_t)(job % (uint64_t)b.nw);
    const int n = v1x_len(g, w);
    if (n <= 1) return;
    uint32_t *jw = b.J + (size_t)blockIdx.x * b.B;
    uint32_t *cnt = b.BCNT + (size_t)blockIdx.x * b.nbk;
    mt_seed_int(mt, w == 0 ? epoch : epoch + w * 10000);
    mt_draws(mt, (uint32_t)(n - 1), [&](uint32_t d) { return (uint32_t)n - d; },
             [&](uint32_t d, uint32_t r) {
                 jw[n - 1 - (int)d] = r;
                 atomicAdd(&cnt[r >> kV1bShift], 1u);
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
    uint32_t *cnt = b.BCNT + (size_t)blockIdx.x * b.nbk;
    if (threadIdx.x < 64) mt_seed_int(sh.mt[0], w == 0 ? epoch : epoch + w * 10000);
    __syncthreads();
    mt_draws_wg(sh, 0, (uint32_t)(n - 1), [&](uint32_t d) { return (uint32_t)n - d; },
                [&](uint32_t d, uint32_t r) {
                    jw[n - 1 - (int)d] = r;
                    atomicAdd(&cnt[r >> kV1bShift], 1u);
                });
}

// exclusive scan of a window's nbk bucket counts in place, one workgroup per window, in tiles of
// kV1xScanNT x 8 counts: coalesced loads into LDS (skewed one word per 32), each thread scans 8
// consecutive counts, one block scan, coalesced stores
constexpr int kV1xScanNT = 1024, kV1xScanPer = 8, kV1xScanTile = kV1xScanNT * kV1xScanPer;
__global__ __launch_bounds__(kV1xScanNT) void k_v1x_bscan(Geometry g, V1xBig b) {
    const uint32_t slot = blockIdx.x;
    const int n = (int)b.nbk;
    uint32_t *CNT = b.BCNT + (size_t)slot * b.nbk;
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

// ---- partition: steps k -> PART by bucket j_k >> 11 ------------------------------------------
// A workgroup per 4096-step chunk of a window: the chunk's steps are counted and ranked per
// bucket in LDS, every bucket present reserves its run of the window's bucket region with one
// global atomic on BCNT (offsets -> ends), the chunk is sorted by bucket in LDS and written as
// those runs (C5: ~8 consecutive steps per bucket and chunk).  Windows of more than
// kV1pLocal buckets (W > 4M) take one global atomic per step instead.
constexpr int kV1pNT = 256, kV1pPer = 16, kV1pChunk = kV1pNT * kV1pPer, kV1pLocal = 2048;
__global__ __launch_bounds__(kV1pNT) void k_v1x_part(Geometry g, V1xBig b) {
    uint32_t slot, xblk;
    if (!v1x_block(b, slot, xblk)) return;
    const uint64_t job = b.j0 + slot;
    const int64_t w = b.w_lo + (int64_t)(job % (uint64_t)b.nw);
    const int n = v1x_len(g, w);
    const uint32_t *J = b.J + (size_t)slot * b.B;
    uint32_t *BC = b.BCNT + (size_t)slot * b.nbk;
    uint32_t *PART = b.PART + (size_t)slot * b.B;
    uint16_t *PARTP = b.PARTP + (size_t)slot * b.B;
    const int k0 = (int)xblk * kV1pChunk, tid = (int)threadIdx.x;
    if (k0 >= n) return;
    const int k1 = k0 + kV1pChunk < n ? k0 + kV1pChunk : n;
    if (b.nbk > (uint32_t)kV1pLocal) {
        for (int k = k0 + tid; k < k1; k += kV1pNT) {
            if (k < 1) continue;
            const uint32_t v = J[k];
            const uint32_t pos = atomicAdd(&BC[v >> kV1bShift], 1u);
            PART[pos] = (uint32_t)k;
            PARTP[pos] = (uint16_t)(v & (kV1bBW - 1u));
        }
        return;
    }
    __shared__ uint32_t hist[kV1pLocal], loff[kV1pLocal], gbase[kV1pLocal];
    __shared__ uint32_t stk[kV1pChunk];
    __shared__ uint16_t stp[kV1pChunk], stb[kV1pChunk];
    __shared__ uint32_t tot[kV1pNT / 64];
    const int nb = (int)b.nbk;
    for (int i = tid; i < nb; i += kV1pNT) hist[i] = 0u;
    __syncthreads();
    uint32_t val[kV1pPer], rk[kV1pPer];
#pragma unroll
    for (int i = 0; i < kV1pPer; i++) {
        const int k = k0 + tid + kV1pNT * i;
        val[i] = (k >= 1 && k < k1) ? J[k] : kV1bNone;
    }
#pragma unroll
    for (int i = 0; i < kV1pPer; i++)
        rk[i] = val[i] != kV1bNone ? atomicAdd(&hist[val[i] >> kV1bShift], 1u) : 0u;
    __syncthreads();
    {   // exclusive scan of hist -> loff (nb <= 2048: 8 per thread), and each bucket's reservation
        constexpr int per = kV1pLocal / kV1pNT;
        uint32_t c[per], sum = 0;
#pragma unroll
        for (int i = 0; i < per; i++) {
            const int bb = tid * per + i;
            c[i] = bb < nb ? hist[bb] : 0u;
            sum += c[i];
        }
        uint32_t total;
        uint32_t run = block_excl_scan<kV1pNT>(sum, tot, total);
#pragma unroll
        for (int i = 0; i < per; i++) {
            const int bb = tid * per + i;
            if (bb < nb) {
                loff[bb] = run;
                if (c[i]) gbase[bb] = atomicAdd(&BC[bb], c[i]);
            }
            run += c[i];
        }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kV1pPer; i++) {
        if (val[i] == kV1bNone) continue;
        const uint32_t bb = val[i] >> kV1bShift, pos = loff[bb] + rk[i];
        stk[pos] = (uint32_t)(k0 + tid + kV1pNT * i);
        stp[pos] = (uint16_t)(val[i] & (kV1bBW - 1u));
        stb[pos] = (uint16_t)bb;
    }
    __syncthreads();
    const int m = k1 - (k0 < 1 ? 1 : k0);
    for (int e = tid; e < m; e += kV1pNT) {
        const uint32_t bb = stb[e];
        const uint32_t pos = gbase[bb] + ((uint32_t)e - loff[bb]);
        PART[pos] = stk[e];
        PARTP[pos] = stp[e];
    }
}

// ---- solve: per bucket, its lists sorted in LDS -> S (successors) and H (first above p) ------
// A workgroup per (window, bucket of 2048 values p): counts its steps per p in LDS, scans them,
// places the steps list by list in LDS (as many p at a time as kV1sCap entries hold: the first
// buckets of long windows hold up to ~2048 (ln(W / 2048) + 1) steps), sorts each list (a thread
// per p; lists are short, ~ln(n / p)) and writes H[p] and the successors S[k].
constexpr int kV1sNT = 256, kV1sCap = 8192;
__global__ __launch_bounds__(kV1sNT) void k_v1x_solve(Geometry g, V1xBig b) {
    uint32_t slot, bk;
    if (!v1x_block(b, slot, bk)) return;
    const uint64_t job = b.j0 + slot;
    const int64_t w = b.w_lo + (int64_t)(job % (uint64_t)b.nw);
    const int n = v1x_len(g, w);
    const uint32_t pbase = bk << kV1bShift;
    if ((int64_t)pbase >= (int64_t)n) return;
    const int plen = n - (int)pbase < (int)kV1bBW ? n - (int)pbase : (int)kV1bBW;
    const uint32_t *BC = b.BCNT + (size_t)slot * b.nbk;
    const uint32_t e0 = bk ? BC[bk - 1] : 0u, e1 = BC[bk];   // (after k_v1x_part: bucket ends)
    const uint32_t *PART = b.PART + (size_t)slot * b.B;
    const uint16_t *PARTP = b.PARTP + (size_t)slot * b.B;
    uint32_t *S = b.S + (size_t)slot * b.B, *H = b.H + (size_t)slot * b.B;
    __shared__ uint32_t off[kV1bBW + 1], cur[kV1bBW], L[kV1sCap];
    __shared__ uint32_t tot[kV1sNT / 64];
    __shared__ int bounds[2];
    const int tid = (int)threadIdx.x;
    for (int p = tid; p <= plen; p += kV1sNT) off[p] = 0u;
    __syncthreads();
    for (uint32_t e = e0 + tid; e < e1; e += kV1sNT) atomicAdd(&off[PARTP[e]], 1u);
    __syncthreads();
    {   // exclusive scan of off[0, plen), 8 per thread; off[plen] = the bucket's steps
        constexpr int per = (int)kV1bBW / kV1sNT;
        uint32_t c[per], sum = 0;
#pragma unroll
        for (int i = 0; i < per; i++) {
            const int p = tid * per + i;
            c[i] = p < plen ? off[p] : 0u;
            sum += c[i];
        }
        uint32_t total;
        uint32_t run = block_excl_scan<kV1sNT>(sum, tot, total);
        __syncthreads();
#pragma unroll
        for (int i = 0; i < per; i++) {
            const int p = tid * per + i;
            if (p < plen) off[p] = run;
            run += c[i];
        }
        if (tid == 0) off[plen] = total;
    }
    __syncthreads();
    int plo = 0;
    while (plo < plen) {
        if (tid == 0) {   // the longest run of lists from plo that fits kV1sCap entries
            int lo = plo + 1, hi = plen;
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (off[mid] - off[plo] <= (uint32_t)kV1sCap) lo = mid; else hi = mid - 1;
            }
            bounds[0] = lo;
        }
        __syncthreads();
        const int phi = bounds[0];
        const uint32_t ob = off[plo];
        for (int p = plo + tid; p < phi; p += kV1sNT) cur[p] = off[p] - ob;
        __syncthreads();
        for (uint32_t e = e0 + tid; e < e1; e += kV1sNT) {
            const int p = (int)PARTP[e];
            if (p >= plo && p < phi) {
                const uint32_t pos = atomicAdd(&cur[p], 1u);
                if (pos < (uint32_t)kV1sCap) L[pos] = PART[e];   // (one list of > kV1sCap steps: never)
            }
        }
        __syncthreads();
        for (int p = plo + tid; p < phi; p += kV1sNT) {
            const int s0 = (int)(off[p] - ob), s1 = (int)(off[p + 1] - ob);
            for (int a = s0 + 1; a < s1; a++) {   // insertion sort of the list (short)
                const uint32_t v = L[a];
                int c = a - 1;
                while (c >= s0 && L[c] > v) { L[c + 1] = L[c]; c--; }
                L[c + 1] = v;
            }
            const uint32_t pa = pbase + (uint32_t)p;
            uint32_t first = kV1bNone;
            for (int a = s0; a < s1; a++) {
                const uint32_t k = L[a];
                if (first == kV1bNone && k > pa) first = k;
                S[k] = a + 1 < s1 ? L[a + 1] : kV1bNone;
            }
            H[pa] = first;
            if (pa == 0u) S[0] = first;   // step 0 heads list 0 (x[0] = its successor's root)
        }
        __syncthreads();
        plo = phi;
    }
}

// ---- output: x[i] = S[i] ? root(S[i]) : j_i (x[0]: 0) -----------------------------------------
// (the window's x[i] once, then the ids of the call's nout ranks from rank_lo)
__global__ __launch_bounds__(256) void k_v1x_out(Geometry g, V1xBig b, const RankDesc *__restrict__ ranks,
                                                 int32_t rank_lo, int32_t nout, int64_t pos_lo, int64_t count,
                                                 int64_t *__restrict__ out, MapArgs ma) {
    uint32_t slot, xblk;
    if (!v1x_block(b, slot, xblk)) return;
    const uint64_t job = b.j0 + slot;
    const int64_t w = b.w_lo + (int64_t)(job % (uint64_t)b.nw);
    const int n = v1x_len(g, w);
    const int64_t wb = w * g.B;
    const int64_t p = wb + (int64_t)(xblk * 256 + threadIdx.x);
    const int i = (int)(p - wb);
    if (i >= n || p < pos_lo || p >= pos_lo + count) return;
    const uint32_t *J = b.J + (size_t)slot * b.B;
    const uint32_t *S = b.S + (size_t)slot * b.B, *H = b.H + (size_t)slot * b.B;
    uint32_t x;
    if (n <= 1) {
        x = 0u;
    } else {
        uint32_t k = S[i];
        if (k == kV1bNone) {
            x = i == 0 ? 0u : J[i];
        } else {
            for (;;) {
                const uint32_t h = H[k];
                if (h == kV1bNone) break;
                k = h;
            }
            x = k;
        }
    }
    for (int32_t r = 0; r < nout; r++)   // (wave-uniform rank: scalar descriptor loads)
        put_id_or_pair(out, ma, (int64_t)r * count + (p - pos_lo), wrap_id(ranks[rank_lo + r].new_start + wb + x, g.N));
}

// The same for two consecutive positions per thread: both climbs in flight together and one
// 16-byte store per rank (ids only; the launcher checks the rows' alignment)
__global__ __launch_bounds__(256) void k_v1x_out2(Geometry g, V1xBig b, const RankDesc *__restrict__ ranks,
                                                  int32_t rank_lo, int32_t nout, int64_t pos_lo, int64_t count,
                                                  int64_t *__restrict__ out) {
    uint32_t slot, xblk;
    if (!v1x_block(b, slot, xblk)) return;
    const uint64_t job = b.j0 + slot;
    const int64_t w = b.w_lo + (int64_t)(job % (uint64_t)b.nw);
    const int n = v1x_len(g, w);
    const int64_t wb = w * g.B;
    const int i0 = (int)(xblk * 512u + 2u * threadIdx.x);
    const int64_t p = wb + i0;
    const int64_t pos_hi = pos_lo + count;
    if (i0 >= n || p + 1 < pos_lo || p >= pos_hi) return;
    const uint32_t *J = b.J + (size_t)slot * b.B;
    const uint32_t *S = b.S + (size_t)slot * b.B, *H = b.H + (size_t)slot * b.B;
    const bool has1 = i0 + 1 < n;
    uint32_t x[2] = {0u, 0u};
    if (n > 1) {
        uint32_t k[2], j[2];
        k[0] = S[i0]; j[0] = J[i0];
        k[1] = has1 ? S[i0 + 1] : kV1bNone; j[1] = has1 ? J[i0 + 1] : 0u;
        bool run[2];
#pragma unroll
        for (int c = 0; c < 2; c++) {
            run[c] = k[c] != kV1bNone;
            x[c] = run[c] ? k[c] : (i0 + c == 0 ? 0u : j[c]);
        }
        while (run[0] || run[1]) {   // both chains' next links in flight together
            uint32_t h[2];
#pragma unroll
            for (int c = 0; c < 2; c++) h[c] = run[c] ? H[x[c]] : kV1bNone;
#pragma unroll
            for (int c = 0; c < 2; c++) {
                if (h[c] == kV1bNone) run[c] = false;
                else x[c] = h[c];
            }
        }
    }
    const bool in0 = p >= pos_lo && p < pos_hi, in1 = has1 && p + 1 >= pos_lo && p + 1 < pos_hi;
    for (int32_t r = 0; r < nout; r++) {   // (wave-uniform rank: scalar descriptor loads)
        const int64_t ns0 = ranks[rank_lo + r].new_start + wb;
        int64_t *o = out + (int64_t)r * count + (p - pos_lo);
        if (in0 && in1) *(longlong2 *)o = make_longlong2(wrap_id(ns0 + x[0], g.N), wrap_id(ns0 + x[1], g.N));
        else if (in0) o[0] = wrap_id(ns0 + x[0], g.N);
        else if (in1) o[1] = wrap_id(ns0 + x[1], g.N);
    }
}

namespace {
// entries per pass of the HBM path (~18 B each: a pass's workspace is <= 2.3 GB while windows
// have at most 2^27 entries; a longer window is one job of ~18 B per entry, up to ~39 GB near
// 2^31 -- pss.h states the cost, and a workspace the device cannot hold fails pss_generate with
// PSS_EHIP)
constexpr int64_t kV1xPassEntries = (int64_t)1 << 27;
int64_t v1x_jobs_per_pass(int64_t B) {
    const int64_t j = kV1xPassEntries / B;
    return j < 1 ? 1 : (j > 65535 ? 65535 : j);
}
uint32_t v1x_nbk(int64_t W) { return (uint32_t)((W + kV1bBW - 1) / kV1bBW); }
// words per job: J, S, H, PART (W each), PARTP (W u16), BCNT (nbk)
size_t v1x_job_words(int64_t W) { return (size_t)4 * W + (size_t)(W + 1) / 2 + v1x_nbk(W); }
}  // namespace

// n = the longest window of the launch.  The 20 bytes after the arrays hold the block scan's
// wave totals of a window shorter than 8 entries (k_v1_exact places them after its own arrays,
// which a short last window ends early) -- always reserved, whatever the longest window (ADVICE
// r05: B = 8 with a 7-entry last window wrote past a 10 * W allocation).
size_t v1_exact_lds_bytes(int64_t n, bool with_mt) {
    return (with_mt ? (size_t)kMtN * sizeof(uint32_t) : 0u) + (size_t)n * sizeof(uint32_t) +
           (size_t)3 * n * sizeof(uint16_t) + 20u;
}

bool v1_exact_supported(const Geometry &g) { return g.B < ((int64_t)1 << 31); }

// the windows' seeded MT states follow the draws (16-byte aligned)
static size_t v1x_st_offset(int64_t jobs, int64_t W) {
    return ((size_t)jobs * (size_t)W * sizeof(uint16_t) + 15u) & ~(size_t)15u;
}

static hipError_t v1x_big_draws(const Geometry &g, const V1xBig &b, int64_t epoch, hipStream_t s);

// the LDS path's draws: J (u16, W per window) then the windows' seeded MT states
static void v1x_small_draws(const Geometry &g, int64_t w_lo, int64_t nw, int64_t epoch, uint32_t *dst,
                            hipStream_t s) {
    uint32_t *ST = (uint32_t *)((char *)dst + v1x_st_offset(nw, g.B < g.ns ? g.B : g.ns));
    launch_mt_seed_streams(MtSeedSpec{epoch, w_lo, 0, 0, (uint32_t)nw}, ST, s);
    hipLaunchKernelGGL(k_v1x_draws, dim3((uint32_t)nw), dim3(64), 0, s, g, w_lo, nw, epoch,
                       (const uint32_t *)ST, (uint16_t *)dst);
}

// A draw slot: the MT draws of a call's windows -- they depend on the epoch and the windows
// alone (V1:165-171) -- made ahead of the call by the runtime (exact lookahead).  LDS windows:
// J and the seeded states; windows through HBM: J and the bucket counts, when one pass covers
// the call (else no slot: 0).
struct V1xSlot { bool ok, big; int64_t w_lo, nw, W; size_t bytes; };
static V1xSlot v1x_slot(const Geometry &g, int64_t pos_lo, int64_t count) {
    V1xSlot t{};
    const int64_t pos_hi = pos_lo + count < g.ns ? pos_lo + count : g.ns;
    if (pos_hi <= pos_lo || !v1_exact_supported(g) || !g.shuffle) return t;
    t.w_lo = pos_lo / g.B;
    t.nw = (pos_hi - 1) / g.B - t.w_lo + 1;
    t.W = g.B < g.ns ? g.B : g.ns;
    if (t.W <= kV1ExactMaxB) {
        t.ok = true;
        t.bytes = v1x_st_offset(t.nw, t.W) + (size_t)t.nw * kMtN * sizeof(uint32_t);
    } else if (t.nw <= v1x_jobs_per_pass(t.W)) {
        t.ok = t.big = true;
        t.bytes = ((size_t)t.nw * (size_t)t.W + (size_t)t.nw * v1x_nbk(t.W)) * sizeof(uint32_t);
    }
    return t;
}

size_t v1_exact_slot_bytes(const Geometry &g, int64_t pos_lo, int64_t count) {
    const V1xSlot t = v1x_slot(g, pos_lo, count);
    return t.ok ? t.bytes : 0;
}

// epochs drawn ahead: windows through HBM on a workgroup each (few, long: C5's 12 keep 12 CUs
// busy for ~3 ms) 8 (C5 V1 exact 3.75 -> 1.12 ms per epoch); one-wave draws of many windows fill
// the chip, and drawn ahead beside the resolution they slowed C2 from 0.40 to 0.80 ms: none.
// At most 4 GiB of slots; none without a slot.
int v1_exact_lookahead_depth(const Geometry &g, int64_t pos_lo, int64_t count) {
    const V1xSlot t = v1x_slot(g, pos_lo, count);
    if (!t.ok) return 0;
    const int want = t.big && t.nw < 1024 ? 8 : 0;
    const size_t cap = ((size_t)4 << 30) / (t.bytes ? t.bytes : 1);
    return cap < (size_t)want ? (int)cap : want;
}

hipError_t launch_v1_exact_draws(const Geometry &g, int64_t pos_lo, int64_t count, int64_t epoch,
                                 uint32_t *slot, hipStream_t s) {
    const V1xSlot t = v1x_slot(g, pos_lo, count);
    if (!t.ok || !slot) return hipErrorInvalidValue;
    if (!t.big) {
        v1x_small_draws(g, t.w_lo, t.nw, epoch, slot, s);
        return hipGetLastError();
    }
    V1xBig b{};
    b.w_lo = t.w_lo; b.nw = t.nw; b.j0 = 0; b.B = (uint32_t)t.W; b.nbk = v1x_nbk(t.W);
    b.nj = (uint32_t)t.nw;
    b.J = slot;
    b.BCNT = slot + (size_t)b.nj * b.B;
    return v1x_big_draws(g, b, epoch, s);
}

size_t v1_exact_ws_bytes(const Geometry &g, int32_t nr, int64_t pos_lo, int64_t count) {
    const int64_t pos_hi = pos_lo + count < g.ns ? pos_lo + count : g.ns;
    if (nr <= 0 || pos_hi <= pos_lo || !v1_exact_supported(g)) return 0;
    const int64_t nw = (pos_hi - 1) / g.B - pos_lo / g.B + 1;
    const int64_t jobs = nw;   // a window's draws and resolution serve every rank of the call
    const int64_t W = g.B < g.ns ? g.B : g.ns;   // the longest window
    if (W <= kV1ExactMaxB)   // the draws (u16), then the windows' seeded MT states
        return v1x_st_offset(jobs, W) + (size_t)jobs * kMtN * sizeof(uint32_t);
    const int64_t pj = jobs < v1x_jobs_per_pass(W) ? jobs : v1x_jobs_per_pass(W);
    return (size_t)pj * v1x_job_words(W) * sizeof(uint32_t);
}

// the draw stage of one pass (J and its bucket counts BCNT)
static hipError_t v1x_big_draws(const Geometry &g, const V1xBig &b, int64_t epoch, hipStream_t s) {
    hipError_t e = hipMemsetAsync(b.BCNT, 0, sizeof(uint32_t) * (size_t)b.nj * b.nbk, s);
    if (e != hipSuccess) return e;
    // few windows: a workgroup per window's MT stream (PSS_V1X_DRAWS_WG=0 / 1 forces a form)
    static const int wg_env = [] {
        const char *e = getenv("PSS_V1X_DRAWS_WG");
        return e ? atoi(e) : -1;
    }();
    const bool wg = wg_env == 0 || wg_env == 1 ? wg_env == 1 : b.nj < 1024;
    // a call's own single pass of few long windows: split over the chip (pss_v2split.h), the
    // scratch being the pass's S, H and PART (free until the partition runs; a slot drawn ahead
    // has none: b.S null)
    if (b.S && b.j0 == 0 && (uint64_t)b.nj == (uint64_t)b.nw &&
        v1x_draws_split(b.w_lo, b.nj, (uint32_t)v1x_len(g, b.w_lo), (uint32_t)v1x_len(g, b.w_lo + b.nw - 1), b.B,
                        b.nbk, epoch, b.J, b.BCNT, b.S, (size_t)3 * b.nj * b.B, wg, s))
        return hipGetLastError();
    if (wg) hipLaunchKernelGGL(k_v1x_draws32_wg, dim3(b.nj), dim3(kMtWgThreads), 0, s, g, b, epoch);
    else hipLaunchKernelGGL(k_v1x_draws32, dim3(b.nj), dim3(64), 0, s, g, b, epoch);
    return hipGetLastError();
}

// slot: the single pass's J and BCNT drawn ahead (v1_exact_slot_bytes), or null
static hipError_t launch_v1_exact_big(const Geometry &g, const RankDesc *ranks, int32_t rank_lo, int32_t nr,
                                      int64_t pos_lo, int64_t count, int64_t epoch, int64_t *out,
                                      uint32_t *ws, uint32_t *slot, hipStream_t s, const MapArgs &ma) {
    const int64_t pos_hi = pos_lo + count < g.ns ? pos_lo + count : g.ns;
    const int64_t w_lo = pos_lo / g.B, w_hi = (pos_hi - 1) / g.B;
    const int64_t nw = w_hi - w_lo + 1;
    const uint64_t jobs = (uint64_t)nw;   // one per window: shared by every rank of the call
    const int64_t W = g.B < g.ns ? g.B : g.ns;   // the longest window: the slice length
    const uint64_t per = (uint64_t)v1x_jobs_per_pass(W);
    const uint32_t B = (uint32_t)W;
    const uint32_t nbk = v1x_nbk(W);
    // the flat grids: XCD-major while they stay below 2^24 workgroups, else 2-D (blockIdx.y = the
    // window slot).  The layout is decided here and handed to the kernels in b.xcd, never inferred
    // from the dim3 (a 2-D grid of one job also has y == 1).  PSS_V1X_GRID2D=1 forces the 2-D form.
    static const bool force2d = [] {
        const char *e = getenv("PSS_V1X_GRID2D");
        return e && atoi(e) == 1;
    }();
    auto grid = [&](V1xBig &b, uint32_t xb) {
        b.xb = xb;
        const uint64_t flat = (uint64_t)xb * (((uint64_t)b.nj + 7) / 8) * 8;
        b.xcd = !force2d && flat < ((uint64_t)1 << 24) ? 1u : 0u;
        return b.xcd ? dim3((uint32_t)flat) : dim3(xb, b.nj);
    };
    for (uint64_t j0 = 0; j0 < jobs; j0 += per) {
        V1xBig b{};
        b.w_lo = w_lo; b.nw = nw; b.j0 = j0; b.B = B; b.nbk = nbk;
        b.nj = (uint32_t)(jobs - j0 < per ? jobs - j0 : per);
        b.J = ws;
        b.S = b.J + (size_t)b.nj * B;
        b.H = b.S + (size_t)b.nj * B;
        b.PART = b.H + (size_t)b.nj * B;
        b.BCNT = b.PART + (size_t)b.nj * B;
        b.PARTP = (uint16_t *)(b.BCNT + (size_t)b.nj * nbk);
        hipError_t e;
        if (slot && jobs <= per) {   // drawn ahead (one pass)
            b.J = slot;
            b.BCNT = slot + (size_t)b.nj * B;
        } else {
            e = v1x_big_draws(g, b, epoch, s);
            if (e != hipSuccess) return e;
        }
        hipLaunchKernelGGL(k_v1x_bscan, dim3(b.nj), dim3(kV1xScanNT), 0, s, g, b);
        V1xBig bp = b;
        const dim3 gp = grid(bp, (B + kV1pChunk - 1) / kV1pChunk);
        hipLaunchKernelGGL(k_v1x_part, gp, dim3(kV1pNT), 0, s, g, bp);
        V1xBig bs = b;
        const dim3 gs = grid(bs, nbk);
        hipLaunchKernelGGL(k_v1x_solve, gs, dim3(kV1sNT), 0, s, g, bs);
        // ids: two positions per thread and 16-byte stores when every rank row's pairs are
        // aligned (count, pos_lo and the window length even, a 16-byte aligned output)
        V1xBig bo = b;
        const bool pairs = !ma.fpos && ((count | pos_lo | g.B) & 1) == 0 && (((uintptr_t)out) & 15u) == 0;
        if (pairs) {
            const dim3 go = grid(bo, (B + 511) / 512);
            hipLaunchKernelGGL(k_v1x_out2, go, dim3(256), 0, s, g, bo, ranks, rank_lo, nr, pos_lo, count, out);
        } else {
            const dim3 go = grid(bo, (B + 255) / 256);
            hipLaunchKernelGGL(k_v1x_out, go, dim3(256), 0, s, g, bo, ranks, rank_lo, nr, pos_lo, count, out, ma);
        }
        e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t launch_v1_exact(const Geometry &g, const RankDesc *ranks, int32_t rank_lo, int32_t nr,
                           int64_t pos_lo, int64_t count, int64_t epoch, int64_t *out, void *ws,
                           hipStream_t s, const MapArgs *mapped, uint32_t *slot) {
    const MapArgs ma = mapped ? *mapped : MapArgs{};
    const int64_t pos_hi = pos_lo + count < g.ns ? pos_lo + count : g.ns;
    if (nr <= 0 || pos_hi <= pos_lo) return hipSuccess;
    if (!v1_exact_supported(g)) return hipErrorInvalidValue;
    if ((g.B < g.ns ? g.B : g.ns) > kV1ExactMaxB) {
        if (!ws) return hipErrorInvalidValue;
        return launch_v1_exact_big(g, ranks, rank_lo, nr, pos_lo, count, epoch, out, (uint32_t *)ws, slot, s, ma);
    }
    const int64_t w_lo = pos_lo / g.B, w_hi = (pos_hi - 1) / g.B;
    const int64_t nw = w_hi - w_lo + 1;
    const size_t lds = v1_exact_lds_bytes(g.B < g.ns ? g.B : g.ns, ws == nullptr);
    static const hipError_t attr = hipFuncSetAttribute(
        (const void *)k_v1_exact, hipFuncAttributeMaxDynamicSharedMemorySize,
        (int)v1_exact_lds_bytes(kV1ExactMaxB, true));
    if (attr != hipSuccess) return attr;
    // with a workspace, the serial MT phases run one wave per window (many windows in flight)
    // ahead of the resolution, the windows' states seeded before them (k_mt_seed_streams, 16
    // streams a wave on vector registers); without one, each workgroup's first wave does them
    // in place
    const uint32_t ngrp = (uint32_t)((nr + kV1FanRanks - 1) / kV1FanRanks);
    // (slot: the draws made ahead -- the slot holds what the workspace's first part would)
    if (ws && !slot) v1x_small_draws(g, w_lo, nw, epoch, (uint32_t *)ws, s);
    hipLaunchKernelGGL(k_v1_exact, dim3((uint32_t)(ngrp * nw)), dim3(kExactNT), lds, s, g, ranks, rank_lo, nr,
                       w_lo, nw, pos_lo, count, epoch, (const uint16_t *)(slot ? (void *)slot : ws), out, ma);
    return hipGetLastError();
}

}  // namespace pss
