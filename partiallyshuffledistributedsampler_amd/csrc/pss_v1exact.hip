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

#include "pss_device.h"

namespace pss {

namespace {
constexpr int kMtN = 624, kMtM = 397;

struct MtInitTable { uint32_t v[kMtN]; };
constexpr MtInitTable make_mt_init() {   // init_genrand(19650218), _randommodule.c
    MtInitTable t{};
    t.v[0] = 19650218u;
    for (int i = 1; i < kMtN; i++) t.v[i] = 1812433253u * (t.v[i - 1] ^ (t.v[i - 1] >> 30)) + (uint32_t)i;
    return t;
}
__constant__ MtInitTable kMtInit = make_mt_init();

constexpr int kExactNT = 256;

// Lanes of one wave hand values to each other through LDS here (the twist reads words other
// lanes wrote one round earlier).  The hardware keeps a wave's LDS operations in order, but
// the compiler reasons per thread and may hoist a load above a store it can prove is to a
// different address; this pins program order.
__device__ __forceinline__ void wave_lds_order() {
    __builtin_amdgcn_wave_barrier();
    __asm__ __volatile__("" ::: "memory");
}

__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
}

__device__ __forceinline__ uint32_t mt_twist_word(uint32_t a, uint32_t b, uint32_t c) {
    const uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
    return c ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
}

// init_by_array(key, klen) (random_seed -> init_by_array, _randommodule.c), klen <= 2.
// Serial; run by one wave with uniform values.  mt[] is LDS.
__device__ void mt_seed(uint32_t *mt, uint32_t key0, uint32_t key1, int klen) {
    const int lane = threadIdx.x & 63;
    // loop 1: i = 1..623, then the wrap (mt[0] = mt[623]) and one more step at i = 1
    uint32_t prev = kMtInit.v[0];
    uint32_t first = 0;
    int j = 0;
    for (int i = 1; i < kMtN; i++) {
        const uint32_t v = (kMtInit.v[i] ^ ((prev ^ (prev >> 30)) * 1664525u)) + (j ? key1 : key0) + (uint32_t)j;
        if (lane == 0) mt[i] = v;
        if (i == 1) first = v;
        prev = v;
        if (++j >= klen) j = 0;
    }
    {   // k = 623: i = 1 again, prev = mt[0] = mt[623]
        const uint32_t v = (first ^ ((prev ^ (prev >> 30)) * 1664525u)) + (j ? key1 : key0) + (uint32_t)j;
        if (lane == 0) mt[1] = v;
        prev = v;
    }
    wave_lds_order();
    // loop 2: i = 2..623, wrap, i = 1; 623 steps.  mt[i] (loop-1 values) come from LDS in
    // 64-word vectors read ahead of the chain.
    for (int i0 = 2; i0 < kMtN; i0 += 64) {
        const int cnt = kMtN - i0 < 64 ? kMtN - i0 : 64;
        const uint32_t vec = (lane < cnt) ? mt[i0 + lane] : 0u;
        uint32_t outv = 0;
        for (int l = 0; l < cnt; l++) {
            const uint32_t old = (uint32_t)__builtin_amdgcn_readlane((int)vec, l);
            const uint32_t v = (old ^ ((prev ^ (prev >> 30)) * 1566083941u)) - (uint32_t)(i0 + l);
            if (lane == l) outv = v;
            prev = v;
        }
        if (lane < cnt) mt[i0 + lane] = outv;
        wave_lds_order();
    }
    {   // wrap: mt[0] = mt[623]; i = 1
        const uint32_t old = mt[1];
        const uint32_t v = (old ^ ((prev ^ (prev >> 30)) * 1566083941u)) - 1u;
        if (lane == 0) { mt[1] = v; mt[0] = 0x80000000u; }
    }
    wave_lds_order();
}

// one MT19937 twist of mt[] in LDS by one wave, in 64-word rounds (program order keeps the
// old / new reads right: see the chunk boundaries 227 = N - M and 623)
__device__ void mt_twist(uint32_t *mt) {
    const int lane = threadIdx.x & 63;
    for (int k0 = 0; k0 < kMtN - 1; k0 += 64) {
        const int kk = k0 + lane;
        uint32_t v = 0;
        if (kk < kMtN - 1) {
            const uint32_t a = mt[kk], b = mt[kk + 1];
            const uint32_t c = kk < kMtN - kMtM ? mt[kk + kMtM] : mt[kk + kMtM - kMtN];
            v = mt_twist_word(a, b, c);
        }
        if (kk < kMtN - 1) mt[kk] = v;
        wave_lds_order();
    }
    if (lane == 0) mt[kMtN - 1] = mt_twist_word(mt[kMtN - 1], mt[0], mt[kMtM - 1]);
    wave_lds_order();
}

__device__ __forceinline__ uint64_t lanemask_lt() {
    const int lane = threadIdx.x & 63;
    return lane ? (~0ull >> (64 - lane)) : 0ull;
}
}  // namespace

// One workgroup per (local rank, window) of [w_lo, w_lo + nw).
__global__ __launch_bounds__(kExactNT) void k_v1_exact(Geometry g, const RankDesc *__restrict__ ranks,
                                                       int32_t rank_lo, int64_t w_lo, int64_t nw,
                                                       int64_t pos_lo, int64_t count, int64_t epoch,
                                                       int64_t *__restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    const int32_t rl = (int32_t)(blockIdx.x / nw);
    const int64_t w = w_lo + (int64_t)(blockIdx.x % nw);
    const int32_t rank = rank_lo + rl;
    const int64_t wb = w * g.B;
    const int n = (int)(g.ns - wb < g.B ? g.ns - wb : g.B);
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    uint32_t *mt = smem;                                   // [624]
    uint32_t *cnt = smem + kMtN;                           // [n + 1] bucket counts -> ends
    uint16_t *jv = (uint16_t *)(cnt + n + 1);              // [n] j_i
    uint16_t *lst = jv + n;                                // [n] steps bucketed by j
    uint16_t *nxt = lst + n;                               // [n] parent -> root
    __shared__ uint32_t tot[kExactNT / 64];

    if (wid == 0 && n > 1) {
        // ---- 1. seed(a): key = 32-bit words of abs(a) (random_seed) ----
        const int64_t a = w == 0 ? epoch : epoch + w * 10000;
        const uint64_t m = a < 0 ? (uint64_t)(-(a + 1)) + 1u : (uint64_t)a;
        const uint32_t k0 = (uint32_t)m, k1 = (uint32_t)(m >> 32);
        mt_seed(mt, k0, k1, k1 ? 2 : 1);
        // ---- 2. the draws of shuffle(range(n)) ----
        int s = n - 1;                       // next draw is j_s = _randbelow(s + 1)
        while (s >= 1) {
            mt_twist(mt);
            for (int q0 = 0; q0 < kMtN && s >= 1; q0 += 64) {
                const int nval = kMtN - q0 < 64 ? kMtN - q0 : 64;
                const uint32_t word = lane < nval ? mt_temper(mt[q0 + lane]) : 0u;
                uint32_t R = 0;
                int st;
                bool acc;
                uint32_t r;
                for (;;) {
                    st = s - lane + (int)R;
                    const bool valid = lane < nval && st >= 1;
                    const uint32_t sp1 = valid ? (uint32_t)st + 1u : 2u;
                    const uint32_t k = 32u - (uint32_t)__builtin_clz(sp1);   // bit_length(st + 1)
                    r = valid ? word >> (32u - k) : 0u;
                    acc = valid && r <= (uint32_t)st;
                    const uint64_t rej = __ballot(valid && !acc);
                    const uint32_t Rn = (uint32_t)__popcll(rej & lanemask_lt());
                    if (__ballot(Rn != R) == 0) break;
                    R = Rn;
                }
                if (acc) jv[st] = (uint16_t)r;
                s -= (int)__popcll(__ballot(acc));
            }
        }
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

hipError_t launch_v1_exact(const Geometry &g, const RankDesc *ranks, int32_t rank_lo, int32_t nr,
                           int64_t pos_lo, int64_t count, int64_t epoch, int64_t *out, hipStream_t s) {
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
    hipLaunchKernelGGL(k_v1_exact, dim3((uint32_t)(nr * nw)), dim3(kExactNT), lds, s, g, ranks, rank_lo,
                       w_lo, nw, pos_lo, count, epoch, out);
    return hipGetLastError();
}

}  // namespace pss
