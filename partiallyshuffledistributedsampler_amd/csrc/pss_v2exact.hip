// pss_v2exact.hip -- V2 in the reference's EXACT order (order mode PSS_ORDER_EXACT): the id
// stream of get_index (V2:96-116) bit for bit, CPython MT19937 included.
//
// The reference's loop, per step: k1 = _randbelow(len(pool1)), emit and `remove` pool1[k1];
// while pool2 is non-empty, k2 = _randbelow(len(pool2)), move pool2[k2] to the END of pool1;
// when pool2 runs dry, `seed(epoch + buffers*10000)` and refill it with the next window of the
// new start (V2:108-112).  That splits into independent pieces:
//
//   draws   every pool2 window is drawn from its own freshly seeded stream (segment 0 from
//           seed(e+2) of init_iter, V2:147; segment s >= 1 from seed(e + (s-1)*10000)), k1 and
//           k2 alternating: one wave per stream (pss_mt.h).  Once pool2 stays empty every step
//           reseeds, so each tail step's k1 is the first draw of its own stream: one LANE per
//           tail step (mt_first_draw_lane), 64 seeds per wave.
//   decode  "remove the k-th, append at the end" is a rank-deletion problem: with the
//           elements numbered in insertion order, step t removes the k_t-th alive one.  A block
//           of steps [a, b) is solved in the frame of its start (alive elements 0..B_a-1, its
//           own insertions after them).  Two sibling blocks combine in ONE merge: the right
//           block's answer q (its own frame) is the q-th survivor of the left block, q +
//           #{i : D_i - i <= q} for the left block's sorted deletions D, and it sorts right after
//           exactly those left entries -- so merging E_i = D_i - i with the right answers (left
//           first on ties) orders the pair and maps the right block at once (a right answer
//           taken after i left entries becomes q + i).  Bottom-up this is a merge sort of
//           (position, step) pairs: 12 levels in LDS per 4096-step tile.  Pools of <= 4096
//           entries then chain the tiles (below); bigger pools merge on through global levels.
//           pool2 windows (no insertions) finish inside one tile when B <= 4096; larger windows
//           are decoded first, as sequences of their own (B alive, no insertions) through the
//           same tile and global levels.  A short last window is padded to B steps of k = 0: its
//           W' real deletions never reach the B - W' padding elements at the end of the order,
//           so its real answers are unchanged.
//   chain   (pools <= 4096) each tile also leaves its survivor list -- the frame positions still
//           alive at its end, in order; the elements alive at a tile's start follow from the
//           previous tile's by that list, so per chunk of tiles the composite map is built in
//           parallel, chunks are linked per rank, and every tile's answers become ids.
//   output  position p < P is old_start + p (initial pool1, V2:135-136); position P + u is
//           the element step u moved over from pool2: window base + its decoded pool2 rank.
//
// tests/test_gpu_parity.py checks the streams against oracle/pss_oracle.c's exact V2 (pinned
// by the reference's recorded streams).
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <map>
#include <memory>
#include <mutex>
#include <tuple>
#include <vector>

#include "pss_mt.h"

namespace pss {

namespace {
constexpr int kTile = 4096;       // steps per LDS decode tile; pool2 windows up to this size decode in one
// consecutive merge outputs per thread (one search each per level; the first log2 of them
// merge levels run in registers)
#ifndef PSS_TILE_OUT
#define PSS_TILE_OUT 16
#endif
constexpr int kTileOut = PSS_TILE_OUT;
static_assert(kTileOut == 8 || kTileOut == 16, "tile outputs per thread: 8 or 16");

struct V2xGeo {                   // one rank's stream, host-computed
    uint32_t P, T, S, B;          // pool1 size, main steps, pool2 windows, shuffle_buffer
    uint32_t ns, tiles1;          // steps, pool1 decode tiles
    uint32_t T2;                  // pool2 draws / decoded ranks per rank, padded: S * B
};

__device__ __forceinline__ uint32_t alive_at(uint32_t B0, uint32_t insu, uint32_t x) {
    return B0 - (x > insu ? x - insu : 0u);
}
}  // namespace

// seed of tail step j (pool2 stays empty: every step reseeds first, V2:107-109)
__device__ __forceinline__ int64_t v2x_tail_seed(const V2xGeo &x, int64_t epoch, uint32_t j) {
    return x.S >= 1 ? epoch + (int64_t)(x.S - 1 + j) * 10000
                    : (j == 0 ? epoch + 2 : epoch + (int64_t)(j - 1) * 10000);
}

// ---- tail draws: one lane per tail step (its own reseeded stream's first draw) ---------------
// 64 tail steps per wave, each lane seeding its own MT (mt_first_draw_lane); the rare lane whose
// first kFirstWords words are all rejected is redone by the whole wave (mt_seed + mt_draws, in
// the wave's 624 words of LDS at mt).
__device__ __forceinline__ void v2x_tail_block(const V2xGeo &x, int64_t epoch, uint32_t rl, uint32_t j0,
                                               uint32_t *__restrict__ K1, uint32_t *mt) {
    uint32_t *k1 = K1 + (size_t)rl * x.ns;
    const int lane = threadIdx.x & 63;
    const uint32_t j = j0 + (uint32_t)lane;
    const bool valid = j < x.P;
    const int64_t seed = v2x_tail_seed(x, epoch, valid ? j : 0u);
    const uint64_t m = seed < 0 ? (uint64_t)(-(seed + 1)) + 1u : (uint64_t)seed;
    const uint32_t key0 = (uint32_t)m, key1 = (uint32_t)(m >> 32);
    const uint32_t n = valid ? x.P - j : 1u;
    uint32_t r = 0;
    const bool ok = mt_first_draw_lane(key0, key1, key1 ? 2 : 1, n, r);
    if (valid && ok) k1[x.T + j] = r;
    uint64_t redo = __ballot(valid && !ok);
    while (redo) {
        const int l = __ffsll((long long)redo) - 1;
        redo &= redo - 1ull;
        const uint32_t jl = j0 + (uint32_t)l;
        mt_seed_int(mt, v2x_tail_seed(x, epoch, jl));
        const uint32_t nl = x.P - jl, t = x.T + jl;
        mt_draws(mt, 1u, [&](uint32_t) { return nl; }, [&](uint32_t, uint32_t rr) { k1[t] = rr; });
        wave_lds_order();
    }
}

#include "pss_v2split.h"

// ---- seeding: the windows' MT states (k_mt_seed_streams' blocks), the tail draws alongside ----
// Both are latency-bound chains on few waves (C2: 191 seeding waves, 64 tail waves), so they share
// one launch ahead of the window draws.
__global__ __launch_bounds__(64) void k_v2x_seed(MtSeedSpec sp, uint32_t *__restrict__ ST, V2xGeo x, int64_t epoch,
                                                 uint32_t *__restrict__ K1) {
    __shared__ uint32_t t[kMtSeedLdsWords];
    const uint32_t nsb = mt_seed_blocks(sp.n);
    if (blockIdx.x < nsb) mt_seed_streams_block(sp, ST, t, blockIdx.x);
    else v2x_tail_block(x, epoch, 0u, (blockIdx.x - nsb) * 64u, K1, t);
}

// ---- draws: one wave per pool2 window's MT stream -----------------------------------------------
// The windows' MT states come seeded by k_v2x_seed (ST: [window][624]).
__global__ __launch_bounds__(64) void k_v2x_draws(V2xGeo x, uint32_t jobs, uint64_t blk0, const uint32_t *__restrict__ ST,
                                                  uint32_t *__restrict__ K1, uint32_t *__restrict__ K2) {
    __shared__ uint32_t mt[kMtN];
    const uint64_t b = blk0 + blockIdx.x;
    const uint32_t rl = (uint32_t)(b / jobs), job = (uint32_t)(b % jobs);
    uint32_t *k1 = K1 + (size_t)rl * x.ns;
    uint32_t *k2 = K2 + (size_t)rl * x.T2;
    if (job < x.S) {          // pool2 window s: k1, k2 alternating from its own stream
        const uint32_t s = job;
        const uint32_t W = x.T - s * x.B < x.B ? x.T - s * x.B : x.B, t0 = s * x.B;
        mt_load(mt, ST + (size_t)s * kMtN);
        mt_draws_pair(mt, W, x.P, [&](bool second, uint32_t i, uint32_t r) {
            if (second) k2[t0 + i] = r;
            else k1[t0 + i] = r;
        });
        for (uint32_t u = W + threadIdx.x; u < x.B; u += 64) k2[t0 + u] = 0;   // padding steps
    }
}

__global__ __launch_bounds__(64) void k_v2x_tail_draws(V2xGeo x, int64_t epoch, uint32_t per_rank,
                                                       uint64_t blk0, uint32_t *__restrict__ K1) {
    __shared__ uint32_t mt[kMtN];
    const uint64_t b = blk0 + blockIdx.x;
    v2x_tail_block(x, epoch, (uint32_t)(b / per_rank), (uint32_t)(b % per_rank) * 64u, K1, mt);
}

// The same draws with a workgroup per window (pss_mt.h mt_draws_pair_wg): long windows, few
// streams (C5: 2^20 steps each, ~11 per rank), which leave most of the chip idle for ~11 ms --
// so the launch also carries the tail draws: blocks past the windows' run ten tail blocks each
// (one per wave) on the CUs the streams do not use (C5: 1.96 ms of k_v2x_tail_draws hidden).
__global__ __launch_bounds__(kMtWgThreads) void k_v2x_draws_wg(V2xGeo x, int64_t epoch, uint32_t jobs, uint64_t blk0,
                                                              uint32_t nr, uint32_t tail_blocks,
                                                              uint32_t *__restrict__ K1, uint32_t *__restrict__ K2) {
    __shared__ MtWgShared sh;
    const uint64_t b = blk0 + blockIdx.x;
    if (b >= (uint64_t)jobs * nr) {   // tail mode: wave w takes tail block 10 (b - windows) + w
        const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));   // (uniform)
        const uint64_t tb = (b - (uint64_t)jobs * nr) * (uint64_t)kMtWgWaves + wv;
        const uint32_t rl = (uint32_t)(tb / tail_blocks);
        if (rl >= nr) return;
        static_assert(sizeof(sh.tw) + sizeof(sh.tw_pad) >= sizeof(uint32_t) * kMtN * kMtWgWaves,
                      "a tail wave's MT state in tw");
        v2x_tail_block(x, epoch, rl, (uint32_t)(tb % tail_blocks) * 64u, K1, (uint32_t *)sh.tw + kMtN * wv);
        return;
    }
    const uint32_t rl = (uint32_t)(b / jobs), job = (uint32_t)(b % jobs);
    if (job >= x.S) return;
    uint32_t *k1 = K1 + (size_t)rl * x.ns;
    uint32_t *k2 = K2 + (size_t)rl * x.T2;
    const uint32_t s = job;
    const uint32_t W = x.T - s * x.B < x.B ? x.T - s * x.B : x.B, t0 = s * x.B;
    if (threadIdx.x < 64) mt_seed_int(sh.mt[0], s == 0 ? epoch + 2 : epoch + (int64_t)(s - 1) * 10000);
    __syncthreads();
    mt_draws_pair_wg(sh, 0, W, x.P, [&](bool second, uint32_t i, uint32_t r) {
        if (second) k2[t0 + i] = r;
        else k1[t0 + i] = r;
    });
    for (uint32_t u = W + threadIdx.x; u < x.B; u += kMtWgThreads) k2[t0 + u] = 0;   // padding steps
}

// ---- decode tiles in LDS: pool1 tiles of kTile steps and whole pool2 windows ---------------
// An entry is one word: (frame position << kStepBits) | step within the tile -- 32-bit when
// every frame position of the launch stays below 2^20 (pools <= 2^20 - kTile: every C2-shaped
// launch), 64-bit otherwise -- so a merge step moves one LDS word, not a value and its step.
// kTileNT threads, kTileOut consecutive outputs each: one merge-path search per thread per
// level, then a walk that reads each entry once.
constexpr int kStepBits = 12;
static_assert((1 << kStepBits) == kTile, "a tile's steps fit the entry's step field");
template <typename EW> struct TileEntry {
    static constexpr int SH = sizeof(EW) == 4 ? kStepBits : 32;
    static __device__ __forceinline__ uint32_t val(EW e) { return (uint32_t)(e >> SH); }
    static __device__ __forceinline__ uint32_t step(EW e) { return (uint32_t)(e & (EW)(kTile - 1)); }
    static __device__ __forceinline__ EW make(uint32_t v, uint32_t st) { return ((EW)v << SH) | (EW)st; }
    static __device__ __forceinline__ EW add(EW e, uint32_t d) { return e + ((EW)d << SH); }
    // LDS index of entry p, skewed by one slot per 128 bytes: a thread's outputs are kTileOut
    // consecutive entries, so the lanes of a wave touch entries kTileOut apart -- unskewed that
    // is 16 (32-bit) / 8 (64-bit) lanes per bank
    static constexpr int SKEW = sizeof(EW) == 4 ? 5 : 4;
    static __device__ __forceinline__ uint32_t ix(uint32_t p) { return p + (p >> SKEW); }
    static constexpr uint32_t kSlots = kTile + (kTile >> SKEW);
};
// The first three merge levels (blocks of 1, 2, 4 -> 8) of a thread's 8 consecutive entries in
// registers: the same fused map-and-merge as the LDS levels, as a sorting network (frame
// positions below 2^28, so that a key fits 32 bits; 64-bit entries since round 4).
// A left entry i gets key (E_i << 4) | i with E_i = D_i - i, a right entry j key (q_j << 4) | 8 | j:
// left-before-right exactly when E_i <= q_j (left first on ties), lefts keep their order on equal E
// (the index below), rights are distinct.  Batcher's odd-even merge of the two sorted halves, then a
// right entry landing at k gains k - j (the left entries now before it).
template <typename EW>
__device__ __forceinline__ void tile_ce(uint32_t &ka, uint32_t &kb, EW &ea, EW &eb) {
    const bool sw = ka > kb;
    const uint32_t k0 = sw ? kb : ka, k1 = sw ? ka : kb;
    const EW e0 = sw ? eb : ea, e1 = sw ? ea : eb;
    ka = k0; kb = k1; ea = e0; eb = e1;
}
template <typename EW>
__device__ __forceinline__ void tile_merge8_regs(EW (&e)[8]) {
    using TE = TileEntry<EW>;
#pragma unroll
    for (int p = 0; p < 4; p++) {   // blocks of 1
        const EW l = e[2 * p], r = e[2 * p + 1];
        const bool take = TE::val(l) <= TE::val(r);
        e[2 * p] = take ? l : r;
        e[2 * p + 1] = take ? TE::add(r, 1u) : l;
    }
    auto keys = [&](int a, int w, uint32_t *k) {
        for (int i = 0; i < w; i++) k[i] = ((TE::val(e[a + i]) - (uint32_t)i) << 4) | (uint32_t)i;
        for (int j = 0; j < w; j++) k[w + j] = (TE::val(e[a + w + j]) << 4) | 8u | (uint32_t)j;
    };
    auto fix = [&](int a, int w, const uint32_t *k) {
        for (int q = 0; q < 2 * w; q++) {
            const uint32_t d = (k[q] & 8u) ? (uint32_t)q - (k[q] & 7u) : 0u;
            e[a + q] = TE::add(e[a + q], d);
        }
    };
#pragma unroll
    for (int a = 0; a < 8; a += 4) {   // blocks of 2
        uint32_t k[4];
        keys(a, 2, k);
        tile_ce(k[0], k[2], e[a], e[a + 2]);
        tile_ce(k[1], k[3], e[a + 1], e[a + 3]);
        tile_ce(k[1], k[2], e[a + 1], e[a + 2]);
        fix(a, 2, k);
    }
    {   // blocks of 4
        uint32_t k[8];
        keys(0, 4, k);
#pragma unroll
        for (int i = 0; i < 4; i++) tile_ce(k[i], k[i + 4], e[i], e[i + 4]);
        tile_ce(k[2], k[4], e[2], e[4]);
        tile_ce(k[3], k[5], e[3], e[5]);
        tile_ce(k[1], k[2], e[1], e[2]);
        tile_ce(k[3], k[4], e[3], e[4]);
        tile_ce(k[5], k[6], e[5], e[6]);
        fix(0, 4, k);
    }
}

// ... and four: two sorted blocks of 8 (tile_merge8_regs on each half) merged in registers by
// Batcher's odd-even merge of 8 + 8 (25 compare-exchanges), same keys (an index and the right
// flag fit the key's low 4 bits).
template <typename EW>
__device__ __forceinline__ void tile_merge16_regs(EW (&e)[16]) {
    using TE = TileEntry<EW>;
    EW lo[8], hi[8];
#pragma unroll
    for (int i = 0; i < 8; i++) { lo[i] = e[i]; hi[i] = e[8 + i]; }
    tile_merge8_regs(lo);
    tile_merge8_regs(hi);
    uint32_t k[16];
#pragma unroll
    for (int i = 0; i < 8; i++) {
        e[i] = lo[i];
        e[8 + i] = hi[i];
        k[i] = ((TE::val(lo[i]) - (uint32_t)i) << 4) | (uint32_t)i;
        k[8 + i] = (TE::val(hi[i]) << 4) | 8u | (uint32_t)i;
    }
#pragma unroll
    for (int i = 0; i < 8; i++) tile_ce(k[i], k[i + 8], e[i], e[i + 8]);
#pragma unroll
    for (int i = 0; i < 4; i++) tile_ce(k[i + 4], k[i + 8], e[i + 4], e[i + 8]);
    tile_ce(k[2], k[4], e[2], e[4]);
    tile_ce(k[3], k[5], e[3], e[5]);
    tile_ce(k[6], k[8], e[6], e[8]);
    tile_ce(k[7], k[9], e[7], e[9]);
    tile_ce(k[10], k[12], e[10], e[12]);
    tile_ce(k[11], k[13], e[11], e[13]);
#pragma unroll
    for (int i = 0; i < 7; i++) tile_ce(k[2 * i + 1], k[2 * i + 2], e[2 * i + 1], e[2 * i + 2]);
#pragma unroll
    for (int q = 0; q < 16; q++) {   // a right entry j landing at q has q - j left entries before it
        const uint32_t d = (k[q] & 8u) ? (uint32_t)q - (k[q] & 7u) : 0u;
        e[q] = TE::add(e[q], d);
    }
}

// largest frame position a launch can produce: pool1 tiles P + kTile, windows B
static bool v2x_narrow(uint32_t P, uint32_t B) {
    return (uint64_t)P + kTile <= ((uint64_t)1 << (32 - kStepBits)) && (uint64_t)B <= ((uint64_t)1 << (32 - kStepBits));
}

template <typename EW, int OUT>
__global__ __launch_bounds__(kTile / OUT) void k_v2x_tile(V2xGeo x, uint32_t per_rank, uint64_t blk0,
                                                      const uint32_t *__restrict__ K1,
                                                      const uint32_t *__restrict__ K2,
                                                      uint32_t *__restrict__ V, uint32_t *__restrict__ O,
                                                      uint32_t *__restrict__ Q2, uint32_t *__restrict__ SV) {
    using TE = TileEntry<EW>;
    constexpr uint32_t NT = kTile / OUT;
    extern __shared__ __attribute__((aligned(16))) uint32_t smem_u32[];
    EW *va = (EW *)smem_u32, *vb = va + TE::kSlots;
    const uint64_t bi = blk0 + blockIdx.x;
    const uint32_t rl = (uint32_t)(bi / per_rank), job = (uint32_t)(bi % per_rank);
    const bool pool1 = job < x.tiles1;
    uint32_t t0, n, B0, insu;
    const uint32_t *src;
    if (pool1) {
        t0 = job * kTile;
        n = x.ns - t0 < (uint32_t)kTile ? x.ns - t0 : (uint32_t)kTile;
        B0 = x.P; insu = x.T;
        src = K1 + (size_t)rl * x.ns + t0;
    } else {
        const uint32_t s = job - x.tiles1;
        t0 = 0;
        n = x.T - s * x.B < x.B ? x.T - s * x.B : x.B;
        B0 = n; insu = 0;
        src = K2 + (size_t)rl * x.T2 + (size_t)s * x.B;
    }
    uint32_t w0 = 1;
    // (the register levels' keys hold a frame position in 28 bits)
    const bool regs = sizeof(EW) == 4 || ((uint64_t)x.P + kTile < ((uint64_t)1 << 28) && x.B < (1u << 28));
    if constexpr (OUT == 8) {
        if (n == (uint32_t)kTile && regs) {   // full tile: a thread's 8 entries merged in registers first
            const uint32_t b = threadIdx.x * 8u;
            EW e[8];
#pragma unroll
            for (int i = 0; i < 8; i++) e[i] = TE::make(src[b + i], b + (uint32_t)i);
            tile_merge8_regs(e);
#pragma unroll
            for (int i = 0; i < 8; i++) va[TE::ix(b + (uint32_t)i)] = e[i];
            w0 = 8;
        }
    } else if constexpr (OUT == 16) {
        if (n == (uint32_t)kTile && regs) {   // full tile: a thread's 16 entries merged in registers first
            const uint32_t b = threadIdx.x * 16u;
            EW e[16];
#pragma unroll
            for (int i = 0; i < 16; i++) e[i] = TE::make(src[b + i], b + (uint32_t)i);
            tile_merge16_regs(e);
#pragma unroll
            for (int i = 0; i < 16; i++) va[TE::ix(b + (uint32_t)i)] = e[i];
            w0 = 16;
        }
    }
    if (w0 == 1)
        for (uint32_t u = threadIdx.x; u < n; u += NT) va[TE::ix(u)] = TE::make(src[u], u);
    __syncthreads();
    // merge levels: sibling blocks [a, m), [m, e) -> [a, e), each sorted by its frame position.
    // Left entries (deletions D, frame a) keep their values; a right entry q (frame m) is the
    // q-th survivor of the left block, i.e. q + #{i : D_i - i <= q} in frame a, and it falls
    // after exactly those left entries -- so one merge of E_i = D_i - i (non-decreasing) with the
    // right values (left first on ties) both orders the pair and maps the right block: a right
    // entry taken after i left ones becomes q + i.  (q beyond the left block's survivors are the
    // right block's own insertions: every E_i <= q there, and q + nL is their frame-a position.)
    const uint32_t p0 = threadIdx.x * (uint32_t)OUT;
    for (uint32_t w = w0; w < n; w <<= 1) {
        if (w >= (uint32_t)OUT) {
            // (wave-uniform) a thread's OUT outputs lie inside one pair: a binary-lifting
            // merge-path search of log2(w) + 1 uniform rounds, then a branch-free walk
            // (both candidates' next entry chosen by select, one LDS read per output)
            const uint32_t q = p0;
            if (q < n) {
                const uint32_t a = q & ~(2u * w - 1u), m = a + w;
                const uint32_t pe = q + (uint32_t)OUT < n ? q + (uint32_t)OUT : n;
                if (m >= n) {
#pragma unroll
                    for (int t = 0; t < OUT; t++)
                        if (q + (uint32_t)t < pe) vb[TE::ix(q + t)] = va[TE::ix(q + t)];
                } else {
                    const uint32_t e = m + w < n ? m + w : n, nL = w, nR = e - m, d = q - a;
                    const uint32_t lo = d > nR ? d - nR : 0u, hi = d < nL ? d : nL;
                    // i = lo + #{consecutive i >= lo : E_L(i) <= R(d - i - 1)} (monotone)
                    uint32_t i = lo;
                    for (uint32_t sp = w; sp; sp >>= 1) {
                        const uint32_t c = i + sp;
                        if (c <= hi) {
                            const uint32_t mid = c - 1u;
                            if (TE::val(va[TE::ix(a + mid)]) - mid <= TE::val(va[TE::ix(m + d - mid - 1u)])) i = c;
                        }
                    }
                    // (exhausted sides read a clamped, valid entry that is never taken; bools
                    // combined bitwise so that no lane takes a branch)
                    const uint32_t lL = nL - 1u, lR = nR - 1u;
                    uint32_t j = d - i;
                    EW xl = va[TE::ix(a + min(i, lL))], xr = va[TE::ix(m + min(j, lR))];
#pragma unroll
                    for (int t = 0; t < OUT; t++) {
                        const bool takeL = (j >= nR) | ((i < nL) & (TE::val(xl) - i <= TE::val(xr)));
                        const EW o = takeL ? xl : TE::add(xr, i);
                        if (q + (uint32_t)t < pe) vb[TE::ix(q + t)] = o;
                        i += (uint32_t)takeL;
                        j = d + (uint32_t)t + 1u - i;
                        if (t + 1 < OUT) {
                            const uint32_t ni = takeL ? a + min(i, lL) : m + min(j, lR);
                            const EW nx = va[TE::ix(ni)];
                            xl = takeL ? nx : xl;
                            xr = takeL ? xr : nx;
                        }
                    }
                }
            }
            __syncthreads();
            EW *t = va; va = vb; vb = t;
            continue;
        }
        // a thread's outputs may span several pairs while 2w < OUT: one walk per pair
        for (uint32_t q = p0; q < p0 + (uint32_t)OUT && q < n;) {
            const uint32_t a = (q / (2 * w)) * (2 * w), m = a + w;
            const uint32_t pe0 = a + 2 * w < p0 + (uint32_t)OUT ? a + 2 * w : p0 + (uint32_t)OUT;
            const uint32_t pe = pe0 < n ? pe0 : n;
            if (m >= n) {
                for (uint32_t p = q; p < pe; p++) vb[TE::ix(p)] = va[TE::ix(p)];
            } else {
                const uint32_t e = m + w < n ? m + w : n, nL = w, nR = e - m, d = q - a;
                auto L = [&](uint32_t i) { return va[TE::ix(a + i)]; };
                auto R = [&](uint32_t j) { return va[TE::ix(m + j)]; };
                uint32_t lo = d > nR ? d - nR : 0u, hi = d < nL ? d : nL;
                while (lo < hi) {
                    const uint32_t mid = (lo + hi) >> 1;
                    if (TE::val(L(mid)) - mid <= TE::val(R(d - mid - 1))) lo = mid + 1; else hi = mid;
                }
                uint32_t i = lo, j = d - lo;
                EW xl = i < nL ? L(i) : (EW)0, xr = j < nR ? R(j) : (EW)0;
                for (uint32_t p = q; p < pe; p++) {
                    const bool takeL = j >= nR || (i < nL && TE::val(xl) - i <= TE::val(xr));
                    if (takeL) {
                        vb[TE::ix(p)] = xl;
                        i++;
                        if (i < nL) xl = L(i);
                    } else {
                        vb[TE::ix(p)] = TE::add(xr, i);
                        j++;
                        if (j < nR) xr = R(j);
                    }
                }
            }
            q = pe;
        }
        __syncthreads();
        EW *t = va; va = vb; vb = t;
    }
    if (pool1 && SV) {
        // chain mode (pools of <= kTile entries): each step's answer in step order, and the
        // tile's survivors -- the frame positions still alive at its end, in order: survivor r
        // is r + #{i : D_i - i <= r} over the sorted deletions D (k_v2x_compose / _emit)
        // both lists are staged in the free LDS buffer (32-bit words, skewed per 128 B) and
        // stored coalesced
        uint32_t *svl = (uint32_t *)vb;
        uint32_t *ans = V + (size_t)rl * x.ns + t0;
        for (uint32_t u = threadIdx.x; u < n; u += NT) {
            const EW e = va[TE::ix(u)];
            const uint32_t st = TE::step(e);
            svl[st + (st >> 5)] = TE::val(e);
        }
        __syncthreads();
        for (uint32_t u = threadIdx.x; u < n; u += NT) ans[u] = svl[u + (u >> 5)];
        __syncthreads();
        const uint32_t Bm = alive_at(B0, insu, t0 + n);
        uint32_t *sv = SV + ((size_t)rl * x.tiles1 + job) * x.P;
        // OUT consecutive survivors per thread: one search for the first, then a walk (E_i =
        // D_i - i is non-decreasing)
        static_assert(NT * OUT >= kTile, "a tile's survivors: OUT per thread");
        const uint32_t r0 = threadIdx.x * (uint32_t)OUT;
        if (r0 < Bm) {
            uint32_t lo = 0, hi = n;   // #{i : D_i - i <= r0}
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if (TE::val(va[TE::ix(mid)]) - mid <= r0) lo = mid + 1; else hi = mid;
            }
            uint32_t i = lo;
            uint32_t e = i < n ? TE::val(va[TE::ix(i)]) - i : 0xFFFFFFFFu;
            for (uint32_t r = r0; r < r0 + (uint32_t)OUT && r < Bm; r++) {
                while (e <= r) {
                    i++;
                    e = i < n ? TE::val(va[TE::ix(i)]) - i : 0xFFFFFFFFu;
                }
                svl[r + (r >> 5)] = r + i;
            }
        }
        __syncthreads();
        for (uint32_t r = threadIdx.x; r < Bm; r += NT) sv[r] = svl[r + (r >> 5)];
    } else if (pool1) {
        uint32_t *v = V + (size_t)rl * x.ns + t0, *o = O + (size_t)rl * x.ns + t0;
        for (uint32_t u = threadIdx.x; u < n; u += NT) { const EW e = va[TE::ix(u)]; v[u] = TE::val(e); o[u] = t0 + TE::step(e); }
    } else {
        // the window's pool2 ranks in step order, staged in the free LDS buffer, stored coalesced
        uint32_t *q = Q2 + (size_t)rl * x.T2 + (size_t)(job - x.tiles1) * x.B;
        uint32_t *stg = (uint32_t *)vb;
        for (uint32_t u = threadIdx.x; u < n; u += NT) {
            const EW e = va[TE::ix(u)];
            const uint32_t st = TE::step(e);
            stg[st + (st >> 5)] = TE::val(e);
        }
        __syncthreads();
        for (uint32_t u = threadIdx.x; u < n; u += NT) q[u] = stg[u + (u >> 5)];
    }
}

// ---- global levels of the pool1 decode: blocks of w steps -> 2w -----------------------------
// Tiled like a GPU merge sort: a workgroup owns kGTile consecutive entries of one rank, finds
// where its tile starts and ends in the sorted lists it reads (one binary search each, in
// HBM), stages those sub-ranges in LDS with coalesced loads, works from LDS (kPer entries per
// thread: one LDS search, then a sequential walk) and writes its tile back coalesced.
constexpr uint32_t kGNT = 256, kPer = 8, kGTile = kGNT * kPer;   // w >= kTile is a multiple
// ranks one output block writes: the decode is shared by every rank of a call, its last stage
// writes each position's id for up to kFanRanks ranks (more ranks: more block rows, each
// re-reading the same decoded entries)
constexpr int32_t kFanRanks = 8;

// Merge-path splits of every gmerge tile's first and end output, all at once (one thread per
// tile boundary, so the binary searches' HBM latency overlaps).
__global__ __launch_bounds__(256) void k_v2x_gsplit(V2xGeo x, uint32_t nr, uint32_t w,
                                                    const uint32_t *__restrict__ V, uint32_t *__restrict__ SP) {
    const uint32_t tpr = (x.ns + kGTile - 1) / kGTile;
    const uint64_t gi = (uint64_t)blockIdx.x * 256 + threadIdx.x;   // (rank, tile, end?)
    if (gi >= (uint64_t)nr * tpr * 2) return;
    const uint32_t rl = (uint32_t)(gi / (2 * tpr)), tt = (uint32_t)(gi % (2 * tpr));
    const uint32_t tile = tt >> 1, endp = tt & 1u;
    const uint32_t *v = V + (size_t)rl * x.ns;
    const uint32_t u0 = tile * kGTile, un = x.ns - u0 < kGTile ? x.ns - u0 : kGTile;
    uint32_t r = 0;
    {
        const uint32_t a = (u0 / (2 * w)) * (2 * w), m = a + w;
        if (m < x.ns) {
            const uint32_t e = m + w < x.ns ? m + w : x.ns, nL = m - a, nR = e - m;
            const uint32_t *L = v + a, *R = v + m;
            const uint32_t d = u0 - a + (endp ? un : 0u);
            uint32_t lo = d > nR ? d - nR : 0u, hi = d < nL ? d : nL;
            while (lo < hi) {   // the fused map-and-merge order of k_v2x_tile
                const uint32_t mid = (lo + hi) >> 1;
                if (L[mid] - mid <= R[d - mid - 1]) lo = mid + 1; else hi = mid;
            }
            r = lo;
        }
    }
    SP[gi] = r;
}

// merge sibling blocks (sorted by position, carrying the step of each entry).  The LDS copies are
// swizzled inside each 32-word row (entry e at e ^ ((e / 32) mod 8)): a thread's merge walk reads
// and writes its own kPer consecutive entries, so unswizzled the 32 lanes of a half-wave hit every
// 8th bank -- 2/3 of the kernel's LDS cycles were bank conflicts (profiles/r04/pmc_exact/)
__device__ __forceinline__ uint32_t gsk(uint32_t e) { return e ^ ((e >> 5) & 7u); }
constexpr uint32_t kGTileSk = kGTile;
// The merge walk keeps a thread's kPer outputs in registers and stores them itself (two 16-byte
// stores per array when the output rows are 16-byte aligned; the lanes of a wave then write 2 KB
// contiguous): no LDS output staging, 16 KB of LDS per workgroup instead of 32 KB
// The last level writes what the lists are for instead of the lists themselves: the decoded pool2
// windows' ranks Q2[window][step] (FIN 1, a scatter inside one window), or the pool1 decode's
// ids / (file, offset) pairs (FIN 2, position p < P is old_start + p, P + u the element step u
// moved over from pool2: its window's base + its decoded pool2 rank)
struct V2xFin {
    Geometry g;
    const RankDesc *ranks;
    int32_t rank_lo;
    int32_t nout;                 // ranks of the call
    uint32_t *VV;                 // FIN 2: the virtual index of every step of the sequence
    uint32_t *Q2;                 // FIN 1: written ([seq][B]); FIN 2: read ([rank][T2])
    int64_t pos_lo, count;
    int64_t *out;
    MapArgs ma;
};
// FIN 2: the decoded sequence's virtual index at step t -- q < P the initial pool1 position, else
// the element's window base + its pool2 rank (window 0 is the old start's second window,
// V2:135-138) -- into VV[t] (u32: v < ns < 2^31).  The merge order is by position, so these are
// scattered 4-byte stores into one sequence-sized array (MALL-resident at C5's 50 MB); the ids of
// every rank of the call then come from k_v2x_fanout in step order, coalesced.
__device__ __forceinline__ void v2x_put(const V2xFin &f, const V2xGeo &x, uint32_t rl, uint32_t q, uint32_t t) {
    uint32_t v;
    if (q < x.P) {
        v = q;
    } else {
        const uint32_t uu = q - x.P, sw = uu / x.B;
        v = (sw + 1u) * x.B + f.Q2[(size_t)rl * x.T2 + uu];
    }
    f.VV[t] = v;
}

// ids of nout ranks from the virtual-index stream VV (position t at VV[t]): v < min(2B, ns) came
// from the old start, the rest from the new one (V2:135-148), wrapped at N (V2:113-114); each
// rank's row written coalesced.
// One-shot: 4 consecutive positions per thread, `per_row` ranks per workgroup row (blockIdx.y),
// 16-byte stores -- the store shape of torch's fill_.  A rank row whose first element sits at an
// odd element index (an odd `count`: every other row) is written in the 16-byte-aligned pairs
// (t0 + 1, t0 + 2), (t0 + 3, t0 + 4), the row's first element alone.  (Round 6: the 16-byte path
// used to need an even count for all rows; C3's 976,563 positions per rank sent all 1024 rows
// of its exact-order fan-out down the 8-byte path with the rank loop in every thread: 14.8 ms
// for the 8 GB.)
// Ranks per workgroup row: 8 for a call of few ranks (one 16-byte VV load serves 8 rows), 1 for
// many (round 6, same box: exact C3's 1024 ranks 2.31 / 2.17 / 2.07 ms per epoch at 8 / 2 / 1
// per row, C2's 8 ranks 0.805 / 0.836 / 0.816 ms; profiles/r06/ab_fanout/).
constexpr int32_t kFanoutRanksFew = 8, kFanoutManyRanks = 64;
__global__ __launch_bounds__(256) void k_v2x_fanout(Geometry g, const RankDesc *__restrict__ ranks, int32_t rank_lo,
                                                    int32_t nout, int32_t per_row, const uint32_t *__restrict__ VV,
                                                    int64_t pos_lo, int64_t count, int64_t *__restrict__ out, MapArgs ma) {
    const int64_t twoB = 2 * g.B < g.ns ? 2 * g.B : g.ns;
    const int64_t pos_hi = pos_lo + count < g.ns ? pos_lo + count : g.ns;
    const int64_t t0 = pos_lo + ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
    if (t0 >= pos_hi) return;
    const int32_t r_lo = (int32_t)blockIdx.y * per_row;
    const int32_t r_hi = nout - r_lo < per_row ? nout : r_lo + per_row;
    if (ma.fpos) {   // (file, offset) pairs: element by element
        for (int64_t t = t0; t < t0 + 4 && t < pos_hi; t++) {
            const int64_t v = VV[t];
            const bool old_side = v < twoB;
            for (int32_t r = r_lo; r < r_hi; r++) {
                const RankDesc rd = ranks[rank_lo + r];
                put_id_or_pair(out, ma, (int64_t)r * count + (t - pos_lo),
                               wrap_id((old_side ? rd.old_start : rd.new_start) + v, g.N));
            }
        }
        return;
    }
    // the values at t0 .. t0 + 4 (t0 + 4: the odd rows' second pair); the 16-byte VV load needs
    // VV + t0 itself 16-byte aligned (VV follows the workspace's other arrays)
    const bool full = t0 + 4 <= pos_hi;
    uint32_t v[5];
    if (full && (((uintptr_t)(VV + t0)) & 15u) == 0) {
        const uint4 w = *(const uint4 *)(VV + t0);
        v[0] = w.x; v[1] = w.y; v[2] = w.z; v[3] = w.w;
    } else {
#pragma unroll
        for (int k = 0; k < 4; k++) v[k] = t0 + k < pos_hi ? VV[t0 + k] : 0u;
    }
    v[4] = t0 + 4 < pos_hi ? VV[t0 + 4] : 0u;
    const bool out16 = (((uintptr_t)out) & 15u) == 0;
    for (int32_t r = r_lo; r < r_hi; r++) {
        const RankDesc rd = ranks[rank_lo + r];
        int64_t id[5];
#pragma unroll
        for (int k = 0; k < 5; k++) id[k] = wrap_id(((int64_t)v[k] < twoB ? rd.old_start : rd.new_start) + (int64_t)v[k], g.N);
        int64_t *row = out + (int64_t)r * count - pos_lo;   // position t at row[t]
        const bool even = ((((int64_t)r * count) & 1) == 0);   // row[t0] 16-byte aligned (t0 - pos_lo even)
        if (out16 && even && full) {
            *(longlong2 *)(row + t0) = make_longlong2(id[0], id[1]);
            *(longlong2 *)(row + t0 + 2) = make_longlong2(id[2], id[3]);
        } else if (out16 && !even) {
            if (t0 == pos_lo) row[t0] = id[0];
            if (t0 + 2 < pos_hi) *(longlong2 *)(row + t0 + 1) = make_longlong2(id[1], id[2]);
            else if (t0 + 1 < pos_hi) row[t0 + 1] = id[1];
            if (t0 + 4 < pos_hi) *(longlong2 *)(row + t0 + 3) = make_longlong2(id[3], id[4]);
            else if (t0 + 3 < pos_hi) row[t0 + 3] = id[3];
        } else {
#pragma unroll
            for (int k = 0; k < 4; k++)
                if (t0 + k < pos_hi) row[t0 + k] = id[k];
        }
    }
}

template <int FIN>
__global__ __launch_bounds__(kGNT) void k_v2x_gmerge(V2xGeo x, uint32_t w, const uint32_t *__restrict__ V,
                                                    const uint32_t *__restrict__ O, uint32_t *__restrict__ Vd,
                                                    uint32_t *__restrict__ Od, const uint32_t *__restrict__ SP,
                                                    V2xFin fin) {
    __shared__ uint32_t sv[kGTileSk], so[kGTileSk];
    const uint32_t tpr = (x.ns + kGTile - 1) / kGTile;
    const uint32_t rl = blockIdx.x / tpr, o0 = (blockIdx.x % tpr) * kGTile;
    const size_t base = (size_t)rl * x.ns;
    const uint32_t *v = V + base, *o = O + base;
    uint32_t *vd = Vd + base, *od = Od + base;
    const uint32_t on = x.ns - o0 < kGTile ? x.ns - o0 : kGTile;
    const uint32_t a = (o0 / (2 * w)) * (2 * w), m = a + w;
    auto emit = [&](uint32_t p, uint32_t val, uint32_t st) {   // output p (of the tile) = (val, st)
        if constexpr (FIN == 0) { vd[o0 + p] = val; od[o0 + p] = st; }
        else if constexpr (FIN == 1) fin.Q2[(size_t)rl * x.ns + st] = val;
        else v2x_put(fin, x, rl, val, st);
    };
    if (m >= x.ns) {                           // lone left block: already merged
        for (uint32_t u = threadIdx.x; u < on; u += kGNT) emit(u, v[o0 + u], o[o0 + u]);
        return;
    }
    const uint32_t i0 = SP[2 * blockIdx.x], i1 = SP[2 * blockIdx.x + 1], dA = o0 - a;   // merge-path splits
    const uint32_t j0 = dA - i0, j1 = dA + on - i1;
    const uint32_t sL = i1 - i0, sR = j1 - j0;   // sL + sR == on
    // (all kPer loads of a thread issued before its LDS stores measured slower: C5 exact 24.5 ->
    // 26.1 ms together with the same change in k_v2x_tile, profiles/r04/ab_gmerge_batch/)
    const uint32_t *L = v + a, *R = v + m;
    for (uint32_t u = threadIdx.x; u < sL; u += kGNT) { sv[gsk(u)] = L[i0 + u]; so[gsk(u)] = o[a + i0 + u]; }
    for (uint32_t u = threadIdx.x; u < sR; u += kGNT) { sv[gsk(sL + u)] = R[j0 + u]; so[gsk(sL + u)] = o[m + j0 + u]; }
    __syncthreads();
    const uint32_t p0 = threadIdx.x * kPer;
    if (p0 >= on) return;
    // the fused map-and-merge of k_v2x_tile: E_i = D_i - i against the right values (frame
    // m), a right entry after i0 + i left ones becomes q + i0 + i (frame a)
    auto lv = [&](uint32_t i) { return sv[gsk(i)]; };
    auto rv = [&](uint32_t j) { return sv[gsk(sL + j)]; };
    uint32_t lo = p0 > sR ? p0 - sR : 0u, hi = p0 < sL ? p0 : sL;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (lv(mid) - (i0 + mid) <= rv(p0 - mid - 1)) lo = mid + 1; else hi = mid;
    }
    uint32_t i = lo, j = p0 - lo;
    const uint32_t pn = on - p0 < kPer ? on - p0 : kPer;
    // branch-free walk: the current entry of each side in registers (an exhausted side holds a
    // clamped, valid LDS entry that is never taken), one LDS read pair per output for the side
    // just consumed
    const uint32_t lL = sL ? sL - 1u : 0u, lR = sR ? sR - 1u : 0u;
    uint32_t xl, ol, xr, orr;
    {
        const uint32_t ia = gsk(min(i, lL)), ib = gsk(sL + min(j, lR));
        xl = sv[ia]; ol = so[ia]; xr = sv[ib]; orr = so[ib];
    }
    uint32_t tv[kPer], to[kPer];
#pragma unroll
    for (uint32_t k = 0; k < kPer; k++) {
        const bool takeL = (j >= sR) | ((i < sL) & (xl - (i0 + i) <= xr));
        tv[k] = takeL ? xl : xr + i0 + i;
        to[k] = takeL ? ol : orr;
        i += (uint32_t)takeL;
        j = p0 + k + 1u - i;
        if (k + 1 < kPer) {
            const uint32_t ix = gsk(takeL ? min(i, lL) : sL + min(j, lR));
            const uint32_t nv = sv[ix], no = so[ix];
            xl = takeL ? nv : xl; ol = takeL ? no : ol;
            xr = takeL ? xr : nv; orr = takeL ? orr : no;
        }
    }
    static_assert(kPer == 8, "two 16-byte stores per array");
    if (FIN == 0 && pn == kPer && ((((uintptr_t)(vd + o0)) | ((uintptr_t)(od + o0))) & 15u) == 0) {
        uint4 *v4 = (uint4 *)(vd + o0 + p0), *o4 = (uint4 *)(od + o0 + p0);
        v4[0] = make_uint4(tv[0], tv[1], tv[2], tv[3]); v4[1] = make_uint4(tv[4], tv[5], tv[6], tv[7]);
        o4[0] = make_uint4(to[0], to[1], to[2], to[3]); o4[1] = make_uint4(to[4], to[5], to[6], to[7]);
    } else {
#pragma unroll
        for (uint32_t k = 0; k < kPer; k++)
            if (k < pn) emit(p0 + k, tv[k], to[k]);
    }
}

// ---- chain mode (pools of <= kTile entries): tiles linked by their survivor lists ----------
// A_j = the absolute insertion numbers of the elements alive at tile j's start (sorted; initial
// element p is number p, the element step t moves over from pool2 is P + t).  Frame position q of
// tile j is A_j[q] below B_j = alive_at(t0_j), else the tile's own insertion P + t0_j + q - B_j,
// and A_{j+1}[r] is frame position S_j[r] of tile j.  Three kernels replace the global merge
// levels: per chunk of tiles the composite survivor map relative to the chunk's start
// (compose), the chunks' A by a parallel prefix over those maps (link levels), then every tile
// again from its chunk's A, emitting the ids of its steps (emit).
constexpr uint32_t kAbs = 0x80000000u;   // composite entry: an absolute insertion number
constexpr int kChainNT = 1024;

struct V2xChain {
    uint32_t nch, tpc;     // chunks per rank, tiles per chunk
    uint32_t *SV, *CC, *AA, *PP;   // PP: the prefix levels' spare buffer (nch maps)
};

__global__ __launch_bounds__(kChainNT) void k_v2x_compose(V2xGeo x, V2xChain ch) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    uint32_t *G = smem, *Gn = smem + x.P;
    const uint32_t rl = blockIdx.x / ch.nch, c = blockIdx.x % ch.nch;
    const uint32_t j0 = c * ch.tpc, j1 = j0 + ch.tpc < x.tiles1 ? j0 + ch.tpc : x.tiles1;
    const uint32_t Ba0 = alive_at(x.P, x.T, j0 * (uint32_t)kTile);
    for (uint32_t r = threadIdx.x; r < Ba0; r += kChainNT) G[r] = r;
    __syncthreads();
    uint32_t Bend = Ba0;
    for (uint32_t j = j0; j < j1; j++) {
        const uint32_t t0 = j * (uint32_t)kTile, n = x.ns - t0 < (uint32_t)kTile ? x.ns - t0 : (uint32_t)kTile;
        const uint32_t Ba = alive_at(x.P, x.T, t0), Bm = alive_at(x.P, x.T, t0 + n);
        const uint32_t *sv = ch.SV + ((size_t)rl * x.tiles1 + j) * x.P;
        for (uint32_t r = threadIdx.x; r < Bm; r += kChainNT) {
            const uint32_t q = sv[r];
            Gn[r] = q < Ba ? G[q] : (kAbs | (x.P + t0 + (q - Ba)));
        }
        __syncthreads();
        uint32_t *t = G; G = Gn; Gn = t;
        Bend = Bm;
    }
    uint32_t *cc = ch.CC + ((size_t)rl * ch.nch + c) * x.P;
    for (uint32_t r = threadIdx.x; r < Bend; r += kChainNT) cc[r] = G[r];
}

// The chunks' A as a parallel prefix instead of k_v2x_link's serial walk (one decoded sequence
// per call since round 5: the walk over ~500 chunks on one workgroup took 0.82 ms at C2).
// P_c maps the alive set at the END of chunk c to the alive set at the start of chunk
// c - 2^k + 1 (entries: a frame index, or kAbs | an absolute insertion number); a level doubles
// the span: P'_c[r] = P_c[r] if absolute, else P_{c-2^k}[P_c[r]] (c >= 2^k).  After
// ceil(log2 nch) levels P_c reaches chunk 0's start, whose alive set is the identity (A_0[r] = r),
// so A at chunk c + 1's start is P_c with the flag cleared (k_v2x_link_fin).
__global__ __launch_bounds__(kChainNT) void k_v2x_link_lvl(V2xGeo x, V2xChain ch, uint32_t span,
                                                            const uint32_t *__restrict__ src,
                                                            uint32_t *__restrict__ dst) {
    const uint32_t c = blockIdx.x;
    const uint32_t j1 = (c + 1) * ch.tpc < x.tiles1 ? (c + 1) * ch.tpc : x.tiles1;
    const uint32_t te = j1 * (uint32_t)kTile < x.ns ? j1 * (uint32_t)kTile : x.ns;
    const uint32_t Bm = alive_at(x.P, x.T, te);
    const uint32_t *pc = src + (size_t)c * x.P;
    uint32_t *dc = dst + (size_t)c * x.P;
    if (c < span) {
        for (uint32_t r = threadIdx.x; r < Bm; r += kChainNT) dc[r] = pc[r];
        return;
    }
    const uint32_t *pp = src + (size_t)(c - span) * x.P;
    for (uint32_t r = threadIdx.x; r < Bm; r += kChainNT) {
        const uint32_t v = pc[r];
        dc[r] = (v & kAbs) ? v : pp[v];
    }
}

__global__ __launch_bounds__(kChainNT) void k_v2x_link_fin(V2xGeo x, V2xChain ch, const uint32_t *__restrict__ pref) {
    const uint32_t c = blockIdx.x;   // A at chunk c's start
    const uint32_t Ba = alive_at(x.P, x.T, c * ch.tpc * (uint32_t)kTile);
    uint32_t *aa = ch.AA + (size_t)c * x.P;
    const uint32_t *pc = pref + (size_t)(c ? c - 1 : 0) * x.P;
    for (uint32_t r = threadIdx.x; r < Ba; r += kChainNT) aa[r] = c ? (pc[r] & ~kAbs) : r;
}

// Software-pipelined over the chunk's tiles: a thread's answers and survivor entries of tile
// j + 1 are loaded (kChainPer of each) while tile j's ids are computed and stored, and tile
// j + 1's pool2 gathers are issued as soon as its alive set is in LDS, one iteration ahead of
// its stores (they land while the next alive set is built).
constexpr int kChainPer = kTile / kChainNT;
static_assert(kChainPer * kChainNT == kTile, "a tile's steps and survivors: kChainPer per thread");

// The decoded sequence is every rank's (the draws depend on the epoch and the window only,
// V2:108,147): block (chunk c, group) writes the ids of ranks [group * kFanRanks, ...) of the call
// -- or, with VV, the virtual indices alone (4 bytes a step), which k_v2x_fanout turns into every
// rank's ids as a one-shot grid (more than one rank: this kernel's ~500 long-running workgroups
// store at about half the rate of a one-shot grid).
__global__ __launch_bounds__(kChainNT) void k_v2x_emit(Geometry g, V2xGeo x, V2xChain ch,
                                                       const RankDesc *__restrict__ ranks, int32_t rank_lo,
                                                       int32_t nout, const uint32_t *__restrict__ ANS,
                                                       const uint32_t *__restrict__ Q2, int64_t pos_lo,
                                                       int64_t count, int64_t *__restrict__ out, MapArgs ma,
                                                       uint32_t *__restrict__ VV) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    uint32_t *A = smem, *An = smem + x.P;
    const uint32_t rl = 0, c = blockIdx.x % ch.nch;
    const int32_t r_a = (int32_t)(blockIdx.x / ch.nch) * kFanRanks;
    const int32_t r_b = r_a + kFanRanks < nout ? r_a + kFanRanks : nout;
    const uint32_t j0 = c * ch.tpc, j1 = j0 + ch.tpc < x.tiles1 ? j0 + ch.tpc : x.tiles1;
    const int64_t pos_hi = pos_lo + count;
    if ((int64_t)j0 * kTile >= pos_hi) return;   // every step of the chunk past the range
    const uint32_t Ba0 = alive_at(x.P, x.T, j0 * (uint32_t)kTile);
    const uint32_t *aa = ch.AA + ((size_t)rl * ch.nch + c) * x.P;
    for (uint32_t r = threadIdx.x; r < Ba0; r += kChainNT) A[r] = aa[r];
    const uint32_t *ans = ANS + (size_t)rl * x.ns;
    const uint32_t *q2 = Q2 + (size_t)rl * x.T2;
    // tile j's answers (q) and survivors (sr) of this thread: u = threadIdx.x + k * kChainNT
    auto load = [&](uint32_t j, uint32_t (&q)[kChainPer], uint32_t (&sr)[kChainPer]) {
        const uint32_t t0 = j * (uint32_t)kTile, n = x.ns - t0 < (uint32_t)kTile ? x.ns - t0 : (uint32_t)kTile;
        const uint32_t Bm = alive_at(x.P, x.T, t0 + n);
        const uint32_t *sv = ch.SV + ((size_t)rl * x.tiles1 + j) * x.P;
#pragma unroll
        for (int k = 0; k < kChainPer; k++) {
            const uint32_t u = threadIdx.x + (uint32_t)k * kChainNT;
            q[k] = u < n ? ans[t0 + u] : 0u;
            sr[k] = u < Bm ? sv[u] : 0u;
        }
    };
    uint32_t q[kChainPer], sr[kChainPer], qn[kChainPer], srn[kChainPer];
    // tile j's insertion numbers (av) and, for elements moved over from pool2, their pool2 ranks
    // (g2), gathered one iteration ahead of the stores that need them
    uint32_t av[kChainPer], g2[kChainPer];
    auto prep = [&](uint32_t j, const uint32_t (&qq)[kChainPer]) {
        const uint32_t t0 = j * (uint32_t)kTile, n = x.ns - t0 < (uint32_t)kTile ? x.ns - t0 : (uint32_t)kTile;
        const uint32_t Ba = alive_at(x.P, x.T, t0);
#pragma unroll
        for (int k = 0; k < kChainPer; k++) {
            const uint32_t u = threadIdx.x + (uint32_t)k * kChainNT;
            const uint32_t a = u < n ? (qq[k] < Ba ? A[qq[k]] : x.P + t0 + (qq[k] - Ba)) : 0u;
            av[k] = a;
            g2[k] = (u < n && a >= x.P) ? q2[a - x.P] : 0u;
        }
    };
    load(j0, q, sr);
    __syncthreads();
    prep(j0, q);
    for (uint32_t j = j0; j < j1; j++) {
        const uint32_t t0 = j * (uint32_t)kTile, n = x.ns - t0 < (uint32_t)kTile ? x.ns - t0 : (uint32_t)kTile;
        if ((int64_t)t0 >= pos_hi) break;
        const bool more = j + 1 < j1;
        if (more) load(j + 1, qn, srn);
        const uint32_t Ba = alive_at(x.P, x.T, t0), Bm = alive_at(x.P, x.T, t0 + n);
        if (more) {   // the elements alive at tile j + 1's start (A is tile j's)
#pragma unroll
            for (int k = 0; k < kChainPer; k++) {
                const uint32_t r = threadIdx.x + (uint32_t)k * kChainNT;
                if (r < Bm) An[r] = sr[k] < Ba ? A[sr[k]] : x.P + t0 + (sr[k] - Ba);
            }
        }
        // tile j's ids: insertion number a < P is initial pool1 (V2:135-136), else the element
        // step a - P moved over from pool2
#pragma unroll
        for (int k = 0; k < kChainPer; k++) {
            const uint32_t u = threadIdx.x + (uint32_t)k * kChainNT;
            const int64_t t = (int64_t)t0 + u;
            if (u >= n || t < pos_lo || t >= pos_hi) continue;
            const uint32_t a = av[k];
            // virtual index: a < P the initial pool1 position, else the element's window base +
            // its pool2 rank (window 0 is the old start's second window, V2:135-138)
            bool old_side;
            int64_t v;
            if (a < x.P) {
                v = a;
                old_side = true;
            } else {
                const uint32_t sw = (a - x.P) / x.B;
                v = (int64_t)(sw + 1) * x.B + g2[k];
                old_side = sw == 0;
            }
            if (VV) {
                VV[t] = (uint32_t)v;
                continue;
            }
            for (int32_t r = r_a; r < r_b; r++) {   // (wave-uniform rank: scalar descriptor loads)
                const RankDesc rd = ranks[rank_lo + r];
                put_id_or_pair(out, ma, (int64_t)r * count + (t - pos_lo),
                               wrap_id((old_side ? rd.old_start : rd.new_start) + v, g.N));
            }
        }
        if (more) {
            __syncthreads();
            uint32_t *tp = A; A = An; An = tp;
#pragma unroll
            for (int k = 0; k < kChainPer; k++) { q[k] = qn[k]; sr[k] = srn[k]; }
            prep(j + 1, q);
        }
    }
}

static int64_t v2x_cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }
static int64_t pos_hi_of(const Geometry &g, int64_t pos_lo, int64_t count) {
    return pos_lo + count < g.ns ? pos_lo + count : g.ns;
}

static void v2x_launch_fanout(const Geometry &g, const RankDesc *ranks, int32_t rank_lo, int32_t nout,
                              const uint32_t *VV, int64_t pos_lo, int64_t count, int64_t *out,
                              const MapArgs &ma, hipStream_t s) {
    const int64_t n = pos_hi_of(g, pos_lo, count) - pos_lo;
    const uint32_t blocks = (uint32_t)v2x_cdiv(n, 1024);   // (n < 2^31: v2_exact_supported)
    const int32_t per_row = nout > kFanoutManyRanks ? 1 : kFanoutRanksFew;
    const uint32_t rows = (uint32_t)v2x_cdiv(nout, per_row);
    if (blocks && rows)
        hipLaunchKernelGGL(k_v2x_fanout, dim3(blocks, rows), dim3(256), 0, s, g, ranks, rank_lo, nout, per_row, VV,
                           pos_lo, count, out, ma);
}

static V2xGeo v2x_geo(const Geometry &g) {
    V2xGeo x{};
    const int64_t P = g.B < g.ns ? g.B : g.ns;
    x.P = (uint32_t)P;
    x.T = (uint32_t)(g.ns - P);
    x.B = (uint32_t)g.B;
    x.S = x.T ? (uint32_t)v2x_cdiv(x.T, g.B) : 0u;
    x.ns = (uint32_t)g.ns;
    x.tiles1 = (uint32_t)v2x_cdiv(g.ns, kTile);
    x.T2 = x.S * x.B;
    return x;
}

// pool2 windows of B steps as sequences of their own: B alive, no insertions
static V2xGeo v2x_window_geo(const V2xGeo &x) {
    V2xGeo w{};
    w.P = x.B; w.T = 0; w.S = 0; w.B = x.B; w.ns = x.B; w.T2 = 0;
    w.tiles1 = (uint32_t)v2x_cdiv(x.B, kTile);
    return w;
}


static size_t v2x_split_words(const V2xGeo &x, int32_t nr) {
    size_t t = (size_t)nr * (size_t)v2x_cdiv(x.ns, kGTile);
    if (x.B > (uint32_t)kTile) {
        const size_t tw = (size_t)nr * x.S * (size_t)v2x_cdiv(x.B, kGTile);
        t = t > tw ? t : tw;
    }
    return 2 * t + 64;
}

bool v2_exact_supported(const Geometry &g) {
    return g.ns < ((int64_t)1 << 31) && g.B < ((int64_t)1 << 30);
}

// Ranks decoded per pass: every flat kernel of the decode launches one thread per (rank, step)
// and the draw / tile launches one block per (rank, job), so a pass keeps ranks x steps below
// 2^30 (thread counts below 2^32) and the workspace is sized for one pass, reused by the next.

// launches of one block per job, cut into pieces of at most 2^20 blocks (2^30 threads)
template <class F>
static void v2x_launch_blocks(uint64_t blocks, F &&launch) {
    constexpr uint64_t kMaxBlocks = (uint64_t)1 << 20;
    for (uint64_t b0 = 0; b0 < blocks; b0 += kMaxBlocks)
        launch(b0, (uint32_t)(blocks - b0 < kMaxBlocks ? blocks - b0 : kMaxBlocks));
}

// a workgroup per pool2 window's MT stream when the windows are long and few: fewer streams
// than 4 per CU (PSS_V2X_DRAWS_WG=0 / 1 forces the wave / workgroup form)
static bool v2x_draws_wg(uint64_t streams, uint32_t B) {
    static const int env = [] {
        const char *e = getenv("PSS_V2X_DRAWS_WG");
        return e ? atoi(e) : -1;
    }();
    if (env == 0 || env == 1) return env == 1;
    return B > (uint32_t)kTile && streams < 1024;
}

// chain mode: pools of at most kTile entries (one decode tile's frame holds the whole pool)
static bool v2x_chain(const V2xGeo &x) { return x.P <= (uint32_t)kTile; }

// chunks of tiles per rank: about two 1024-thread workgroups per CU over the pass's ranks
static V2xChain v2x_chain_plan(const V2xGeo &x, int32_t nr) {
    V2xChain ch{};
#ifndef PSS_CHAIN_CHUNKS
#define PSS_CHAIN_CHUNKS 512
#endif
    uint32_t want = (uint32_t)((PSS_CHAIN_CHUNKS + nr - 1) / (nr > 0 ? nr : 1));
    if (want < 1) want = 1;
    if (want > x.tiles1) want = x.tiles1;
    ch.tpc = (x.tiles1 + want - 1) / want;
    ch.nch = (x.tiles1 + ch.tpc - 1) / ch.tpc;
    return ch;
}

// The workspace of a call: the decode's arrays, then a draw slot -- the epoch's draws K1 (ns
// words), K2 (T2 words) and the windows' seeded MT states ST (S x 624, the one-wave draw form).
// A slot depends on the epoch and (ns, B) only, so the runtime can fill slots of coming epochs
// ahead of their calls (pss_runtime.cpp, exact lookahead) and hand one to launch_v2_exact.
// (rounded up to 4 words: the slot that follows in the workspace -- whose K1 doubles as VV, read
// by 16-byte loads in k_v2x_fanout -- starts 16-byte aligned)
static size_t v2x_rest_words(const V2xGeo &x) {
    const int32_t nr = 1;   // one decoded sequence serves every rank of a call (v2x_pass)
    size_t w;
    if (v2x_chain(x)) {   // ANS (ns), Q2 (T2), survivors, chunk maps, chunk starts
        const V2xChain ch = v2x_chain_plan(x, nr);
        w = (size_t)x.ns + (size_t)x.T2 + (size_t)x.tiles1 * x.P + (size_t)3 * ch.nch * x.P;
    } else {
        // V, O, Vd, Od (ns each), Q2 (T2), tile splits.  Windows beyond kTile are decoded in V, O,
        // Vd, Od (S * B <= ns).
        w = (size_t)4 * x.ns + (size_t)x.T2 + v2x_split_words(x, nr);
    }
    return (w + 3u) & ~(size_t)3u;
}
static size_t v2x_slot_words(const V2xGeo &x) { return (size_t)x.ns + (size_t)x.T2 + (size_t)x.S * kMtN; }

size_t v2_exact_ws_bytes(const Geometry &g, int32_t nr_all) {
    if (!v2_exact_supported(g) || nr_all <= 0) return 0;
    const V2xGeo x = v2x_geo(g);
    return (v2x_rest_words(x) + v2x_slot_words(x)) * sizeof(uint32_t);
}

size_t v2_exact_slot_bytes(const Geometry &g) {
    if (!v2_exact_supported(g)) return 0;
    return v2x_slot_words(v2x_geo(g)) * sizeof(uint32_t);
}

// the draws of one epoch into a slot: the pool2 windows' k1 / k2 (seeded ahead, then one wave or
// one workgroup per window) and the tail's first draws
static void v2x_draws(const V2xGeo &x, int64_t epoch, uint32_t *slot, hipStream_t s) {
    const uint32_t nr = 1;
    uint32_t *K1 = slot, *K2 = slot + x.ns, *ST = K2 + x.T2;
    const uint32_t tail_blocks = (x.P + 63u) / 64u;
    if (x.S) {
        // few long windows (the streams alone do not fill the chip): a workgroup per stream, the
        // tail draws riding along on the idle CUs
        const bool wg = v2x_draws_wg((uint64_t)x.S * (uint64_t)nr, x.B);
        const uint64_t wblocks = (uint64_t)x.S * (uint64_t)nr;
        const uint64_t tblocks = wg ? ((uint64_t)tail_blocks * (uint64_t)nr + kMtWgWaves - 1) / kMtWgWaves : 0u;
        if (!wg)   // (nr = 1: one decoded sequence; S < 2^31 / B windows, tail_blocks <= 2^24)
            hipLaunchKernelGGL(k_v2x_seed, dim3(mt_seed_blocks(x.S) + tail_blocks), dim3(64), 0, s,
                               MtSeedSpec{epoch, 0, -1, 2, x.S}, ST, x, epoch, K1);
        v2x_launch_blocks(wblocks + tblocks, [&](uint64_t b0, uint32_t nb) {
            if (wg) hipLaunchKernelGGL(k_v2x_draws_wg, dim3(nb), dim3(kMtWgThreads), 0, s, x, epoch, x.S, b0,
                                       nr, tail_blocks, K1, K2);
            else hipLaunchKernelGGL(k_v2x_draws, dim3(nb), dim3(64), 0, s, x, x.S, b0, (const uint32_t *)ST, K1, K2);
        });
    } else {
        v2x_launch_blocks((uint64_t)tail_blocks * (uint64_t)nr, [&](uint64_t b0, uint32_t nb) {
            hipLaunchKernelGGL(k_v2x_tail_draws, dim3(nb), dim3(64), 0, s, x, epoch, tail_blocks, b0, K1);
        });
    }
}

// PSS_EXACT_SPLIT=0 / 1: the exact orders' long-window draws in the workgroup form / in the split
// form (pss_v2split.h) for any window length the scratch holds; by default the split form where
// the workgroup form would run (few long windows), the windows hold at least kSpMinWindow entries
// and the plan covers most of a window.  (Cold epochs at C2's files, same box: V2 B = 2^14 / 2^16
// even, 2^18 3.33 against 5.02 ms; V1 2^14 1.42 / 1.56, 2^16 1.58 / 1.36, 2^18 1.75 / 1.95 --
// profiles/r06/exact_split/pool_size_probe_*.txt.)
constexpr uint32_t kSpMinWindow = 1u << 17;
static int sp_env() {
    static const int env = [] {
        const char *e = getenv("PSS_EXACT_SPLIT");
        return e ? atoi(e) : -1;
    }();
    return env;
}

// Scratch layout and the launches of the split draws for a.S streams (windows): hb the plan of
// windows 0 .. S-2, hl of the last one; x carries the V2 tail (V1: none).  false when the scratch
// cannot hold it.
template <bool kV1>
static bool sp_launch(V2xSp a, const SpPlanHost *hb, const SpPlanHost *hl, const V2xGeo &x, int64_t epoch,
                      uint32_t *scratch, size_t scratch_words, hipStream_t s) {
    if (!scratch) return false;
    a.pl[0] = sp_plan_dev(*hb);
    a.pl[1] = sp_plan_dev(*hl);
    const size_t nseg = std::max(hb->seg.size(), hl->seg.size());
    a.nsegmax = (uint32_t)nseg;
    const size_t nwp = ((size_t)std::max(hb->nt, hl->nt) * kMtN + 3u) & ~(size_t)3u;
    a.nwp = (uint32_t)nwp;
    const size_t w_words = (size_t)a.S * nwp, w_rec = (size_t)a.S * nseg * kSpRec * 2u;
    const size_t w_ss = (size_t)a.S * nseg * 2u, w_anc = (size_t)a.S * (kSpPh + 1) * 4u;
    if (w_words + w_rec + w_ss + w_anc > scratch_words || nwp >= ((size_t)1 << 32)) return false;
    a.words = scratch;
    a.rec = reinterpret_cast<uint2 *>(scratch + w_words);
    a.ss = reinterpret_cast<uint2 *>(scratch + w_words + w_rec);
    a.anc = scratch + w_words + w_rec + w_ss;
    const uint32_t tail_blocks = kV1 ? 0u : (x.P + 63u) / 64u, tail_wg = (tail_blocks + 3u) / 4u;
    const uint32_t nph = std::max(std::max(hb->nph, 1u), std::max(hl->nph, 1u));
    // the twists phase p needs: up to its last segment's end, all of them for a window's last
    // phase (its walk runs the remainder)
    uint32_t need[kSpPh] = {};
    for (uint32_t p = 0; p < nph; p++)
        for (const SpPlanHost *h : {hb, hl}) {
            uint32_t n = h->nt;
            if (p + 1u < std::max(h->nph, 1u)) {
                const uint4 sg = h->seg[h->ph[p + 1] - 1u];
                n = std::min(h->nt, (sg.x + sg.y + (uint32_t)kMtN - 1u) / (uint32_t)kMtN);
            }
            need[p] = std::max(need[p], n);
        }
    for (uint32_t p = 1; p < nph; p++) need[p] = std::max(need[p], need[p - 1]);
#ifdef PSS_DIAG_SP_TAIL_APART   // timing build: the generator alone on the caller's stream, then the tail
    SpSide *side = nullptr;
    hipLaunchKernelGGL(k_v2x_sp_gen<kV1>, dim3(a.S), dim3(kSpGenThreads), 0, s, a, x, epoch, 0u, need[nph - 1]);
    if (tail_blocks)
        hipLaunchKernelGGL(k_v2x_tail_draws, dim3(tail_blocks), dim3(64), 0, s, x, epoch, tail_blocks, (uint64_t)0, a.K1);
    const bool gen_done = true;
#else
    SpSide *side = sp_side();
    const bool gen_done = false;
#endif
    std::unique_lock<std::mutex> lk;
    if (side) {   // generator chunks on the side stream, each phase waits for the words it reads
        lk = std::unique_lock<std::mutex>(side->mu);
        (void)hipEventRecord(side->start, s);   // (the scratch is the previous call's decode arrays)
        (void)hipStreamWaitEvent(side->g, side->start, 0);
        uint32_t t = 0;
        for (uint32_t p = 0; p < nph; p++) {
            if (need[p] > t || p == 0) {
                hipLaunchKernelGGL(k_v2x_sp_gen<kV1>, dim3(a.S + (t == 0 ? tail_wg : 0u)), dim3(kSpGenThreads), 0,
                                   side->g, a, x, epoch, t, need[p]);
                t = need[p];
            }
            (void)hipEventRecord(side->ev[p], side->g);
        }
    } else if (!gen_done) {
        hipLaunchKernelGGL(k_v2x_sp_gen<kV1>, dim3(a.S + tail_wg), dim3(kSpGenThreads), 0, s, a, x, epoch, 0u,
                           need[nph - 1]);
    }
    for (uint32_t p = 0; p < nph; p++) {
        uint32_t segs = 0;
        for (const SpPlanHost *h : {hb, hl})
            if (p < h->nph) segs = std::max(segs, h->ph[p + 1] - h->ph[p]);
        if (side) (void)hipStreamWaitEvent(s, side->ev[p], 0);
        const uint32_t items = kV1 ? segs : 2u * segs;   // (V1: one role)
        if (segs) hipLaunchKernelGGL(k_v2x_sp_lvl1<kV1>, dim3((items + 3u) / 4u, a.S), dim3(256), 0, s, a, p);
        hipLaunchKernelGGL(k_v2x_sp_walk<kV1>, dim3(a.S), dim3(64), 0, s, a, p);
    }
    if (nseg) hipLaunchKernelGGL(k_v2x_sp_emit<kV1>, dim3((uint32_t)((nseg + 3u) / 4u), a.S), dim3(256), 0, s, a);
    if (kV1)
        hipLaunchKernelGGL(k_v1x_sp_count, dim3((uint32_t)((std::max(hb->W, hl->W) + kSpCountPer - 1u) / kSpCountPer), a.S),
                           dim3(256), 0, s, a);
    return true;
}

// The draws of a call that brings no slot, for long windows (pss_v2split.h): the windows' words
// generated beside the tail draws, then the segments' pieces, the walk and the emission spread
// over the chip, phase by phase.  Its scratch is the decode's arrays (free until the tiles run);
// false (the workgroup form runs instead) when the geometry or the scratch does not suit it.
static bool v2x_draws_split(const V2xGeo &x, int64_t epoch, uint32_t *slot, uint32_t *scratch,
                            size_t scratch_words, hipStream_t s) {
    const int env = sp_env();
    if (env == 0 || !x.S) return false;
    if (env != 1 && (!v2x_draws_wg((uint64_t)x.S, x.B) || x.B < kSpMinWindow)) return false;
    const uint32_t Wl = x.T - (x.S - 1u) * x.B;
    const SpPlanHost *hl = sp_plan_get(Wl, x.P, false);
    const SpPlanHost *hb = x.S > 1 ? sp_plan_get(x.B, x.P, false) : hl;
    if (!hl || !hb) return false;
    // worth it where most of a full window's words fall in phases
    if (env != 1 && (double)hb->qend < 0.5 * hb->words) return false;
    V2xSp a{};
    a.S = x.S; a.B = x.B; a.P = x.P;
    a.kb1 = 32u - (uint32_t)__builtin_clz(x.P);
    a.K1 = slot;
    a.K2 = slot + x.ns;
    return sp_launch<false>(a, hb, hl, x, epoch, scratch, scratch_words, s);
}

// V1 (pss_v1exact.hip v1x_big_draws): the draws of nj windows from w_lo (full ones of n_full
// entries, the last of n_last) into J[job][B] and the bucket counts BCNT[job][nbk] (zeroed by the
// caller), with the scratch given (null: none -- the draws made ahead into a slot); false: the
// workgroup form runs instead
bool v1x_draws_split(int64_t w_lo, uint32_t nj, uint32_t n_full, uint32_t n_last, uint32_t B, uint32_t nbk,
                     int64_t epoch, uint32_t *J, uint32_t *BCNT, uint32_t *scratch, size_t scratch_words,
                     bool wg_form, hipStream_t s) {
    const int env = sp_env();
    if (env == 0 || !nj || !scratch || n_full < 2) return false;
    if (env != 1 && (!wg_form || n_full < kSpMinWindow)) return false;
    const SpPlanHost *hl = sp_plan_get(n_last, 0u, true);
    const SpPlanHost *hb = nj > 1 ? sp_plan_get(n_full, 0u, true) : hl;
    if (!hl || !hb) return false;
    if (env != 1 && (double)hb->qend < 0.5 * hb->words) return false;
    V2xSp a{};
    a.S = nj; a.B = B; a.P = 0u; a.kb1 = 1u;
    a.K1 = J;
    a.K2 = BCNT;
    a.w0 = w_lo;
    a.nbk = nbk;
    const V2xGeo x{};   // (no tail)
    return sp_launch<true>(a, hb, hl, x, epoch, scratch, scratch_words, s);
}

// epochs drawn ahead: the few long windows of the workgroup form keep ~S CUs busy for
// milliseconds, so several epochs' draws run side by side (8: C5 V2 exact 10.9 -> 3.4 ms per
// epoch); the one-wave form already fills the chip, and drawn ahead beside the decode it slowed
// C2 from 0.83 to 1.19 ms (profiles/r05/ab_exact_tile.txt §7): none.  At most 4 GiB of slots.
int v2_exact_lookahead_depth(const Geometry &g) {
    if (!v2_exact_supported(g)) return 0;
    const V2xGeo x = v2x_geo(g);
    const int want = x.S && v2x_draws_wg((uint64_t)x.S, x.B) ? 8 : 0;
    const size_t sb = v2x_slot_words(x) * sizeof(uint32_t);
    const size_t cap = ((size_t)4 << 30) / (sb ? sb : 1);
    return cap < (size_t)want ? (int)cap : want;
}

hipError_t launch_v2_exact_draws(const Geometry &g, int64_t epoch, uint32_t *slot, hipStream_t s) {
    if (!v2_exact_supported(g) || !slot) return hipErrorInvalidValue;
    v2x_draws(v2x_geo(g), epoch, slot, s);
    return hipGetLastError();
}

// global merge levels w = kTile, 2 kTile, ... of nr sequences of x.ns > kTile steps (V, O sorted
// per block of w on entry); the last level writes what `fin_mode` asks (k_v2x_gmerge's FIN)
static void v2x_global_levels(const V2xGeo &x, uint32_t nr, uint32_t *V, uint32_t *O, uint32_t *Vd,
                              uint32_t *Od, uint32_t *SP, int fin_mode, const V2xFin &fin, hipStream_t s) {
    const int64_t tiles = (int64_t)nr * v2x_cdiv(x.ns, kGTile);
    const dim3 gridt((uint32_t)tiles), grids((uint32_t)v2x_cdiv(2 * tiles, 256));
    for (uint32_t w = kTile; w < x.ns; w <<= 1) {   // each level: fused map-and-merge
        hipLaunchKernelGGL(k_v2x_gsplit, grids, dim3(256), 0, s, x, nr, w, V, SP);
        const bool last = (uint64_t)2 * w >= x.ns;
        if (!last) hipLaunchKernelGGL(k_v2x_gmerge<0>, gridt, dim3(kGNT), 0, s, x, w, V, O, Vd, Od, SP, fin);
        else if (fin_mode == 1) hipLaunchKernelGGL(k_v2x_gmerge<1>, gridt, dim3(kGNT), 0, s, x, w, V, O, Vd, Od, SP, fin);
        else hipLaunchKernelGGL(k_v2x_gmerge<2>, gridt, dim3(kGNT), 0, s, x, w, V, O, Vd, Od, SP, fin);
        uint32_t *t = V; V = Vd; Vd = t;
        t = O; O = Od; Od = t;
    }
}

// The draws of every pool2 window and of the tail come from streams seeded by the epoch and the
// window alone (seed(e + 2) for segment 0, seed(e + (s - 1) 10000), seed(e + buffers 10000) per
// tail step, V2:107-109,147) and the pool sizes are the same for every rank (ns = ceil(N / R)),
// so the decoded stream of virtual indices is the same for all of them; a rank's ids are that
// stream through its (old, new) start (V2:135-148).  One pass decodes it once and its last stage
// writes the ids of all nr ranks of the call.  slot: the epoch's draws (v2x_draws), already made
// when the call brings one, else made here into the workspace's own slot.
static hipError_t v2x_pass(const Geometry &g, const V2xGeo &x, const RankDesc *ranks, int32_t rank_lo,
                           int32_t nout, int64_t pos_lo, int64_t count, int64_t epoch,
                           int64_t *out, uint32_t *ws, uint32_t *slot, hipStream_t s, const MapArgs &ma) {
    const int32_t nr = 1, nr_plan = 1;   // decoded sequences
    const uint32_t ngrp = (uint32_t)v2x_cdiv(nout, kFanRanks);   // output block rows
    const size_t nsr = (size_t)nr * x.ns, tr = (size_t)nr * x.T2;
    // merge-levels layout: V | O | Vd | Od | Q2 | splits, then the slot K1 | K2 | ST
    // chain layout:        V (answers) | Q2 | survivors | chunk maps | chunk starts, then the slot
    const bool chain = v2x_chain(x);
    if (!slot) {
        const size_t rest = v2x_rest_words(x);
        slot = ws + rest;
        // the decode's arrays are free until the tiles run: the split draws' scratch
        if (!v2x_draws_split(x, epoch, slot, ws, rest, s)) v2x_draws(x, epoch, slot, s);
    }
    uint32_t *K1 = slot, *K2 = slot + x.ns;
    uint32_t *V = ws;
    uint32_t *O = chain ? nullptr : V + nsr, *Vd = chain ? nullptr : O + nsr, *Od = chain ? nullptr : Vd + nsr;
    uint32_t *Q2 = chain ? V + nsr : Od + nsr;
    const uint32_t nru = (uint32_t)nr;
    const bool narrow = v2x_narrow(x.P, x.B);
    // one decode-tile launch of nb blocks from block b0 (the entry width; kTileOut merge outputs
    // per thread -- 4 and 16 measured slower, 6.46 / 5.9 against 5.1-5.2 ms at C2, round 3)
    auto tile = [&](uint64_t b0, uint32_t nb, const V2xGeo &xg, uint32_t per, const uint32_t *k1,
                    const uint32_t *k2, uint32_t *v, uint32_t *o, uint32_t *q2, uint32_t *sv, size_t lds) {
        if (narrow)
            hipLaunchKernelGGL((k_v2x_tile<uint32_t, kTileOut>), dim3(nb), dim3(kTile / kTileOut), lds, s, xg, per, b0, k1, k2, v, o, q2, sv);
        else
            hipLaunchKernelGGL((k_v2x_tile<uint64_t, kTileOut>), dim3(nb), dim3(kTile / kTileOut), lds, s, xg, per, b0, k1, k2, v, o, q2, sv);
    };
    const size_t kTileLds0 = narrow ? 2 * TileEntry<uint32_t>::kSlots * sizeof(uint32_t)
                                    : 2 * TileEntry<uint64_t>::kSlots * sizeof(uint64_t);
    if (chain) {
        uint32_t *ANS = V;
        V2xChain ch = v2x_chain_plan(x, nr_plan);   // the workspace's plan (a last pass may be short)
        ch.SV = Q2 + tr;
        ch.CC = ch.SV + (size_t)nr * x.tiles1 * x.P;
        ch.AA = ch.CC + (size_t)nr * ch.nch * x.P;
        ch.PP = ch.AA + (size_t)nr * ch.nch * x.P;
        const uint32_t per_rank = x.tiles1 + x.S;
        v2x_launch_blocks((uint64_t)per_rank * nru, [&](uint64_t b0, uint32_t nb) {
            tile(b0, nb, x, per_rank, K1, K2, ANS, (uint32_t *)nullptr, Q2, ch.SV, kTileLds0);
        });
        const size_t lds = 2 * (size_t)x.P * sizeof(uint32_t);
        hipLaunchKernelGGL(k_v2x_compose, dim3(nru * ch.nch), dim3(kChainNT), lds, s, x, ch);
        {   // the chunks' A: log2(nch) prefix levels between CC and the spare buffer PP
            uint32_t *src = ch.CC, *dst = ch.PP;
            for (uint32_t span = 1; span < ch.nch; span <<= 1) {
                hipLaunchKernelGGL(k_v2x_link_lvl, dim3(ch.nch), dim3(kChainNT), 0, s, x, ch, span,
                                   (const uint32_t *)src, dst);
                uint32_t *t = src; src = dst; dst = t;
            }
            hipLaunchKernelGGL(k_v2x_link_fin, dim3(ch.nch), dim3(kChainNT), 0, s, x, ch, (const uint32_t *)src);
        }
        // K1 (the draws) is free once the tiles ran: the virtual indices for the fan-out
#ifndef PSS_CHAIN_FAN
#define PSS_CHAIN_FAN 1
#endif
        const bool fan = PSS_CHAIN_FAN && nout > 1;
        hipLaunchKernelGGL(k_v2x_emit, dim3((fan ? 1u : ngrp) * ch.nch), dim3(kChainNT), lds, s, g, x, ch, ranks,
                           rank_lo, nout, ANS, (const uint32_t *)Q2, pos_lo, count, out, ma, fan ? K1 : nullptr);
        if (fan) v2x_launch_fanout(g, ranks, rank_lo, nout, K1, pos_lo, count, out, ma, s);
        return hipGetLastError();
    }
    uint32_t *SP = Q2 + tr;                    // merge-path splits: 2 words per tile
    const bool big_windows = x.B > (uint32_t)kTile && x.S > 0;
    const size_t kTileLds = kTileLds0;
    if (big_windows) {          // pool2 windows first, as nr * S sequences of B steps
        const V2xGeo xw = v2x_window_geo(x);
        const uint32_t nseq = nru * x.S;
        v2x_launch_blocks((uint64_t)xw.tiles1 * nseq, [&](uint64_t b0, uint32_t nb) {
            tile(b0, nb, xw, xw.tiles1, K2, K2, V, O, Q2, (uint32_t *)nullptr, kTileLds);
        });
        V2xFin fw{};
        fw.Q2 = Q2;   // [seq][B] == [rank][T2] (T2 = S * B)
        v2x_global_levels(xw, nseq, V, O, Vd, Od, SP, 1, fw, s);
    }
    // pool1 tiles (and, for B <= kTile, the windows in the same launch)
    const uint32_t per_rank = x.tiles1 + (big_windows ? 0u : x.S);
    v2x_launch_blocks((uint64_t)per_rank * nru, [&](uint64_t b0, uint32_t nb) {
        tile(b0, nb, x, per_rank, K1, K2, V, O, Q2, (uint32_t *)nullptr, kTileLds);
    });
    V2xFin f{};
    f.g = g; f.ranks = ranks; f.rank_lo = rank_lo; f.nout = nout; f.Q2 = Q2;
    f.pos_lo = pos_lo; f.count = count; f.out = out; f.ma = ma;
    // the last level's virtual indices go to a spare list buffer: O and Od alternate as the
    // levels' step lists, V / Vd as their positions; the last level reads one pair and writes
    // neither, and K1 (the draws, consumed by the pool1 tiles) is free by then
    f.VV = K1;
    v2x_global_levels(x, nru, V, O, Vd, Od, SP, 2, f, s);
    v2x_launch_fanout(g, ranks, rank_lo, nout, K1, pos_lo, count, out, ma, s);
    return hipGetLastError();
}

hipError_t launch_v2_exact(const Geometry &g, const RankDesc *ranks, int32_t rank_lo, int32_t nr,
                           int64_t pos_lo, int64_t count, int64_t epoch, int64_t *out, uint32_t *ws,
                           hipStream_t s, const MapArgs *mapped, uint32_t *slot) {
    const int64_t pos_hi = pos_lo + count < g.ns ? pos_lo + count : g.ns;
    if (nr <= 0 || pos_hi <= pos_lo) return hipSuccess;
    if (!v2_exact_supported(g) || !ws) return hipErrorInvalidValue;
    const V2xGeo x = v2x_geo(g);
    static const hipError_t attr = [] {
        const int lds = 2 * (int)TileEntry<uint64_t>::kSlots * (int)sizeof(uint64_t);
        return hipFuncSetAttribute((const void *)k_v2x_tile<uint64_t, kTileOut>,
                                   hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    }();
    if (attr != hipSuccess) return attr;
    const MapArgs ma = mapped ? *mapped : MapArgs{};
    return v2x_pass(g, x, ranks, rank_lo, nr, pos_lo, count, epoch, out, ws, slot, s, ma);
}

}  // namespace pss
