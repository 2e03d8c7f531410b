// pss_v2grp.hip -- V2 pools beyond LDS (P1 > kLdsSlotMax): the grouped slot machine
// (reference semantics V2:96-116 with pool1 = min(B, ns) > 16384).
//
// The P1 slots are split into G = ceil(P1 / 4096) groups; burst t / 16 of the step stream draws
// inside group (t / 16) mod G (pss_common.h slot_draw_grouped).  Each (rank, group) is an
// independent slot machine of <= 4096 slots, so one 64-lane wave replays it with its table in
// 16 KB of LDS -- the same one-exchange-per-step replay as the small-pool kernel, with no HBM
// slot table and no chunk bucketing.  At C5 (B = 2^20, 8 ranks) that is 2048 streams of ~45K
// steps: one wave each, one round of the chip, no last-occurrence pass at all.
//
//   k_g_keys     per rank: slot key, tail / init Feistel keys, every pool2 window's round keys
//   k_g_lastocc  (only when a stream is cut into several tiles) per (rank, group, tile): the
//                last step that drew each slot -> VAL = the value it inserted, or kNone
//   k_g_emit     per (rank, group, tile), one wave: slot table at the tile's start (initial
//                Feistel-permuted window 0, or the VAL walk-back), then the replay, 256 steps
//                per iteration; the last tile of a group stores its final table in FIN
//   k_g_tail     final pool drained in the order of the tail Feistel bijection of [0, P1),
//                gathered from FIN
#include <type_traits>

#include "pss_device.h"

namespace pss {

static inline int64_t gdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// key table layout per local rank (words): [0, 2) slot key, [8, 16) tail keys,
// [16, 24) init keys, [24 + 8 (w - 1), + 8) round keys of pool2 window w = 1 .. W
constexpr int64_t kGKeySlot = 0, kGKeyTail = 8, kGKeyInit = 16, kGKeyWin = 24;

struct GPlan {
    int64_t P1, T, W;        // slots, steps, pool2 windows
    int64_t Tg_max;          // longest group sub-stream
    int64_t L, tiles;        // sub-steps per tile (multiple of 256), tiles per group stream
    int64_t kt_stride;       // key-table words per local rank
    Groups gr;
    uint32_t Smax;           // largest group
    uint32_t B32, hB, walk_full, w_last, len_last, h_last, hP, twoB;
};

static GPlan gplan(const Geometry &g, int32_t nr, int cus) {
    GPlan p{};
    p.P1 = g.B < g.ns ? g.B : g.ns;
    p.T = g.ns - p.P1;
    p.W = p.T > 0 ? 1 + (p.T - 1) / g.B : 0;
    p.gr = v2_groups((uint32_t)p.P1);
    p.Smax = group_size(p.gr, 0);
    p.Tg_max = (int64_t)group_steps(p.gr, 0, (uint64_t)p.T);   // group 0 draws the most
    // one round of waves (8 per CU: 16-20 KB of LDS each); a stream is cut into tiles only
    // when the groups alone do not fill the chip, and never below 4 * Smax steps per tile
    const int64_t streams = (int64_t)(nr > 0 ? nr : 1) * p.gr.G;
    const int64_t want = gdiv(8LL * cus, streams);
    const int64_t most = p.Tg_max > 0 ? gdiv(p.Tg_max, 4LL * p.Smax) : 1;
    p.tiles = want < 1 ? 1 : (want > most ? most : want);
    if (p.tiles < 1) p.tiles = 1;
    p.L = p.Tg_max > 0 ? gdiv(gdiv(p.Tg_max, p.tiles), 256) * 256 : 256;
    p.tiles = p.Tg_max > 0 ? gdiv(p.Tg_max, p.L) : 1;
    p.kt_stride = kGKeyWin + kRoundKeyWords * p.W;
    p.B32 = (uint32_t)g.B;
    p.hB = feistel_half_bits(p.B32);
    p.walk_full = p.B32 != (1u << (2 * p.hB));
    p.w_last = (uint32_t)p.W;
    p.len_last = p.W > 0 ? (uint32_t)(g.ns - p.W * g.B) : 0;
    p.h_last = feistel_half_bits(p.len_last > 0 ? p.len_last : 1);
    p.hP = feistel_half_bits((uint32_t)p.P1);
    p.twoB = (uint32_t)(2 * g.B < g.ns ? 2 * g.B : g.ns);
    return p;
}

static int gcus() {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    return n;
}

// ---- keys ------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_g_keys(Geometry g, int32_t rank_lo, int64_t W,
                                                int64_t stride, uint32_t *__restrict__ kt) {
    const int32_t rl = (int32_t)blockIdx.y;
    const uint32_t rank = (uint32_t)(rank_lo + rl);
    const int64_t item = (int64_t)blockIdx.x * 256 + threadIdx.x;
    uint32_t *b = kt + rl * stride;
    uint32_t k[kRoundKeyWords];
    if (item == 0) {
        const SlotKey sk = slot_key(g, rank);
        b[kGKeySlot] = sk.s0; b[kGKeySlot + 1] = sk.s1;
        return;
    }
    int64_t off;
    if (item == 1) { round_keys8(g.key0, g.key1, 0, rank, DOM_V2_TAIL, k); off = kGKeyTail; }
    else if (item == 2) { round_keys8(g.key0, g.key1, 0, rank, DOM_V2_INIT, k); off = kGKeyInit; }
    else if (item < W + 3) {
        const int64_t w = item - 2;
        round_keys8(g.key0, g.key1, (uint32_t)w, rank, DOM_V2_INS, k);
        off = kGKeyWin + kRoundKeyWords * (w - 1);
    } else {
        return;
    }
#pragma unroll
    for (int i = 0; i < kRoundKeyWords; i++) b[off + i] = k[i];
}

// value inserted at (32-bit) step t: pool2 window w = 1 + t / B in Feistel order
__device__ __forceinline__ uint32_t g_ins(const GPlan &pl, const uint32_t *ktr, uint32_t t) {
    const uint32_t w = 1 + t / pl.B32;
    const uint32_t p = t - (w - 1) * pl.B32;
    const bool lastw = w == pl.w_last;
    const uint32_t len = lastw ? pl.len_last : pl.B32;
    const uint32_t h = lastw ? pl.h_last : pl.hB;
    return w * pl.B32 + feistel(p, len, h, ktr + kGKeyWin + kRoundKeyWords * (w - 1));
}

// ---- pass A: last occurrence per (rank, group, tile < tiles - 1) -------------------------------
__global__ __launch_bounds__(256) void k_g_lastocc(Geometry g, GPlan pl, int32_t rank_lo,
                                                   const uint32_t *__restrict__ KT,
                                                   uint32_t *__restrict__ VAL) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    const uint32_t nt = (uint32_t)(pl.tiles - 1);
    const uint32_t tile = blockIdx.x % nt;
    const uint32_t sg = blockIdx.x / nt;                   // rl * G + group
    const uint32_t grp = sg % pl.gr.G;
    const int32_t rl = (int32_t)(sg / pl.gr.G);
    const uint32_t *ktr = KT + rl * pl.kt_stride;
    const uint32_t S = group_size(pl.gr, grp);
    const uint32_t Tg = (uint32_t)group_steps(pl.gr, grp, (uint64_t)pl.T);
    const uint32_t ulo = tile * (uint32_t)pl.L < Tg ? tile * (uint32_t)pl.L : Tg;
    const uint32_t uhi = Tg - ulo < (uint32_t)pl.L ? Tg : ulo + (uint32_t)pl.L;
    uint32_t *lastT = smem;
    for (uint32_t s = threadIdx.x; s < S; s += 256) lastT[s] = 0;
    const uint32_t s0 = ktr[kGKeySlot], s1 = ktr[kGKeySlot + 1];
    __syncthreads();
    for (uint32_t u = ulo + threadIdx.x; u < uhi; u += 256) {
        const uint32_t t = (uint32_t)group_step(pl.gr, grp, u);
        atomicMax(&lastT[scale32(slot_hash(t, s0, s1), S)], u - ulo + 1);
    }
    __syncthreads();
    uint32_t *V = VAL + ((int64_t)sg * nt + tile) * pl.Smax;
    for (uint32_t s = threadIdx.x; s < S; s += 256) {
        const uint32_t lt = lastT[s];
        V[s] = lt ? g_ins(pl, ktr, (uint32_t)group_step(pl.gr, grp, ulo + lt - 1)) : kNone;
    }
}

// ---- pass B: replay ---------------------------------------------------------------------------
typedef __attribute__((address_space(3))) volatile uint8_t g_lds_vu8;

template <bool NARROW>
struct GIds {   // virtual index <-> slot word <-> emitted id
    uint32_t twoB, old32, new32, N32;
    RankDesc rd;
    Geometry g;
    __device__ __forceinline__ uint32_t to_slot(uint32_t v) const {
        if constexpr (NARROW) return (uint32_t)emit_id<true>(v, twoB, old32, new32, N32, rd, g);
        else return v;
    }
    __device__ __forceinline__ int64_t from_slot(uint32_t x) const {
        if constexpr (NARROW) return (int64_t)x;
        else return emit_id<false>(x, twoB, old32, new32, N32, rd, g);
    }
};

// One 64-step batch without relying on the lane-ordered exchange: a collision probe byte per
// slot (S <= 4096), then lanes that drew the same slot are chained through shuffles -- the
// first exchanges the last peer's insertion, the others take the previous peer's.
__device__ __forceinline__ uint32_t xchg_unordered(uint32_t *buf, g_lds_vu8 *mark, uint32_t k,
                                                   uint32_t ins, bool valid, int lane) {
    if (valid) mark[k] = (uint8_t)lane;
    const uint32_t probe = mark[k];
    const bool clash = valid && probe != (uint32_t)lane;
    uint64_t cm = __ballot(clash);
    if (cm == 0) return valid ? atomicExch(&buf[k], ins) : 0u;
    uint64_t m = valid ? (1ull << lane) : 0ull;
    while (cm) {
        const int cl = __ffsll((long long)cm) - 1;
        const uint32_t sc = (uint32_t)__builtin_amdgcn_readlane((int)k, cl);
        const bool same = valid && k == sc;
        const uint64_t mm = __ballot(same);
        if (same) m = mm;
        cm &= ~mm;
    }
    const uint64_t lower = m & ((1ull << lane) - 1ull);
    const int hi_lane = m ? 63 - __clzll((long long)m) : lane;
    const int prev_lane = lower ? 63 - __clzll((long long)lower) : lane;
    const uint32_t ins_last = (uint32_t)__shfl((int)ins, hi_lane);
    const uint32_t ins_prev = (uint32_t)__shfl((int)ins, prev_lane);
    return (valid && !lower) ? atomicExch(&buf[k], ins_last) : ins_prev;
}

template <bool ORDERED, bool NARROW>
__global__ __launch_bounds__(64) void k_g_emit(Geometry g, GPlan pl, const RankDesc *__restrict__ ranks,
                                               int32_t rank_lo, const uint32_t *__restrict__ KT,
                                               const uint32_t *__restrict__ VAL,
                                               uint32_t *__restrict__ FIN, int do_fin,
                                               int64_t pos_lo, int64_t count,
                                               int64_t *__restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    uint32_t *buf = smem;                                            // Smax slot words
    g_lds_vu8 *mark = (g_lds_vu8 *)(smem + pl.Smax);                  // !ORDERED: Smax bytes
    const int lane = threadIdx.x;
    const uint32_t ntl = (uint32_t)pl.tiles;
    const uint32_t tile = blockIdx.x % ntl;
    const uint32_t sg = blockIdx.x / ntl;
    const uint32_t grp = sg % pl.gr.G;
    const int32_t rl = (int32_t)(sg / pl.gr.G);
    const uint32_t rank = (uint32_t)(rank_lo + rl);
    const uint32_t *ktr = KT + rl * pl.kt_stride;
    const uint32_t S = group_size(pl.gr, grp), base = group_base(pl.gr, grp);
    const uint32_t Tg = (uint32_t)group_steps(pl.gr, grp, (uint64_t)pl.T);
    const uint32_t ulo = tile * (uint32_t)pl.L < Tg ? tile * (uint32_t)pl.L : Tg;
    const uint32_t uhi = Tg - ulo < (uint32_t)pl.L ? Tg : ulo + (uint32_t)pl.L;
    const int64_t pos_hi = pos_lo + count;
    const bool last = tile == ntl - 1;
    bool emits = false;
    if (ulo < uhi) {
        const int64_t tf = (int64_t)group_step(pl.gr, grp, ulo);
        const int64_t tl = (int64_t)group_step(pl.gr, grp, uhi - 1);
        emits = tl >= pos_lo && tf < pos_hi;
    }
    if (!emits && !(last && do_fin)) return;
    const RankDesc rd = ranks[rank];
    GIds<NARROW> ids;
    ids.twoB = pl.twoB;
    ids.old32 = (uint32_t)rd.old_start; ids.new32 = (uint32_t)rd.new_start;
    ids.N32 = (uint32_t)g.N;
    ids.rd = rd;
    ids.g = g;
    // slot table at the tile's start: the last value an earlier tile inserted into each slot,
    // else the initial content -- window 0 permuted by the init Feistel bijection of [0, P1)
    {
        const uint32_t *ik = ktr + kGKeyInit;
        const int64_t ntv = pl.tiles - 1;
        const uint32_t *Vg = VAL + (int64_t)sg * ntv * pl.Smax;
        for (uint32_t s = lane; s < S; s += 64) {
            uint32_t v = kNone;
            for (int64_t tt = (int64_t)tile - 1; tt >= 0 && v == kNone; tt--) v = Vg[tt * pl.Smax + s];
            if (v == kNone) v = feistel(base + s, (uint32_t)pl.P1, pl.hP, ik);
            buf[s] = ids.to_slot(v);
        }
    }
    __syncthreads();
    const uint32_t s0 = ktr[kGKeySlot], s1 = ktr[kGKeySlot + 1];
    int64_t *o = out + (int64_t)rl * count - pos_lo;
    const uint32_t G = pl.gr.G, B = pl.B32;
    const bool pow2 = (S & (S - 1u)) == 0u;
    const uint32_t shS = 32u - (uint32_t)ceil_log2_u64(S);
    const bool full_emit = emits && (int64_t)group_step(pl.gr, grp, ulo) >= pos_lo &&
                           (int64_t)group_step(pl.gr, grp, uhi - 1) < pos_hi;
    // per lane and sub-batch j: the step t_j of sub-step u0 + 64 j + lane and its pool2
    // position (w_j, p_j), advanced by 256 G steps per iteration without division
    uint32_t tj[4], wj[4], pj[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
        tj[j] = (uint32_t)group_step(pl.gr, grp, (uint64_t)ulo + 64u * j + lane);
        wj[j] = 1 + tj[j] / B;
        pj[j] = tj[j] - (wj[j] - 1) * B;
    }
    const uint32_t dT = 256u * G;
    const bool win_fast = !pl.walk_full;
    for (uint32_t u0 = ulo; u0 < uhi; u0 += 256) {
        // wave-uniform window of the iteration's first step; the iteration spans < B steps,
        // so every lane is in window wa or wa + 1
        const uint32_t wa = (uint32_t)__builtin_amdgcn_readfirstlane((int)wj[0]);
        const uint32_t *ka = ktr + kGKeyWin + kRoundKeyWords * (wa - 1);
        uint32_t KA[kFeistelRounds], KB[kFeistelRounds];
#pragma unroll
        for (int i = 0; i < kFeistelRounds; i++) KA[i] = ka[i];
        const bool two = wa < pl.w_last;   // window wa + 1 exists
#pragma unroll
        for (int i = 0; i < kFeistelRounds; i++) KB[i] = two ? ka[kRoundKeyWords + i] : 0u;
        const bool fast = win_fast && wa + 1 < pl.w_last && u0 + 256 <= uhi && full_emit;
        uint32_t k[4], ins[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const uint32_t hsh = slot_hash(tj[j], s0, s1);
            k[j] = pow2 ? hsh >> shS : scale32(hsh, S);
            const bool b = wj[j] != wa;
            uint32_t kk[kFeistelRounds];
#pragma unroll
            for (int i = 0; i < kFeistelRounds; i++) kk[i] = b ? KB[i] : KA[i];
            if (fast) {
                ins[j] = wj[j] * B + feistel_once(pj[j], pl.hB, kk);
            } else {
                const bool lastw = wj[j] == pl.w_last;
                const bool valid = u0 + 64u * j + lane < uhi;
                ins[j] = valid ? wj[j] * B + feistel(pj[j], lastw ? pl.len_last : B,
                                                     lastw ? pl.h_last : pl.hB, kk)
                               : 0u;
            }
        }
        uint32_t v[4];
        if constexpr (ORDERED) {
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const bool valid = fast || u0 + 64u * j + lane < uhi;
                v[j] = valid ? atomicExch(&buf[k[j]], ids.to_slot(ins[j])) : 0u;
            }
        } else {
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const bool valid = fast || u0 + 64u * j + lane < uhi;
                v[j] = xchg_unordered(buf, mark, k[j], ids.to_slot(ins[j]), valid, lane);
            }
        }
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const bool valid = fast || u0 + 64u * j + lane < uhi;
            if (valid && (fast || ((int64_t)tj[j] >= pos_lo && (int64_t)tj[j] < pos_hi)))
                o[tj[j]] = ids.from_slot(v[j]);
            tj[j] += dT;
            pj[j] += dT;
            if (pj[j] >= B) { pj[j] -= B; wj[j]++; }
        }
    }
    if (last && do_fin) {
        __syncthreads();
        uint32_t *F = FIN + (int64_t)rl * pl.P1 + base;
        for (uint32_t s = lane; s < S; s += 64) F[s] = buf[s];
    }
}

// ---- tail ---------------------------------------------------------------------------------
template <bool NARROW>
__global__ __launch_bounds__(256) void k_g_tail(Geometry g, GPlan pl, const RankDesc *__restrict__ ranks,
                                                int32_t rank_lo, const uint32_t *__restrict__ KT,
                                                const uint32_t *__restrict__ FIN,
                                                int64_t pos_lo, int64_t count,
                                                int64_t *__restrict__ out) {
    const int32_t rl = (int32_t)blockIdx.y;
    const RankDesc rd = ranks[rank_lo + rl];
    GIds<NARROW> ids;
    ids.twoB = pl.twoB;
    ids.old32 = (uint32_t)rd.old_start; ids.new32 = (uint32_t)rd.new_start;
    ids.N32 = (uint32_t)g.N;
    ids.rd = rd;
    ids.g = g;
    const uint32_t *tk = KT + rl * pl.kt_stride + kGKeyTail;
    uint32_t kk[kFeistelRounds];
#pragma unroll
    for (int i = 0; i < kFeistelRounds; i++) kk[i] = tk[i];
    const uint32_t P1 = (uint32_t)pl.P1;
    const uint32_t *F = FIN + (int64_t)rl * pl.P1;
    int64_t *o = out + (int64_t)rl * count - pos_lo;
    const int64_t pos_hi = pos_lo + count;
    for (uint32_t j = blockIdx.x * 256u + threadIdx.x; j < P1; j += gridDim.x * 256u) {
        const int64_t pos = pl.T + j;
        if (pos < pos_lo || pos >= pos_hi) continue;
        o[pos] = ids.from_slot(F[feistel(j, P1, pl.hP, kk)]);
    }
}

// ------------------------------------------------------------------------------------------
// launcher
// ------------------------------------------------------------------------------------------
bool v2_grouped(const Geometry &g) { return (g.B < g.ns ? g.B : g.ns) > (int64_t)kLdsSlotMax; }

// VAL ring buffer: key table (nr * kt_stride) then the per-tile last-occurrence tables
size_t v2_grp_val_bytes(const Geometry &g, int32_t nr) {
    const GPlan p = gplan(g, nr, gcus());
    const size_t words = (size_t)nr * (size_t)p.kt_stride +
                         (size_t)nr * p.gr.G * (size_t)(p.tiles - 1) * p.Smax;
    return words * sizeof(uint32_t);
}

// FIN: the final slot table of every rank (read by the tail)
size_t v2_grp_fin_bytes(const Geometry &g, int32_t nr) {
    const int64_t P1 = g.B < g.ns ? g.B : g.ns;
    return (size_t)nr * (size_t)P1 * sizeof(uint32_t);
}

hipError_t launch_v2_grp(const Geometry &g, const RankDesc *ranks, int32_t rank_lo, int32_t nr,
                         int64_t pos_lo, int64_t count, int64_t *out, uint32_t *VALws,
                         uint32_t *FIN, hipStream_t s, const Marker &mk, bool ordered, int stage) {
    const int64_t pos_hi = pos_lo + count < g.ns ? pos_lo + count : g.ns;
    if (nr <= 0 || pos_hi <= pos_lo) return hipSuccess;
    const GPlan pl = gplan(g, nr, gcus());
    const bool do_pre = stage != V2_STAGE_EMIT, do_emit = stage != V2_STAGE_PRE;
    uint32_t *KT = VALws;
    uint32_t *VAL = VALws + (size_t)nr * (size_t)pl.kt_stride;
    if (do_pre) {
        mk(K_V2_LASTOCC, s);
        const int64_t items = pl.W + 3;
        hipLaunchKernelGGL(k_g_keys, dim3((uint32_t)gdiv(items, 256), (uint32_t)nr), dim3(256), 0, s,
                           g, rank_lo, pl.W, pl.kt_stride, KT);
        if (pl.tiles > 1)
            hipLaunchKernelGGL(k_g_lastocc, dim3((uint32_t)((int64_t)nr * pl.gr.G * (pl.tiles - 1))), dim3(256),
                               (size_t)pl.Smax * 4, s, g, pl, rank_lo, (const uint32_t *)KT, VAL);
        if (!do_emit) mk(-1, s);
    }
    if (!do_emit) return hipGetLastError();
    const bool need_tail = pos_hi > pl.T;
    const bool narrow = g.N + g.ns < (int64_t)UINT32_MAX;
    const int do_fin = need_tail ? 1 : 0;
    if (pl.T > 0) {
        mk(K_V2_EMIT, s);
        const dim3 grid((uint32_t)((int64_t)nr * pl.gr.G * pl.tiles));
        // LDS padded so that a CU takes exactly 8 waves (2 per SIMD, balanced) instead of 9
        size_t lds = (size_t)pl.Smax * 4 + (ordered ? 0 : (size_t)pl.Smax) + 16;
        if (lds * 9 <= 160 * 1024) lds = 160 * 1024 / 9 + 16;
#define PSS_GE(O, N) hipLaunchKernelGGL((k_g_emit<O, N>), grid, dim3(64), lds, s, g, pl, ranks, rank_lo, \
                                        (const uint32_t *)KT, (const uint32_t *)VAL, FIN, do_fin, pos_lo, count, out)
        if (ordered && narrow) PSS_GE(true, true);
        else if (ordered) PSS_GE(true, false);
        else if (narrow) PSS_GE(false, true);
        else PSS_GE(false, false);
#undef PSS_GE
    }
    if (need_tail) {
        mk(K_V2_TAIL, s);
        if (pl.T == 0) {
            // no steps: the final table is the initial one -- written by a one-tile emit of
            // the empty stream (each group wave stores its initial table)
            const dim3 grid((uint32_t)((int64_t)nr * pl.gr.G * pl.tiles));
            const size_t lds = (size_t)pl.Smax * 4 + (ordered ? 0 : (size_t)pl.Smax) + 16;
            if (narrow)
                hipLaunchKernelGGL((k_g_emit<true, true>), grid, dim3(64), lds, s, g, pl, ranks, rank_lo,
                                   (const uint32_t *)KT, (const uint32_t *)VAL, FIN, 1, pos_lo, count, out);
            else
                hipLaunchKernelGGL((k_g_emit<true, false>), grid, dim3(64), lds, s, g, pl, ranks, rank_lo,
                                   (const uint32_t *)KT, (const uint32_t *)VAL, FIN, 1, pos_lo, count, out);
        }
        const dim3 grid((uint32_t)gdiv(pl.P1 < 262144 ? pl.P1 : 262144, 256), (uint32_t)nr);
        if (narrow)
            hipLaunchKernelGGL((k_g_tail<true>), grid, dim3(256), 0, s, g, pl, ranks, rank_lo,
                               (const uint32_t *)KT, (const uint32_t *)FIN, pos_lo, count, out);
        else
            hipLaunchKernelGGL((k_g_tail<false>), grid, dim3(256), 0, s, g, pl, ranks, rank_lo,
                               (const uint32_t *)KT, (const uint32_t *)FIN, pos_lo, count, out);
    }
    mk(-1, s);
    return hipGetLastError();
}

hipError_t init_kernel_attributes_v2grp() {
    const int big = 160 * 1024;
    hipError_t e = hipSuccess;
#define PSS_ATTR(fn) { hipError_t x = hipFuncSetAttribute((const void *)(fn), hipFuncAttributeMaxDynamicSharedMemorySize, big); if (x != hipSuccess) e = x; }
    PSS_ATTR((k_g_emit<true, true>));
    PSS_ATTR((k_g_emit<true, false>));
    PSS_ATTR((k_g_emit<false, true>));
    PSS_ATTR((k_g_emit<false, false>));
    PSS_ATTR(k_g_lastocc);
#undef PSS_ATTR
    return e;
}

}  // namespace pss
