// pss_v2grp.hip -- V2 pools beyond LDS (P1 > kLdsSlotMax): the grouped slot machine
// (reference semantics V2:96-116 with pool1 = min(B, ns) > 16384).
//
// The P1 slots are split into G = ceil(P1 / 4096) groups; burst t / 32 of the step stream draws
// inside group (t / 32) mod G (pss_common.h slot_draw_grouped).  Each (rank, group) is an
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
//                per iteration; the wave of a group's last tile then drains the group's final
//                table from LDS into its tail positions (pss_common.h group_tail_pos)
#include <type_traits>

#include "pss_device.h"

namespace pss {

static inline int64_t gdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// cache-policy bits of the run stores: none (sc0 measured neutral, 173.4 vs 173.1 us, round 3)
constexpr int kGStoreAux = 0;

// key table layout per local rank (words): [0, 2) slot key, [8, 16) init keys,
// [16 + 8 (w - 1), + 8) round keys of pool2 window w = 1 .. W
constexpr int64_t kGKeySlot = 0, kGKeyInit = 8, kGKeyWin = 16;

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
    if (item == 1) { round_keys8(g.key0, g.key1, 0, rank, DOM_V2_INIT, k); off = kGKeyInit; }
    else if (item < W + 2) {
        const int64_t w = item - 1;
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
        atomicMax(&lastT[group_slot(pl.gr, grp, S, u, t, s0, s1)], u - ulo + 1);
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
typedef unsigned int g_u32x2 __attribute__((ext_vector_type(2)));

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

// Four one-pass Feistel chains under wave-uniform round keys K (a full window of 4^h elements).
// h <= kFeistelH16: packed 16-bit pairs (feistel4_pk16).  Wider: the keyed-carry form of feistel_pass --
// with A_i = R_i ^ K_i, A_{i+1} = A_{i-1} ^ F(A_i) ^ (K_{i-1} ^ K_{i+1}) (one 3-input xor per
// round, F = one full-rate 24-bit multiply + bit-field extract); output L = A_5 ^ K_5, R = A_4 ^ F(A_5) ^ K_4.
// Same values as feistel_once on each chain.
// a ^ b ^ k in one v_bitop3_b32 (truth table 0x96) with the wave-uniform k read from an SGPR;
// hipcc fuses only some 3-input xors itself
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t k) {
    uint32_t r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "s"(k));
    return r;
}

template <bool PACKED>
__device__ __forceinline__ void feistel4_uniform(const uint32_t x[4], uint32_t h, const uint32_t K[6],
                                                 uint32_t y[4]) {
    if constexpr (PACKED) {
        uint32_t kp[kFeistelRounds];
#pragma unroll
        for (int i = 0; i < kFeistelRounds; i++) kp[i] = (K[i] & 0xFFFFu) * 0x10001u;
        feistel4_pk16(x, h, kp, y);
    } else {
        const uint32_t mask = (1u << h) - 1u, sh = 24u - h;
        const uint32_t K02 = K[0] ^ K[2], K13 = K[1] ^ K[3], K24 = K[2] ^ K[4], K35 = K[3] ^ K[5];
        // F = bits [24 - h, 24) of the 24-bit product: one v_mul_u32_u24 and one v_bfe_u32, so
        // that each round is mul, bfe and a single 3-input xor (v_bitop3)
        auto F = [&](uint32_t a) -> uint32_t {
            return __builtin_amdgcn_ubfe((a & 0xFFFFFFu) * kFeistelM24, sh, h);
        };
#pragma unroll
        for (int c = 0; c < 4; c++) {
            const uint32_t A0 = (x[c] & mask) ^ K[0];
            const uint32_t A1 = xor3(x[c] >> h, F(A0), K[1]);
            const uint32_t A2 = xor3(A0, F(A1), K02);
            const uint32_t A3 = xor3(A1, F(A2), K13);
            const uint32_t A4 = xor3(A2, F(A3), K24);
            const uint32_t A5 = xor3(A3, F(A4), K35);
            y[c] = ((A5 ^ K[5]) << h) | xor3(A4, F(A5), K[4]);
        }
    }
}

// feistel4_uniform<false> when the four inputs xb + c 64 G (c < 4) share their low h bits and the
// run advances them by multiples of 2^h (64 G % 2^h == 0): A0 = (xb & mask) ^ K0 and
// C1 = F(A0) ^ K1 are then constants of the run, and chain c's left half is lb + c g64h with
// lb = xb >> h.  Same values, four instructions fewer per chain.
__device__ __forceinline__ void feistel4_rinv(uint32_t lb, uint32_t g64h, uint32_t A0, uint32_t C1,
                                              uint32_t h, const uint32_t K[6], uint32_t y[4]) {
    const uint32_t sh = 24u - h;
    const uint32_t K02 = K[0] ^ K[2], K13 = K[1] ^ K[3], K24 = K[2] ^ K[4], K35 = K[3] ^ K[5];
    auto F = [&](uint32_t a) -> uint32_t {
        return __builtin_amdgcn_ubfe((a & 0xFFFFFFu) * kFeistelM24, sh, h);
    };
#pragma unroll
    for (int c = 0; c < 4; c++) {
        const uint32_t A1 = (lb + (uint32_t)c * g64h) ^ C1;
        const uint32_t A2 = xor3(A0, F(A1), K02);
        const uint32_t A3 = xor3(A1, F(A2), K13);
        const uint32_t A4 = xor3(A2, F(A3), K24);
        const uint32_t A5 = xor3(A3, F(A4), K35);
        y[c] = ((A5 ^ K[5]) << h) | xor3(A4, F(A5), K[4]);
    }
}

// feistel4_rinv on the 16-bit round function (halves of up to kFeistelH16 bits), two chains per
// register: chains 0, 1 in the half-words of the first, 2, 3 of the second.  Lp0 / Lp1 hold the
// chains' left halves, A0p = A0 (both half-words), C1p = F16(A0) ^ K1 (both half-words); the
// keys kp are the round keys' low half-words doubled.  Keyed carry as in feistel4_uniform, one
// packed multiply, one packed shift and one 3-input xor per round and register.
__device__ __forceinline__ void feistel4_rinv16(uint32_t Lp0, uint32_t Lp1, uint32_t A0p, uint32_t C1p,
                                                uint32_t h, const uint32_t kp[6], uint32_t y[4]) {
    const pss_u16x2 M = {(unsigned short)kFeistelM16, (unsigned short)kFeistelM16};
    const pss_u16x2 SH = {(unsigned short)(16u - h), (unsigned short)(16u - h)};
    auto F = [&](uint32_t a) -> uint32_t {
        return __builtin_bit_cast(uint32_t, (__builtin_bit_cast(pss_u16x2, a) * M) >> SH);
    };
    const uint32_t K02 = kp[0] ^ kp[2], K13 = kp[1] ^ kp[3], K24 = kp[2] ^ kp[4], K35 = kp[3] ^ kp[5];
    const uint32_t A10 = Lp0 ^ C1p, A11 = Lp1 ^ C1p;
    const uint32_t A20 = xor3(A0p, F(A10), K02), A21 = xor3(A0p, F(A11), K02);
    const uint32_t A30 = xor3(A10, F(A20), K13), A31 = xor3(A11, F(A21), K13);
    const uint32_t A40 = xor3(A20, F(A30), K24), A41 = xor3(A21, F(A31), K24);
    const uint32_t A50 = xor3(A30, F(A40), K35), A51 = xor3(A31, F(A41), K35);
    const uint32_t L0 = A50 ^ kp[5], L1 = A51 ^ kp[5];
    const uint32_t R0 = xor3(A40, F(A50), kp[4]), R1 = xor3(A41, F(A51), kp[4]);
    y[0] = ((L0 & 0xFFFFu) << h) | (R0 & 0xFFFFu);
    y[1] = ((L0 >> 16) << h) | (R0 >> 16);
    y[2] = ((L1 & 0xFFFFu) << h) | (R1 & 0xFFFFu);
    y[3] = ((L1 >> 16) << h) | (R1 >> 16);
}

// Table-wide Feistel pass of a wave: out[s] = f(feistel(off + s, n, h, K)) for s < cnt, four
// chains per lane; the one-pass forms when n = 4^h (no cycle walking), else the walking one.
template <class Put>
__device__ __forceinline__ void feistel_table(uint32_t off, uint32_t cnt, uint32_t n, uint32_t h,
                                              const uint32_t *Kg, int lane, Put put) {
    uint32_t K[kFeistelRounds];
#pragma unroll
    for (int i = 0; i < kFeistelRounds; i++) K[i] = __builtin_amdgcn_readfirstlane(Kg[i]);
    if (n == (1u << (2 * h))) {
        for (uint32_t s0 = 0; s0 < cnt; s0 += 256) {
            uint32_t x[4], y[4];
#pragma unroll
            for (int j = 0; j < 4; j++) x[j] = off + s0 + 64u * j + (uint32_t)lane;
            if (feistel_packed_ok(h)) feistel4_uniform<true>(x, h, K, y);
            else if (h > kFeistelH16) feistel4_uniform<false>(x, h, K, y);
            else for (int j = 0; j < 4; j++) y[j] = feistel_once(x[j], h, K);
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const uint32_t s = s0 + 64u * j + (uint32_t)lane;
                if (s < cnt) put(s, y[j]);
            }
        }
    } else {
        for (uint32_t s = lane; s < cnt; s += 64) put(s, feistel(off + s, n, h, K));
    }
}

// MAPPED (pss_generate_mapped; ORDERED only): each id is written as (int32 file position, int32
// offset) through the epoch's bucketed map (map_one_bucketed, the map of pss_map) into ma.fpos /
// ma.off, where the plain replay writes the int64 id -- the same 8 bytes per step, no id pass.
template <bool ORDERED, bool NARROW, bool PACKED, bool POW2, bool MAPPED = false>
__global__ __launch_bounds__(64) void k_g_emit(Geometry g, GPlan pl, const RankDesc *__restrict__ ranks,
                                               int32_t rank_lo, const uint32_t *__restrict__ KT,
                                               const uint32_t *__restrict__ VAL, int do_tail,
                                               int64_t pos_lo, int64_t count,
                                               int64_t *__restrict__ out, RankArgs ra, int use_ra,
                                               MapArgs ma) {
    static_assert(ORDERED || !MAPPED, "the mapped replay runs on the lane-ordered exchange path");
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
    const bool drain = tile == ntl - 1 && do_tail;
    bool emits = false, full_emit = false;
    if (ulo < uhi) {
        const int64_t tf = (int64_t)group_step(pl.gr, grp, ulo);
        const int64_t tl = (int64_t)group_step(pl.gr, grp, uhi - 1);
        emits = tl >= pos_lo && tf < pos_hi;
        full_emit = tf >= pos_lo && tl < pos_hi;
    }
    if (!emits && !drain) return;
    const RankDesc rd = use_ra ? ra.r[rl] : ranks[rank];   // (kernel argument: a scalar load)
    GIds<NARROW> ids;
    ids.twoB = pl.twoB;
    ids.old32 = (uint32_t)rd.old_start; ids.new32 = (uint32_t)rd.new_start;
    ids.N32 = (uint32_t)g.N;
    ids.rd = rd;
    ids.g = g;
    // slot table at the tile's start: the last value an earlier tile inserted into each slot,
    // else the initial content -- window 0 permuted by the init Feistel bijection of [0, P1)
    if (tile == 0) {
        feistel_table(base, S, (uint32_t)pl.P1, pl.hP, ktr + kGKeyInit, lane,
                      [&](uint32_t s, uint32_t v) { buf[s] = ids.to_slot(v); });
    } else {
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
    int32_t *ofp = ma.fpos + (int64_t)rl * count - pos_lo, *ooff = ma.off + (int64_t)rl * count - pos_lo;
    auto put = [&](int64_t pos, int64_t id) {   // one id, outside the runs' buffer stores
        if constexpr (MAPPED) {
            int32_t f, of;
            map_id_fast(ma, id, f, of);
            ofp[pos] = f;
            ooff[pos] = of;
        } else {
            o[pos] = id;
        }
    };
    const uint32_t G = pl.gr.G, B = pl.B32;
    const uint32_t G64 = 64u * G, G256 = 256u * G;
    const uint32_t shS = 32u - (uint32_t)ceil_log2_u64(S);
    const bool gpow2 = (S & (S - 1u)) == 0u;         // this group pairs its draws
    // lane l serves sub-steps u0 + 64 j + l: step t_first + c_lane + j * 64 G, where t_first is
    // the iteration's first step (wave-uniform, advanced by 256 G per iteration without
    // division, together with its pool2 window wa and offset pa)
    // (bursts of kBurst = 32 steps: lanes 0-31 and 32-63 each serve one burst's consecutive
    // steps, so a store instruction writes two runs of 32 positions -- 256 B of ids, 128 B of
    // file positions -- where bursts of 16 wrote four runs of 64 / 128 B)
    static_assert(kBurst == 16 || kBurst == 32 || kBurst == 64, "a store covers 64 / kBurst bursts");
    const uint32_t c_lane = ((uint32_t)lane / kBurst) * kBurst * G + ((uint32_t)lane % kBurst);
    const uint32_t span = (256u - kBurst) * G + kBurst - 1u;   // last step of an iteration - first step
    uint32_t t_first = (uint32_t)group_step(pl.gr, grp, ulo);
    uint32_t wa = 1 + t_first / B;
    uint32_t pa = t_first - (wa - 1) * B;
    const bool runs_ok = full_emit && !pl.walk_full;
    uint32_t u0 = ulo;
    // round keys of window wk (Kc) and of wk + 1 (Kn, issued a run ahead of its first use)
    const int32_t W = (int32_t)pl.W;
    auto win_keys = [&](uint32_t w, uint32_t Kx[kFeistelRounds]) {
        if (w >= 1u && (int32_t)w <= W) {
            const uint32_t *kw = ktr + kGKeyWin + kRoundKeyWords * (w - 1);
#pragma unroll
            for (int i = 0; i < kFeistelRounds; i++) Kx[i] = __builtin_amdgcn_readfirstlane(kw[i]);
        } else {
#pragma unroll
            for (int i = 0; i < kFeistelRounds; i++) Kx[i] = 0u;
        }
    };
    uint32_t wk = wa, Kc[kFeistelRounds], Kn[kFeistelRounds];
    win_keys(wk, Kc);
    win_keys(wk + 1u, Kn);
    // the last pool2 window (len_last < B values) runs on the same machinery when its Feistel
    // half width is B's: a first pass as in a full window, then the lanes whose image lies at or
    // beyond len_last walk on (cycle walking, wave-uniform keys)
    const bool last_runs = pl.h_last == pl.hB;
    while (u0 < uhi) {
        // a run of whole iterations inside the window wa: keys in SGPRs, no bookkeeping
        uint32_t n = 0;
        const bool wlast = wa == pl.w_last;
        const uint32_t wlen = wlast ? pl.len_last : B;
        if (runs_ok && (wa < pl.w_last || (wlast && last_runs)) && pa + span < wlen && uhi - u0 >= 256u) {
            const uint32_t by_win = (wlen - 1u - span - pa) / G256 + 1u;
            const uint32_t by_end = (uhi - u0) / 256u;
            n = by_win < by_end ? by_win : by_end;
        }
        if (n) {
            if (wa != wk) {
                if (wa == wk + 1u) {
#pragma unroll
                    for (int i = 0; i < kFeistelRounds; i++) Kc[i] = Kn[i];
                } else {
                    win_keys(wa, Kc);
                }
                wk = wa;
                win_keys(wk + 1u, Kn);
            }
            uint32_t K[kFeistelRounds];
#pragma unroll
            for (int i = 0; i < kFeistelRounds; i++) K[i] = Kc[i];
            // ids of the window's values wa B + y: one add when the window maps contiguously
            const uint32_t wB = wa * B;
            const uint32_t id_first = ids.to_slot(wB), id_last = ids.to_slot(wB + wlen - 1u);
            // wave-uniform branch conditions (readfirstlane: scalar branches, no exec-masked
            // copies of the run loops)
            const bool contig = __builtin_amdgcn_readfirstlane(
                NARROW && id_last - id_first == wlen - 1u && ((wB < pl.twoB) == (wB + wlen - 1u < pl.twoB)));
            const bool walk = __builtin_amdgcn_readfirstlane(wlen != (1u << (2u * pl.hB)));
            uint32_t tb = t_first + c_lane, xb = pa + c_lane;
            // the run's stores through a buffer descriptor on its wave-uniform base: 32-bit
            // per-lane offsets, no 64-bit address registers rewritten under in-flight stores
            // (with those, hipcc drained vmcnt(0) every iteration)
            auto rsrc_at = [&](const void *p, uint32_t bytes) {
                const uint64_t b64 = (uint64_t)(uintptr_t)p;
                const uint32_t lo32 = __builtin_amdgcn_readfirstlane((uint32_t)b64);
                const uint32_t hi32 = __builtin_amdgcn_readfirstlane((uint32_t)(b64 >> 32));
                return __builtin_amdgcn_make_buffer_rsrc((void *)(((uint64_t)hi32 << 32) | lo32), 0,
                                                         (int)bytes, 0x00020000);
            };
            const __amdgpu_buffer_rsrc_t orsrc = rsrc_at(MAPPED ? (const void *)(ofp + t_first) : (const void *)(o + t_first),
                                                         n * G256 * (MAPPED ? 4u : 8u));
            const __amdgpu_buffer_rsrc_t frsrc = rsrc_at(MAPPED ? (const void *)(ooff + t_first) : (const void *)(o + t_first),
                                                         n * G256 * (MAPPED ? 4u : 8u));
            (void)frsrc;
            uint32_t voff = c_lane * (MAPPED ? 4u : 8u);              // per-lane byte offsets
            const uint32_t hmask = (1u << pl.hB) - 1u;
            auto body = [&](auto ctg, auto rinv, auto wlk) {
                constexpr bool RINV = decltype(rinv)::value;
                uint32_t A0 = 0u, C1 = 0u, lb = 0u;
                uint32_t Lp0 = 0u, Lp1 = 0u, A0p = 0u, C1p = 0u, kp[kFeistelRounds];
                const uint32_t g64h = G64 >> pl.hB, g256h = G256 >> pl.hB, g256p = g256h * 0x10001u;
                if constexpr (RINV) {
                    A0 = (xb & hmask) ^ K[0];
                    lb = xb >> pl.hB;
                    if constexpr (PACKED) {   // the 16-bit round function, chains paired
                        C1 = ((((A0 * kFeistelM16) & 0xFFFFu) >> (16u - pl.hB))) ^ K[1];
                        A0p = (A0 & 0xFFFFu) * 0x10001u;
                        C1p = (C1 & 0xFFFFu) * 0x10001u;
                        Lp0 = lb | ((lb + g64h) << 16);
                        Lp1 = (lb + 2u * g64h) | ((lb + 3u * g64h) << 16);
#pragma unroll
                        for (int i = 0; i < kFeistelRounds; i++) kp[i] = (K[i] & 0xFFFFu) * 0x10001u;
                    } else {
                        C1 = __builtin_amdgcn_ubfe((A0 & 0xFFFFFFu) * kFeistelM24, 24u - pl.hB, pl.hB) ^ K[1];
                    }
                }
                for (uint32_t it = 0; it < n; it++) {
                    uint32_t k[4];
                    if (POW2 || gpow2) {    // paired draws: sub-steps u, u + 64 share one hash
                        const uint32_t h0 = slot_hash(tb, s0, s1), h2 = slot_hash(tb + 2u * G64, s0, s1);
                        k[0] = h0 >> shS; k[1] = (h0 << 16) >> shS;
                        k[2] = h2 >> shS; k[3] = (h2 << 16) >> shS;
                    } else {
#pragma unroll
                        for (int j = 0; j < 4; j++) k[j] = scale32(slot_hash(tb + j * G64, s0, s1), S);
                    }
                    uint32_t y[4], v[4];
                    if constexpr (RINV && PACKED) {
                        feistel4_rinv16(Lp0, Lp1, A0p, C1p, pl.hB, kp, y);
                        Lp0 += g256p;
                        Lp1 += g256p;
                    } else if constexpr (RINV) {
                        feistel4_rinv(lb, g64h, A0, C1, pl.hB, K, y);
                        lb += g256h;
                    } else {
                        const uint32_t x[4] = {xb, xb + G64, xb + 2u * G64, xb + 3u * G64};
                        feistel4_uniform<PACKED>(x, pl.hB, K, y);
                    }
                    if constexpr (decltype(wlk)::value) {   // cycle walking in the last window
#pragma unroll
                        for (int j = 0; j < 4; j++)
                            while (y[j] >= wlen) y[j] = feistel_once(y[j], pl.hB, K);
                    }
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        const uint32_t in = decltype(ctg)::value ? id_first + y[j] : ids.to_slot(wB + y[j]);
                        if constexpr (ORDERED) v[j] = atomicExch(&buf[k[j]], in);
                        else v[j] = xchg_unordered(buf, mark, k[j], in, true, lane);
                    }
                    if constexpr (MAPPED) {
                        // the four (file, offset) pairs: the uniform-length map branch-free for
                        // every lane, the general map only when some lane needs it (one ballot
                        // per iteration, not an exec-masked branch per value)
                        int32_t f[4], of[4];
                        uint64_t idv[4];
                        bool slow = !ma.uni;
#pragma unroll
                        for (int j = 0; j < 4; j++) {
                            idv[j] = (uint64_t)ids.from_slot(v[j]);
                            const uint32_t q = udiv_apply((uint32_t)idv[j], ma.um, ma.ul);
                            f[j] = (int32_t)q;
                            of[j] = (int32_t)((uint32_t)idv[j] - q * ma.uL);
                            slow |= idv[j] >= (uint64_t)ma.T;
                        }
                        if (__builtin_amdgcn_ballot_w64(slow) != 0u) {
#pragma unroll
                            for (int j = 0; j < 4; j++) map_id_fast(ma, (int64_t)idv[j], f[j], of[j]);
                        }
#pragma unroll
                        for (int j = 0; j < 4; j++) {
                            __builtin_amdgcn_raw_buffer_store_b32((uint32_t)f[j], orsrc, (int)voff, (int)(4u * (uint32_t)j * G64), 0);
                            __builtin_amdgcn_raw_buffer_store_b32((uint32_t)of[j], frsrc, (int)voff, (int)(4u * (uint32_t)j * G64), 0);
                        }
                    }
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        if constexpr (MAPPED) {
                        } else {
                            const uint64_t id = (uint64_t)ids.from_slot(v[j]);
                            const g_u32x2 d = {(uint32_t)id, (uint32_t)(id >> 32)};
                            __builtin_amdgcn_raw_buffer_store_b64(d, orsrc, (int)voff, (int)(8u * (uint32_t)j * G64), kGStoreAux);
                        }
                    }
                    tb += G256;
                    xb += G256;
                    voff += (MAPPED ? 4u : 8u) * G256;
                }
            };
            auto go = [&](auto wlk) {
                if ((G64 & hmask) == 0u) {   // run-invariant right halves (feistel4_rinv / _rinv16)
                    if (contig) body(std::true_type{}, std::true_type{}, wlk);
                    else body(std::false_type{}, std::true_type{}, wlk);
                } else {
                    if (contig) body(std::true_type{}, std::false_type{}, wlk);
                    else body(std::false_type{}, std::false_type{}, wlk);
                }
            };
            if (walk) go(std::true_type{});
            else go(std::false_type{});
            t_first += n * G256;
            pa += n * G256;
            // MAPPED: a run that ends on its window's end hands the next run the next window;
            // otherwise each window begins with one iteration of the general path below (11 of
            // C5's 175 iterations per stream).  Round 6, same box, 3 rounds each: the mapped
            // replay 0.248 -> 0.225 ms; the id replay LOST with it (558 -> 542 G idx/s, its
            // VALU 52.9M -> 46.9M per launch) and with a store drain in its place (541), so the
            // id replay keeps the general iteration (profiles/r06/ab_grouped_wrap/)
            if (MAPPED && pa >= B) { pa -= B; wa++; }
            u0 += 256u * n;
            continue;
        }
        // one whole iteration straddling the boundary of two full windows wa, wa + 1 (both
        // non-walking): the run machinery with each lane's round keys picked from the two
        // windows' SGPR keys (one v_cndmask per key word) and the paired slot hashes
        if (runs_ok && wa + 1u < pl.w_last && pa < B && pa + span >= B && uhi - u0 >= 256u) {
            if (wa != wk) {
                if (wa == wk + 1u) {
#pragma unroll
                    for (int i = 0; i < kFeistelRounds; i++) Kc[i] = Kn[i];
                } else {
                    win_keys(wa, Kc);
                }
                wk = wa;
                win_keys(wk + 1u, Kn);
            }
            const uint32_t tb = t_first + c_lane;
            uint32_t k[4];
            if (POW2 || gpow2) {
                const uint32_t h0 = slot_hash(tb, s0, s1), h2 = slot_hash(tb + 2u * G64, s0, s1);
                k[0] = h0 >> shS; k[1] = (h0 << 16) >> shS;
                k[2] = h2 >> shS; k[3] = (h2 << 16) >> shS;
            } else {
#pragma unroll
                for (int j = 0; j < 4; j++) k[j] = scale32(slot_hash(tb + j * G64, s0, s1), S);
            }
            uint32_t in[4];
            bool nxt[4];
            uint32_t pj[4];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                pj[j] = pa + c_lane + j * G64;
                nxt[j] = pj[j] >= B;
                if (nxt[j]) pj[j] -= B;
            }
            if constexpr (PACKED) {
                // the 16-bit round function, chains paired per register as in the runs, each
                // half-word under its own window's key (per-lane selects of the two windows'
                // key half-words)
                const uint32_t h = pl.hB, mask = (1u << h) - 1u;
                const pss_u16x2 M = {(unsigned short)kFeistelM16, (unsigned short)kFeistelM16};
                const pss_u16x2 SH = {(unsigned short)(16u - h), (unsigned short)(16u - h)};
                uint32_t L0 = (pj[0] >> h) | ((pj[1] >> h) << 16), R0 = (pj[0] & mask) | ((pj[1] & mask) << 16);
                uint32_t L1 = (pj[2] >> h) | ((pj[3] >> h) << 16), R1 = (pj[2] & mask) | ((pj[3] & mask) << 16);
#pragma unroll
                for (int i = 0; i < kFeistelRounds; i++) {
                    const uint32_t lo = Kc[i] & 0xFFFFu, lon = Kn[i] & 0xFFFFu, hi = Kc[i] << 16, hin = Kn[i] << 16;
                    const uint32_t k0 = (nxt[0] ? lon : lo) | (nxt[1] ? hin : hi);
                    const uint32_t k1 = (nxt[2] ? lon : lo) | (nxt[3] ? hin : hi);
                    const uint32_t f0 = __builtin_bit_cast(uint32_t, (__builtin_bit_cast(pss_u16x2, R0 ^ k0) * M) >> SH);
                    const uint32_t f1 = __builtin_bit_cast(uint32_t, (__builtin_bit_cast(pss_u16x2, R1 ^ k1) * M) >> SH);
                    const uint32_t t0 = L0 ^ f0, t1 = L1 ^ f1;
                    L0 = R0; R0 = t0;
                    L1 = R1; R1 = t1;
                }
                const uint32_t y[4] = {((L0 & 0xFFFFu) << h) | (R0 & 0xFFFFu), ((L0 >> 16) << h) | (R0 >> 16),
                                       ((L1 & 0xFFFFu) << h) | (R1 & 0xFFFFu), ((L1 >> 16) << h) | (R1 >> 16)};
#pragma unroll
                for (int j = 0; j < 4; j++) in[j] = ids.to_slot((wa + (nxt[j] ? 1u : 0u)) * B + y[j]);
            } else {
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    uint32_t Kl[kFeistelRounds];
#pragma unroll
                    for (int i = 0; i < kFeistelRounds; i++) Kl[i] = nxt[j] ? Kn[i] : Kc[i];
                    in[j] = ids.to_slot((wa + (nxt[j] ? 1u : 0u)) * B + feistel_once(pj[j], pl.hB, Kl));
                }
            }
            uint32_t vv[4];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                if constexpr (ORDERED) vv[j] = atomicExch(&buf[k[j]], in[j]);
                else vv[j] = xchg_unordered(buf, mark, k[j], in[j], true, lane);
            }
#pragma unroll
            for (int j = 0; j < 4; j++) put((int64_t)tb + j * G64, ids.from_slot(vv[j]));
            t_first += G256;
            pa += G256;
            while (pa >= B) { pa -= B; wa++; }
            u0 += 256u;
            continue;
        }
        // one iteration across a window boundary, partly valid or partly emitted
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const uint32_t u = u0 + 64u * j + (uint32_t)lane;
            const bool valid = u < uhi;
            const uint32_t t = t_first + c_lane + j * G64;
            uint32_t p = pa + c_lane + j * G64, w = wa;
            while (p >= B) { p -= B; w++; }
            uint32_t kk = 0u, in = 0u;
            if (valid) {
                kk = group_slot(pl.gr, grp, S, u, t, s0, s1);
                const uint32_t *kwl = ktr + kGKeyWin + kRoundKeyWords * (w - 1);
                uint32_t K[kFeistelRounds];
#pragma unroll
                for (int i = 0; i < kFeistelRounds; i++) K[i] = kwl[i];
                const bool lastw = w == pl.w_last;
                in = ids.to_slot(w * B + (lastw || pl.walk_full
                                              ? feistel(p, lastw ? pl.len_last : B, lastw ? pl.h_last : pl.hB, K)
                                              : feistel_once(p, pl.hB, K)));
            }
            uint32_t vv;
            if constexpr (ORDERED) vv = valid ? atomicExch(&buf[kk], in) : 0u;
            else vv = xchg_unordered(buf, mark, kk, in, valid, lane);
            if (valid && (int64_t)t >= pos_lo && (int64_t)t < pos_hi) put(t, ids.from_slot(vv));
        }
        t_first += G256;
        pa += G256;
        while (pa >= B) { pa -= B; wa++; }
        u0 += 256u;
    }
    if (drain) {
        // the group's final table is this wave's LDS: drain it in its tail order
        __syncthreads();
        uint32_t tk[kRoundKeyWords];
        round_keys8(g.key0, g.key1, grp, rank, DOM_V2_TAIL, tk);
        const uint32_t hS = feistel_half_bits(S);
        feistel_table(0u, S, S, hS, tk, lane, [&](uint32_t e, uint32_t s) {
            const int64_t pos = pl.T + group_tail_pos(pl.gr, grp, e);
            if (pos >= pos_lo && pos < pos_hi) put(pos, ids.from_slot(buf[s]));
        });
    }
}

// ------------------------------------------------------------------------------------------
// launcher
// ------------------------------------------------------------------------------------------
bool v2_grouped(const Geometry &g) { return (g.B < g.ns ? g.B : g.ns) > (int64_t)kLdsSlotMax; }

int64_t v2_grp_tiles(const Geometry &g, int32_t nr) { return gplan(g, nr, gcus()).tiles; }

// VAL ring buffer: key table (nr * kt_stride) then the per-tile last-occurrence tables
size_t v2_grp_val_bytes(const Geometry &g, int32_t nr) {
    const GPlan p = gplan(g, nr, gcus());
    const size_t words = (size_t)nr * (size_t)p.kt_stride +
                         (size_t)nr * p.gr.G * (size_t)(p.tiles - 1) * p.Smax;
    return words * sizeof(uint32_t);
}

hipError_t launch_v2_grp(const Geometry &g, const RankDesc *ranks, int32_t rank_lo, int32_t nr,
                         int64_t pos_lo, int64_t count, int64_t *out, uint32_t *VALws,
                         hipStream_t s, const Marker &mk, bool ordered, int stage,
                         const RankArgs *rank_args, const MapArgs *mapped) {
    if (mapped && !ordered) return hipErrorNotSupported;
    const int64_t pos_hi = pos_lo + count < g.ns ? pos_lo + count : g.ns;
    if (nr <= 0 || pos_hi <= pos_lo) return hipSuccess;
    const GPlan pl = gplan(g, nr, gcus());
    const bool do_pre = stage != V2_STAGE_EMIT, do_emit = stage != V2_STAGE_PRE;
    uint32_t *KT = VALws;
    uint32_t *VAL = VALws + (size_t)nr * (size_t)pl.kt_stride;
    if (do_pre) {
        mk(K_V2_LASTOCC, s);
        const int64_t items = pl.W + 2;
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
    mk(K_V2_EMIT, s);
    const dim3 grid((uint32_t)((int64_t)nr * pl.gr.G * pl.tiles));
    // LDS padded so that a CU takes exactly 8 waves (2 per SIMD, balanced) instead of 9
    size_t lds = (size_t)pl.Smax * 4 + (ordered ? 0 : (size_t)pl.Smax) + 16;
    if (lds * 9 <= 160 * 1024) lds = 160 * 1024 / 9 + 16;
    const int dt = need_tail ? 1 : 0;
    RankArgs ra;
    const int use_ra = rank_args ? 1 : 0;
    if (rank_args) ra = *rank_args;
    const bool packed = feistel_packed_ok(pl.hB);   // grouped pools: B > 16384, so hB >= 8
    const bool pow2 = pl.gr.r == 0 && (pl.gr.q & (pl.gr.q - 1u)) == 0u;   // every group 2^b slots
    const MapArgs ma = mapped ? *mapped : MapArgs{};
#define PSS_GE(O, N, PK, P2) do { if (mapped) hipLaunchKernelGGL((k_g_emit<true, N, PK, P2, true>), grid, dim3(64), lds, s, g, pl, \
                                                                     ranks, rank_lo, (const uint32_t *)KT, (const uint32_t *)VAL, dt, \
                                                                     pos_lo, count, out, ra, use_ra, ma); \
                                  else hipLaunchKernelGGL((k_g_emit<O, N, PK, P2>), grid, dim3(64), lds, s, g, pl, ranks, \
                                                          rank_lo, (const uint32_t *)KT, (const uint32_t *)VAL, dt, pos_lo, count, \
                                                          out, ra, use_ra, ma); } while (0)
#define PSS_GE2(O, N) do { if (packed && pow2) PSS_GE(O, N, true, true); else if (packed) PSS_GE(O, N, true, false); \
                           else if (pow2) PSS_GE(O, N, false, true); else PSS_GE(O, N, false, false); } while (0)
    if (ordered && narrow) PSS_GE2(true, true);
    else if (ordered) PSS_GE2(true, false);
    else if (narrow) PSS_GE2(false, true);
    else PSS_GE2(false, false);
#undef PSS_GE2
#undef PSS_GE
    mk(-1, s);
    return hipGetLastError();
}

hipError_t init_kernel_attributes_v2grp() {
    const int big = 160 * 1024;
    hipError_t e = hipSuccess;
#define PSS_ATTR(fn) { hipError_t x = hipFuncSetAttribute((const void *)(fn), hipFuncAttributeMaxDynamicSharedMemorySize, big); if (x != hipSuccess) e = x; }
    PSS_ATTR((k_g_emit<true, true, true, true>));
    PSS_ATTR((k_g_emit<true, true, true, false>));
    PSS_ATTR((k_g_emit<true, true, false, true>));
    PSS_ATTR((k_g_emit<true, true, false, false>));
    PSS_ATTR((k_g_emit<true, false, true, true>));
    PSS_ATTR((k_g_emit<true, false, true, false>));
    PSS_ATTR((k_g_emit<true, false, false, true>));
    PSS_ATTR((k_g_emit<true, false, false, false>));
    PSS_ATTR((k_g_emit<false, true, true, true>));
    PSS_ATTR((k_g_emit<false, true, true, false>));
    PSS_ATTR((k_g_emit<false, true, false, true>));
    PSS_ATTR((k_g_emit<false, true, false, false>));
    PSS_ATTR((k_g_emit<false, false, true, true>));
    PSS_ATTR((k_g_emit<false, false, true, false>));
    PSS_ATTR((k_g_emit<false, false, false, true>));
    PSS_ATTR((k_g_emit<false, false, false, false>));
    PSS_ATTR((k_g_emit<true, true, true, true, true>));
    PSS_ATTR((k_g_emit<true, true, true, false, true>));
    PSS_ATTR((k_g_emit<true, true, false, true, true>));
    PSS_ATTR((k_g_emit<true, true, false, false, true>));
    PSS_ATTR((k_g_emit<true, false, true, true, true>));
    PSS_ATTR((k_g_emit<true, false, true, false, true>));
    PSS_ATTR((k_g_emit<true, false, false, true, true>));
    PSS_ATTR((k_g_emit<true, false, false, false, true>));
    PSS_ATTR(k_g_lastocc);
#undef PSS_ATTR
    return e;
}

}  // namespace pss
