// pss_mt.h -- CPython 3.10 MT19937 on one wave (order mode PSS_ORDER_EXACT): seeding
// (`random_seed` -> init_by_array, _randommodule.c), the twist in LDS, tempering, and a
// speculative reader that turns the word stream into `_randbelow(n)` draws (random.py:239-249)
// 64 words at a time.  Shared by pss_v1exact.hip and pss_v2exact.hip.
#pragma once
#include <type_traits>

#include "pss_device.h"

namespace pss {
namespace {
constexpr int kMtN = 624, kMtM = 397;

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
// lane L of v := s (a scalar): v_writelane_b32 (no clang builtin in this toolchain)
template <int L>
__device__ __forceinline__ uint32_t write_lane(uint32_t v, uint32_t s) {
    __asm__ volatile("v_writelane_b32 %0, %1, %2" : "+v"(v) : "s"(s), "n"(L));
    return v;
}

template <int L0, int Lend, class F>
__device__ __forceinline__ void unroll_lanes(F &&f) {
    if constexpr (L0 < Lend) {
        f(std::integral_constant<int, L0>{});
        unroll_lanes<L0 + 1, Lend>(f);
    }
}

__device__ void mt_seed(uint32_t *mt, uint32_t key0, uint32_t key1, int klen) {
    const int lane = threadIdx.x & 63;
    // Both chains run on scalar registers; each 64 results are collected into one VGPR with
    // v_writelane (lane = step within the group) and stored with a single LDS write.
    // loop 1: k = 0..622 at i = k + 1, then the wrap (mt[0] = mt[623]) and k = 623 at i = 1;
    // step k adds key[k % klen] + k % klen.  init_genrand(19650218)'s words g are generated
    // alongside (an independent chain, cheaper than a scalar-cache load per step).
    const uint32_t add_even = key0, add_odd = klen == 2 ? key1 + 1u : key0;
    uint32_t g = 19650218u;
    uint32_t prev = g;
    uint32_t first = 0;
    for (int i0 = 1; i0 < kMtN; i0 += 64) {
        uint32_t vec = 0;
        unroll_lanes<0, 64>([&](auto lc) {
            constexpr int l = decltype(lc)::value;
            const int i = i0 + l;
            if (i < kMtN) {
                g = 1812433253u * (g ^ (g >> 30)) + (uint32_t)i;
                const uint32_t v = (g ^ ((prev ^ (prev >> 30)) * 1664525u)) + (((i - 1) & 1) ? add_odd : add_even);
                vec = write_lane<l>(vec, v);
                prev = v;
            }
        });
        if (i0 == 1) first = (uint32_t)__builtin_amdgcn_readlane((int)vec, 0);
        if (i0 + lane < kMtN) mt[i0 + lane] = vec;
    }
    {   // k = 623: i = 1 again, prev = mt[0] = mt[623]; 623 is odd
        const uint32_t v = (first ^ ((prev ^ (prev >> 30)) * 1664525u)) + add_odd;
        if (lane == 0) mt[1] = v;
        prev = v;
    }
    wave_lds_order();
    // loop 2: i = 2..623, wrap, i = 1; 623 steps.  mt[i] (loop-1 values) come from LDS in
    // 64-word vectors read ahead of the chain.
    for (int i0 = 2; i0 < kMtN; i0 += 64) {
        const uint32_t vin = (i0 + lane < kMtN) ? mt[i0 + lane] : 0u;
        uint32_t vec = 0;
        unroll_lanes<0, 64>([&](auto lc) {
            constexpr int l = decltype(lc)::value;
            const int i = i0 + l;
            if (i < kMtN) {
                const uint32_t old = (uint32_t)__builtin_amdgcn_readlane((int)vin, l);
                const uint32_t v = (old ^ ((prev ^ (prev >> 30)) * 1566083941u)) - (uint32_t)i;
                vec = write_lane<l>(vec, v);
                prev = v;
            }
        });
        if (i0 + lane < kMtN) mt[i0 + lane] = vec;
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

namespace {
// seed(a) for an int a: key = the 32-bit words of abs(a) (random_seed), |a| < 2^64
__device__ __forceinline__ void mt_seed_int(uint32_t *mt, int64_t a) {
    const uint64_t m = a < 0 ? (uint64_t)(-(a + 1)) + 1u : (uint64_t)a;
    const uint32_t k0 = (uint32_t)m, k1 = (uint32_t)(m >> 32);
    mt_seed(mt, k0, k1, k1 ? 2 : 1);
}

// Draws d = 0 .. nd-1 of a freshly seeded stream: draw d is _randbelow(bound(d)) (bound >= 1),
// handed to emit(d, r).  Words come 64 at a time; lane l of a block assumes it serves draw
// d0 + l - R_l (R_l = rejections among lower lanes) and the block iterates R to the fixed
// point -- lane l is final after l passes, a block settles in ~5.  One wave.
// One 64-word block of mt_draws at draw index d0 (the lanes = the block's words, nval of them):
// the fixed point above; returns the draws the block made.
template <class Bound, class Emit>
__device__ __forceinline__ uint32_t draw_block(uint32_t word, int nval, uint32_t d0, uint32_t nd, Bound &bound,
                                               Emit &emit) {
    const int lane = threadIdx.x & 63;
    uint32_t R = 0, d, r;
    bool acc;
    for (;;) {
        d = d0 + (uint32_t)lane - R;
        const bool valid = lane < nval && d < nd;
        const uint32_t n = valid ? bound(d) : 2u;
        const uint32_t k = 32u - (uint32_t)__builtin_clz(n);   // n.bit_length()
        r = word >> (32u - k);
        acc = valid && r < n;
        const uint64_t rej = __ballot(valid && !acc);
        const uint32_t Rn = (uint32_t)__popcll(rej & lanemask_lt());
        if (__ballot(Rn != R) == 0) break;
        R = Rn;
    }
    if (acc) emit(d, r);
    return (uint32_t)__popcll(__ballot(acc));
}

template <class Bound, class Emit>
__device__ void mt_draws(uint32_t *mt, uint32_t nd, Bound bound, Emit emit) {
    const int lane = threadIdx.x & 63;
    uint32_t d0 = 0;
    while (d0 < nd) {
        mt_twist(mt);
        for (int q0 = 0; q0 < kMtN && d0 < nd; q0 += 64) {
            const int nval = kMtN - q0 < 64 ? kMtN - q0 : 64;
            const uint32_t word = lane < nval ? mt_temper(mt[q0 + lane]) : 0u;
            d0 += draw_block(word, nval, d0, nd, bound, emit);
        }
    }
}

// Draws of one V2 pool2 window's stream (V2:101-106): k1 = _randbelow(P) and k2 =
// _randbelow(W - j) alternating, k1 first, until W k2 draws are made; emit(false, i, r) for the
// i-th k1, emit(true, j, r) for the j-th k2.  mt_draws's fixed point re-derives every lane's
// draw index after each pass, and with two alternating bounds one rejection flips the role of
// every later lane, so a block settles only after about as many passes as it has rejections.
// Here the roles come from a 2-state automaton instead: lane l maps the role it is offered
// (0 = k1, 1 = k2) to the role the next lane is offered (f(0) = accepted as k1 ? 1 : 0, f(1) =
// accepted as k2 ? 0 : 1), and an inclusive DPP scan of the composed maps gives every lane its
// role in one pass.  Only the k2 bound depends on the lane's k2 index j, and only through values
// within a few counts of a threshold: the block guesses j, derives the roles and the true j, and
// repeats until no guess changes (almost always after two passes).
// A map of the two roles is either a constant or "xor k": encoded as (const << 1) | k, where k =
// its image of role 0 (so the identity is 0).  g after f: g if g is constant, else f with its k
// flipped by g's -- two VALU ops and a select, where the table form took eight.
__device__ __forceinline__ uint32_t role_compose(uint32_t g, uint32_t f) {   // g after f
    // g ^ (g constant ? 0 : f): the constant flag sign-extended into a mask (v_bfe_i32), then
    // one v_bitop3 (table 0xB4 = S0 ^ (S1 & ~S2)); in plain C hipcc folds it back into a
    // compare and a select
    uint32_t cm, r;
    asm("v_bfe_i32 %0, %1, 1, 1" : "=v"(cm) : "v"(g));
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xb4" : "=v"(r) : "v"(g), "v"(f), "v"(cm));
    return r;
}
__device__ __forceinline__ uint32_t role_apply(uint32_t h, uint32_t s) {
    return (h & 2u) ? (h & 1u) : (s ^ (h & 1u));
}
template <int CTRL, int ROWMASK>
__device__ __forceinline__ uint32_t dpp_role(uint32_t x) {
    // lanes without a source (or in masked rows) read the identity map (0): bound_ctrl zero-fill
    // for the row shifts, the pre-set old value for the masked broadcast rows
    if constexpr (ROWMASK == 0xF) return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, 0xF, 0xF, true);
    else return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, ROWMASK, 0xF, false);
}
// lane l - 1's value (lane 0: 0) by a DPP wave shift, where a shuffle takes an LDS round trip
__device__ __forceinline__ uint32_t wave_prev_lane(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x138, 0xF, 0xF, true);   // wave_shr:1
}
__device__ __forceinline__ uint32_t wave_role_scan(uint32_t x) {
    x = role_compose(x, dpp_role<0x111, 0xF>(x));
    x = role_compose(x, dpp_role<0x112, 0xF>(x));
    x = role_compose(x, dpp_role<0x114, 0xF>(x));
    x = role_compose(x, dpp_role<0x118, 0xF>(x));
    x = role_compose(x, dpp_role<0x142, 0xA>(x));
    x = role_compose(x, dpp_role<0x143, 0xC>(x));
    return x;
}

// One 64-word block of a pool2 window's stream, exactly (the wave's lanes = the block's words):
// the role scan settles it in one pass where every k2 verdict is fixed over the block's possible
// k2 indices (lane l: [i2, i2 + ceil(l / 2)]), else the lanes' k2 indices are guessed and re-derived to the fixed
// point.  Emits the block's draws and advances (st, i1, i2).
template <class Emit>
__device__ __forceinline__ void pair_block(uint32_t word, bool valid, uint32_t W, uint32_t P, uint32_t kb1,
                                           uint32_t &st, uint32_t &i1, uint32_t &i2, Emit &emit) {
    const int lane = threadIdx.x & 63;
    const uint64_t below = lanemask_lt();
    const uint32_t r1 = word >> (32u - kb1);
    const bool a1 = valid && r1 < P;
    uint32_t j = 0, r2 = 0, role = 0, Fx = 0;
    bool a2 = false;
    // one scan of the role maps for the k2 verdicts a2 (at k2 indices jg); returns the lanes'
    // true k2 indices in j
    auto pass = [&](uint32_t n2, uint32_t rr) {
        r2 = rr;
        a2 = valid && rr < n2;
        // offered k1: accepted -> k2 next, else k1; offered k2: accepted -> k1, else k2
        const uint32_t f = ((a1 != a2) ? 2u : 0u) | (a1 ? 1u : 0u);
        Fx = wave_role_scan(f);
        const uint32_t Fp = wave_prev_lane(Fx);
        role = lane ? role_apply(Fp, st) : st;
        const uint64_t m2 = __ballot(valid && role == 1u && a2);
        j = i2 + (uint32_t)__popcll(m2 & below);
    };
    // an accepted k2 is followed by a k1 offer, so the lanes below l hold at most ceil(l / 2)
    // accepted k2 draws and lane l's k2 index lies in [i2, i2 + ceil(l / 2)]: where every lane's
    // k2 verdict is the same over its range (all but ~0.5 % of lanes), one scan settles the block;
    // otherwise iterate guess -> true index
    const uint32_t jl = i2 + ((uint32_t)lane + 1u) / 2u;
    const uint32_t nhi = i2 < W ? W - i2 : 1u, nlo = jl < W ? W - jl : 1u;
    const uint32_t kbh = 32u - (uint32_t)__builtin_clz(nhi);
    const uint32_t rh = word >> (32u - kbh);
    const bool sure = kbh == 32u - (uint32_t)__builtin_clz(nlo) && (rh < nlo || rh >= nhi);
    if (__ballot(valid && !sure) == 0) {
        pass(nlo, rh);
    } else {
        uint32_t jg = i2 + (uint32_t)lane / 3u;
        for (;;) {
            const uint32_t n2 = jg < W ? W - jg : 1u;
            pass(n2, word >> (32u - (32u - (uint32_t)__builtin_clz(n2))));
            if (__ballot(valid && j != jg) == 0) break;
            jg = j;
        }
    }
    const bool acc = valid && (role ? a2 : a1);
    const uint64_t m1 = __ballot(acc && role == 0u), m2 = __ballot(acc && role == 1u);
    if (acc) {
        if (role == 0u) {
            const uint32_t i = i1 + (uint32_t)__popcll(m1 & below);
            if (i < W) emit(false, i, r1);
        } else if (j < W) {
            emit(true, j, r2);
        }
    }
    i1 += (uint32_t)__popcll(m1);
    i2 += (uint32_t)__popcll(m2);
    st = role_apply((uint32_t)__builtin_amdgcn_readlane((int)Fx, 63), st);
}

template <class Emit>
__device__ void mt_draws_pair(uint32_t *mt, uint32_t W, uint32_t P, Emit emit) {
    const int lane = threadIdx.x & 63;
    const uint32_t kb1 = 32u - (uint32_t)__builtin_clz(P);
    uint32_t i1 = 0, i2 = 0, st = 0;   // k1 / k2 draws made, role offered to the next word
    while (i2 < W) {
        mt_twist(mt);
        for (int q0 = 0; q0 < kMtN && i2 < W; q0 += 64) {
            const int nval = kMtN - q0 < 64 ? kMtN - q0 : 64;
            const bool valid = lane < nval;
            const uint32_t word = valid ? mt_temper(mt[q0 + lane]) : 0u;
            pair_block(word, valid, W, P, kb1, st, i1, i2, emit);
        }
    }
}

// The same draws on a workgroup of kMtWgThreads (16 waves) per stream, for long windows (C5's
// pool2 windows are 2^20 steps and there are only ~11 per rank: one wave per stream left most of
// the chip idle).  The stream is consumed in ROUNDS of kMtRound twists (kMtRound * 624 words);
// one wave -- the generator, the last -- twists and tempers the NEXT round into the other half
// of a double-buffered ring (three dependent 227-word steps per twist, in program order inside
// the wave: no barrier), while the other fifteen consume the current round in three
// barrier-separated phases:
//   summaries  each 64-word block of the round, wave w taking blocks w, w + 15, ...: where every
//              verdict of the block is fixed over the index window its start can lie in, its
//              transfer -- V2: the composed role map and the k1 / k2 acceptances for either start
//              role; V1: the draws it makes -- comes from one role scan (a popcount) without knowing
//              where the block starts.  The window is the expected index at the block's word offset
//              (the round's acceptance rate) +- 6 standard deviations, clipped to what is possible
//              at all; a start outside it only costs the block its shortcut
//   combine    wave 0 walks the round's blocks in order: a settled block whose true start lies in
//              its window is one transfer, any other block runs exactly (pair_block / draw_block,
//              which emit) -- where round 3 ran every block after the first unsettled one exactly
//   emit       each wave emits its settled blocks from their now known start states.
// Three barriers per round where round 3 took three per twist, and the combine a prefix scan per
// run of settled blocks: C5 V2 exact draws 14.2 -> 11.5 ms.  Rounds of 4 / 6 / 8 / 10 twists and
// window margins of 4 / 6 sd, same box: 11.75 / 11.5 / 11.75 / 15.8 ms at 4 sd, 12.4 ms at 6 sd
// with 8 twists (profiles/r04/mt_ab/, tools/stamp_mt.hip): what is left is per-block work on
// the stream's one CU -- ~160 clocks per 64-word block in the summaries, ~135 in the combine
// (the blocks run exactly: the last ~3 % of a window, where k2's bound is small), ~115 in emit.
// 16 waves (15 consumers, 4 blocks each per round) against 10 (9, 7): C5 exact V2 24.6 -> 22.5 ms,
// 12 waves 23.3 ms, same box (round 4, profiles/r04/ab_mt_waves/).
#ifndef PSS_MT_WG_THREADS
#define PSS_MT_WG_THREADS 1024
#endif
constexpr int kMtWgThreads = PSS_MT_WG_THREADS;   // consumer waves and the generator (the last)
constexpr int kMtBlocks = (kMtN + 63) / 64;   // 10 per twist: nine of 64 words, one of 48
constexpr int kMtWgWaves = kMtWgThreads / 64;
#ifndef PSS_MT_ROUND
#define PSS_MT_ROUND 6
#endif
#ifndef PSS_MT_SD
#define PSS_MT_SD 4
#endif
constexpr int kMtRound = PSS_MT_ROUND;                    // twists per round (even)
constexpr int kMtRoundWords = kMtRound * kMtN;
constexpr int kMtRoundBlocks = kMtRound * kMtBlocks;      // 60
constexpr int kMtConsumers = kMtWgWaves - 1;
constexpr int kMtPerWave = (kMtRoundBlocks + kMtConsumers - 1) / kMtConsumers;   // 7
static_assert(kMtRound % 2 == 0, "the generator's state buffer returns to mt[cur] after a round");
static_assert(kMtRoundBlocks <= 128, "the combiner keeps the summaries in two lanes sets");

constexpr int kMtTwPad = kMtN * kMtWgWaves > 2 * kMtRoundWords ? kMtN * kMtWgWaves - 2 * kMtRoundWords : 1;
struct MtWgShared {
    uint32_t mt[2][kMtN];                 // generator state, double-buffered across a twist
    uint32_t tw[2][kMtRoundWords];        // tempered words: the round consumed, the next one
    uint32_t tw_pad[kMtTwPad];            // (V2 tail blocks: one MT state per wave from tw on)
    uint32_t sum[kMtRoundBlocks][6];      // settled?, role map | draws, c1(0), c1(1), c2(0), c2(1)
    uint32_t win[kMtRoundBlocks][2];      // index window [lo, hi] the block's summary assumed
    uint32_t start[kMtRoundBlocks][4];    // (st, i1, i2) or (d) at each block's start; [3] = 1:
                                          // handled by the combiner (ran exactly, or past the end)
    uint32_t state[4];                    // st, i1, i2 | d
};

// diagnostic build only (-DPSS_MT_STAMPS, tools/stamp_mt.hip): per-workgroup clock sums of the
// round phases -- [0..2] summaries / combine / emit (wave 0, barrier to barrier), [3..5] the
// generator's share of each phase, [6] blocks run exactly, [7] rounds
#ifdef PSS_MT_STAMPS
__device__ uint64_t pss_mt_stamps[4096][8];
#define PSS_MT_T(v) const uint64_t v = __builtin_amdgcn_s_memtime()
#define PSS_MT_ADD(slot_, val_) do { if ((threadIdx.x & 63) == 0 && blockIdx.x < 4096u) pss_mt_stamps[blockIdx.x][slot_] += (val_); } while (0)
#else
#define PSS_MT_T(v) do { } while (0)
#define PSS_MT_ADD(slot_, val_) do { } while (0)
#endif

// generator wave: step p (0..2) of one twist, o -> nw, tempered words into tw: new[k] for k in
// [227 p, 227 p + 227) (new[k] needs new[k - 227] from k = 227 on), 64 lanes x 4
__device__ __forceinline__ void mt_gen_step(const uint32_t *o, uint32_t *nw, uint32_t *tw, int p, int lane) {
    constexpr int D = kMtN - kMtM;   // 227
    uint32_t v[4];
#pragma unroll
    for (int it = 0; it < 4; it++) {
        const int tt = lane + 64 * it, k = tt + D * p;
        v[it] = 0u;
        if (tt < D && k < kMtN) {
            if (p == 0) v[it] = mt_twist_word(o[k], o[k + 1], o[k + kMtM]);
            else if (k < kMtN - 1) v[it] = mt_twist_word(o[k], o[k + 1], nw[k - D]);
            else v[it] = mt_twist_word(o[kMtN - 1], nw[0], nw[kMtM - 1]);
        }
    }
#pragma unroll
    for (int it = 0; it < 4; it++) {
        const int tt = lane + 64 * it, k = tt + D * p;
        if (tt < D && k < kMtN) {
            nw[k] = v[it];
            tw[k] = mt_temper(v[it]);
        }
    }
    wave_lds_order();
}

// steps [s_lo, s_hi) of a round's 3 kMtRound twist steps, the round's words into tw (generator
// wave only; the round starts from mt[cur] and, kMtRound being even, ends there)
__device__ __forceinline__ void mt_gen_round(MtWgShared &sh, int cur, uint32_t *tw, int s_lo, int s_hi,
                                             int lane) {
    for (int s = s_lo; s < s_hi; s++) {
        const int t = s / 3, p = s - 3 * t, c = cur ^ (t & 1);
        mt_gen_step(sh.mt[c], sh.mt[c ^ 1], tw + t * kMtN, p, lane);
    }
}

// block b of a round: its first word and valid words
__device__ __forceinline__ int mt_block_q0(int b) { return (b / kMtBlocks) * kMtN + 64 * (b % kMtBlocks); }
__device__ __forceinline__ int mt_block_nval(int b) { return b % kMtBlocks == kMtBlocks - 1 ? kMtN - 64 * (kMtBlocks - 1) : 64; }

// index window of a block's start: x0 + the expected count at word offset wb (rate per word) +-
// 6 sd + 8 (var = the count's variance per word), clipped to [x0, x0 + cap(wb)] (what the words
// before it can reach at all)
__device__ __forceinline__ void mt_window(uint32_t x0, float rate, float var, uint32_t wb, uint32_t cap,
                                          uint32_t &lo, uint32_t &hi) {
    const float e = rate * (float)wb;
    const float m = (float)PSS_MT_SD * __builtin_sqrtf(var * (float)wb + 1.0f) + 8.0f;
    const float l = e - m, h = e + m;
    lo = x0 + (l > 0.0f ? (uint32_t)l : 0u);
    const uint32_t hh = (uint32_t)h + 1u;
    hi = x0 + (hh < cap ? hh : cap);
    if (lo > hi) lo = hi;
}

template <class Emit>
__device__ void mt_draws_pair_wg(MtWgShared &sh, int cur, uint32_t W, uint32_t P, Emit emit) {
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const bool gen = wv == kMtWgWaves - 1;
    const uint32_t kb1 = 32u - (uint32_t)__builtin_clz(P);
    const uint64_t below = lanemask_lt();
    const float acc1 = (float)P / (float)(1ull << kb1);
    if (tid == 0) { sh.state[0] = 0u; sh.state[1] = 0u; sh.state[2] = 0u; }
    if (gen) mt_gen_round(sh, cur, sh.tw[0], 0, 3 * kMtRound, lane);
    __syncthreads();
    for (int rs = 0;; rs ^= 1) {
        if (sh.state[2] >= W) break;   // (uniform: read after a barrier)
        PSS_MT_T(t0);
        const uint32_t *tc = sh.tw[rs];
        uint32_t *tn = sh.tw[rs ^ 1];
        // ---- summaries (consumers) | the next round's first third (generator)
        const uint32_t i2_0 = sh.state[2];
        const uint32_t n2_0 = i2_0 < W ? W - i2_0 : 1u;
        const float acc2 = (float)n2_0 / (float)(1ull << (32u - (uint32_t)__builtin_clz(n2_0)));
        // k2 draws per word: a step takes Geom(acc1) + Geom(acc2) words, so over w words the
        // count has mean w / E and variance ~ w Var / E^3 (renewal process)
        const float Ex = 1.0f / acc1 + 1.0f / acc2;
        const float Vx = (1.0f - acc1) / (acc1 * acc1) + (1.0f - acc2) / (acc2 * acc2);
        const float rate = 1.0f / Ex, var = Vx / (Ex * Ex * Ex);
        uint32_t Fkeep[kMtPerWave];
        bool a1k[kMtPerWave], a2k[kMtPerWave];
        if (gen) {
            mt_gen_round(sh, cur, tn, 0, kMtRound, lane);
            PSS_MT_T(tg); PSS_MT_ADD(3, tg - t0);
        } else {
#pragma unroll
            for (int s = 0; s < kMtPerWave; s++) {
                Fkeep[s] = 0u; a1k[s] = false; a2k[s] = false;
                const int b = wv + kMtConsumers * s;
                if (b >= kMtRoundBlocks) break;
                const int q0 = mt_block_q0(b), nval = mt_block_nval(b);
                const bool valid = lane < nval;
                const uint32_t word = valid ? tc[q0 + lane] : 0u;
                const bool a1 = valid && (word >> (32u - kb1)) < P;
                uint32_t jlo, jhi;   // the k2 index at the block's start (at most 1 per 2 words)
                mt_window(i2_0, rate, var, (uint32_t)q0, (uint32_t)q0 / 2u + 1u, jlo, jhi);
                const uint32_t jtop = jhi + ((uint32_t)lane + 1u) / 2u;   // (pair_block's per-lane range)
                const uint32_t nhi = jlo < W ? W - jlo : 1u, nlo = jtop < W ? W - jtop : 1u;
                const uint32_t kbh = 32u - (uint32_t)__builtin_clz(nhi);
                const uint32_t rh = word >> (32u - kbh);
                const bool sure = kbh == 32u - (uint32_t)__builtin_clz(nlo) && (rh < nlo || rh >= nhi);
                const bool settled = __ballot(valid && !sure) == 0;
                if (settled) {
                    const bool a2 = valid && rh < nlo;
                    const uint32_t Fx = wave_role_scan(((a1 != a2) ? 2u : 0u) | (a1 ? 1u : 0u));
                    const uint32_t Fp = wave_prev_lane(Fx);
                    uint32_t c[4];
#pragma unroll
                    for (uint32_t s0 = 0; s0 < 2; s0++) {
                        const uint32_t role = lane ? role_apply(Fp, s0) : s0;
                        const bool acc = valid && (role ? a2 : a1);
                        c[s0] = (uint32_t)__popcll(__ballot(acc && role == 0u));
                        c[2 + s0] = (uint32_t)__popcll(__ballot(acc && role == 1u));
                    }
                    const uint32_t F63 = (uint32_t)__shfl((int)Fx, 63);   // (all lanes: a shuffle reads active lanes)
                    if (lane == 0) {
                        sh.sum[b][0] = 1u; sh.sum[b][1] = F63;
                        sh.sum[b][2] = c[0]; sh.sum[b][3] = c[1]; sh.sum[b][4] = c[2]; sh.sum[b][5] = c[3];
                        sh.win[b][0] = jlo; sh.win[b][1] = jhi;
                    }
                    Fkeep[s] = Fp; a1k[s] = a1; a2k[s] = a2;
                } else if (lane == 0) {
                    sh.sum[b][0] = 0u;
                }
            }
        }
        __syncthreads();
        PSS_MT_T(t1);
        if (wv == 0) PSS_MT_ADD(0, t1 - t0);
        // ---- combine (wave 0) | second third
        if (gen) {
            mt_gen_round(sh, cur, tn, kMtRound, 2 * kMtRound, lane);
            PSS_MT_T(tg); PSS_MT_ADD(4, tg - t1);
        } else if (wv == 0) {
            // the round's blocks in order, 64 at a time (lane = block): an inclusive scan of the
            // settled blocks' transfers from the first unresolved block f gives every block's
            // start; the blocks up to the first one that is unsettled or whose start falls outside
            // its window take their starts from it, that block runs exactly, and the scan resumes
            // after it
            uint32_t st = sh.state[0], i1 = sh.state[1], i2 = sh.state[2];
            bool fin = false;   // past the stream's end
            for (int h = 0; h < 2 && !fin; h++) {
                const int b = 64 * h + lane;
                const bool inb = b < kMtRoundBlocks;
                const uint32_t vs = inb ? sh.sum[b][0] : 0u;
                uint32_t F = 0u, a0 = 0u, a1 = 0u, c0 = 0u, c1 = 0u, lo = 0u, hi = 0u;
                if (vs) {
                    F = sh.sum[b][1]; a0 = sh.sum[b][2]; a1 = sh.sum[b][3];
                    c0 = sh.sum[b][4]; c1 = sh.sum[b][5]; lo = sh.win[b][0]; hi = sh.win[b][1];
                }
                const int nb = kMtRoundBlocks - 64 * h < 64 ? kMtRoundBlocks - 64 * h : 64;
                int f = 0;
                while (f < nb) {
                    // transfer of lane l (identity below f): (role map, k1 / k2 draws per start role)
                    uint32_t tF = lane >= f && vs ? F : 0u;
                    uint32_t t10 = lane >= f && vs ? a0 : 0u, t11 = lane >= f && vs ? a1 : 0u;
                    uint32_t t20 = lane >= f && vs ? c0 : 0u, t21 = lane >= f && vs ? c1 : 0u;
#pragma unroll
                    for (int d = 1; d < 64; d <<= 1) {   // inclusive scan: (earlier) then (this)
                        const uint32_t pF = (uint32_t)__shfl_up((int)tF, d), p10 = (uint32_t)__shfl_up((int)t10, d);
                        const uint32_t p11 = (uint32_t)__shfl_up((int)t11, d), p20 = (uint32_t)__shfl_up((int)t20, d);
                        const uint32_t p21 = (uint32_t)__shfl_up((int)t21, d);
                        if (lane >= d) {
                            const uint32_t q0 = role_apply(pF, 0u), q1 = role_apply(pF, 1u);
                            const uint32_t n10 = p10 + (q0 ? t11 : t10), n11 = p11 + (q1 ? t11 : t10);
                            const uint32_t n20 = p20 + (q0 ? t21 : t20), n21 = p21 + (q1 ? t21 : t20);
                            tF = role_compose(tF, pF);
                            t10 = n10; t11 = n11; t20 = n20; t21 = n21;
                        }
                    }
                    // exclusive prefix -> each lane's start state
                    const uint32_t eF = (uint32_t)__shfl_up((int)tF, 1), e10 = (uint32_t)__shfl_up((int)t10, 1);
                    const uint32_t e11 = (uint32_t)__shfl_up((int)t11, 1), e20 = (uint32_t)__shfl_up((int)t20, 1);
                    const uint32_t e21 = (uint32_t)__shfl_up((int)t21, 1);
                    const bool first = lane == 0;
                    const uint32_t sst = first ? st : role_apply(eF, st);
                    const uint32_t si1 = i1 + (first ? 0u : (st ? e11 : e10));
                    const uint32_t si2 = i2 + (first ? 0u : (st ? e21 : e20));
                    const bool ok = lane >= f && lane < nb && vs && si2 < W && si2 >= lo && si2 <= hi;
                    const uint64_t bad = __ballot(lane >= f && lane < nb && !ok);
                    const int g = bad ? __ffsll((long long)bad) - 1 : nb;
                    if (lane >= f && lane < g) {
                        sh.start[b][0] = sst; sh.start[b][1] = si1; sh.start[b][2] = si2; sh.start[b][3] = 0u;
                    }
                    if (g >= nb) {   // every block through: the state after the set's last block
                        const int e = nb - 1;
                        const uint32_t lF = (uint32_t)__builtin_amdgcn_readlane((int)tF, e);
                        const uint32_t l10 = (uint32_t)__builtin_amdgcn_readlane((int)t10, e);
                        const uint32_t l11 = (uint32_t)__builtin_amdgcn_readlane((int)t11, e);
                        const uint32_t l20 = (uint32_t)__builtin_amdgcn_readlane((int)t20, e);
                        const uint32_t l21 = (uint32_t)__builtin_amdgcn_readlane((int)t21, e);
                        i1 += st ? l11 : l10;
                        i2 += st ? l21 : l20;
                        st = role_apply(lF, st);
                        break;
                    }
                    // the state at block g's start
                    st = (uint32_t)__builtin_amdgcn_readlane((int)sst, g);
                    i1 = (uint32_t)__builtin_amdgcn_readlane((int)si1, g);
                    i2 = (uint32_t)__builtin_amdgcn_readlane((int)si2, g);
                    // block g: past the stream's end (so is every block after it), or run exactly
                    const int bg = 64 * h + g;
                    if (i2 >= W) {
                        for (int r = bg + lane; r < kMtRoundBlocks; r += 64) {
                            sh.start[r][0] = st; sh.start[r][1] = i1; sh.start[r][2] = i2; sh.start[r][3] = 1u;
                        }
                        fin = true;
                        break;
                    }
                    if (lane == 0) {
                        sh.start[bg][0] = st; sh.start[bg][1] = i1; sh.start[bg][2] = i2; sh.start[bg][3] = 1u;
                    }
                    PSS_MT_ADD(6, 1);
                    const int q0 = mt_block_q0(bg), nval = mt_block_nval(bg);
                    const bool valid = lane < nval;
                    pair_block(valid ? tc[q0 + lane] : 0u, valid, W, P, kb1, st, i1, i2, emit);
                    f = g + 1;
                }
            }
            if (lane == 0) { sh.state[0] = st; sh.state[1] = i1; sh.state[2] = i2; }
        }
        __syncthreads();
        PSS_MT_T(t2);
        if (wv == 0) PSS_MT_ADD(1, t2 - t1);
        // ---- emit the settled blocks the combiner only chained | last third
        if (gen) {
            mt_gen_round(sh, cur, tn, 2 * kMtRound, 3 * kMtRound, lane);
            PSS_MT_T(tg); PSS_MT_ADD(5, tg - t2);
        } else {
#pragma unroll
            for (int s = 0; s < kMtPerWave; s++) {
                const int b = wv + kMtConsumers * s;
                if (b >= kMtRoundBlocks) break;
                if (!sh.sum[b][0] || sh.start[b][3]) continue;
                const int q0 = mt_block_q0(b), nval = mt_block_nval(b);
                const bool valid = lane < nval;
                const uint32_t word = valid ? tc[q0 + lane] : 0u;
                const uint32_t st = sh.start[b][0], i1 = sh.start[b][1], i2 = sh.start[b][2];
                const uint32_t role = lane ? role_apply(Fkeep[s], st) : st;
                const bool acc = valid && (role ? a2k[s] : a1k[s]);
                const uint64_t m1 = __ballot(acc && role == 0u), m2 = __ballot(acc && role == 1u);
                if (acc) {
                    if (role == 0u) {
                        const uint32_t i = i1 + (uint32_t)__popcll(m1 & below);
                        if (i < W) emit(false, i, word >> (32u - kb1));
                    } else {
                        const uint32_t j = i2 + (uint32_t)__popcll(m2 & below);
                        const uint32_t jlo = sh.win[b][0];
                        const uint32_t nhi = jlo < W ? W - jlo : 1u;
                        if (j < W) emit(true, j, word >> (32u - (32u - (uint32_t)__builtin_clz(nhi))));
                    }
                }
            }
        }
        __syncthreads();
        PSS_MT_T(t3);
        if (wv == 0) { PSS_MT_ADD(2, t3 - t2); PSS_MT_ADD(7, 1); }
    }
}

// mt_draws on a workgroup per stream (V1 windows beyond LDS: ~12 windows per rank at C5), for a
// non-increasing bound(d), in the rounds of mt_draws_pair_wg: a block whose every verdict is
// fixed over the bounds of its window's draw indices (lane l: [lo, hi + l]) makes exactly
// popc(accepted) draws wherever in the window it starts.
template <class Bound, class Emit>
__device__ void mt_draws_wg(MtWgShared &sh, int cur, uint32_t nd, Bound bound, Emit emit) {
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const bool gen = wv == kMtWgWaves - 1;
    const uint64_t below = lanemask_lt();
    if (tid == 0) sh.state[0] = 0u;
    if (gen) mt_gen_round(sh, cur, sh.tw[0], 0, 3 * kMtRound, lane);
    __syncthreads();
    for (int rs = 0;; rs ^= 1) {
        if (sh.state[0] >= nd) break;
        const uint32_t *tc = sh.tw[rs];
        uint32_t *tn = sh.tw[rs ^ 1];
        const uint32_t d0 = sh.state[0];
        const uint32_t n0 = bound(d0);
        // draws per word: acceptance a; over w words the count is Binomial(w, a)
        const float rate = (float)n0 / (float)(1ull << (32u - (uint32_t)__builtin_clz(n0)));
        const float var = rate * (1.0f - rate);
        bool acck[kMtPerWave];
        uint32_t rk[kMtPerWave];
        if (gen) {
            mt_gen_round(sh, cur, tn, 0, kMtRound, lane);
        } else {
#pragma unroll
            for (int s = 0; s < kMtPerWave; s++) {
                acck[s] = false; rk[s] = 0u;
                const int b = wv + kMtConsumers * s;
                if (b >= kMtRoundBlocks) break;
                const int q0 = mt_block_q0(b), nval = mt_block_nval(b);
                const bool valid = lane < nval;
                const uint32_t word = valid ? tc[q0 + lane] : 0u;
                uint32_t dlo, dhi;
                mt_window(d0, rate, var, (uint32_t)q0, (uint32_t)q0, dlo, dhi);
                const uint32_t dtop = dhi + (uint32_t)lane;   // lane l: at most l draws below it
                const uint32_t nhi = bound(dlo < nd ? dlo : nd - 1u), nlo = bound(dtop < nd ? dtop : nd - 1u);
                const uint32_t kbh = 32u - (uint32_t)__builtin_clz(nhi);
                const uint32_t r = word >> (32u - kbh);
                const bool sure = kbh == 32u - (uint32_t)__builtin_clz(nlo) && (r < nlo || r >= nhi);
                if (__ballot(valid && !sure) == 0) {
                    const bool acc = valid && r < nlo;
                    const uint32_t cnt = (uint32_t)__popcll(__ballot(acc));
                    if (lane == 0) { sh.sum[b][0] = 1u; sh.sum[b][1] = cnt; sh.win[b][0] = dlo; sh.win[b][1] = dhi; }
                    acck[s] = acc;
                    rk[s] = r;
                } else if (lane == 0) {
                    sh.sum[b][0] = 0u;
                }
            }
        }
        __syncthreads();
        if (gen) {
            mt_gen_round(sh, cur, tn, kMtRound, 2 * kMtRound, lane);
        } else if (wv == 0) {
            // as in mt_draws_pair_wg: a prefix sum of the settled blocks' draw counts from the
            // first unresolved block, up to the first block that is unsettled or out of its window
            uint32_t d = sh.state[0];
            bool fin = false;
            for (int h = 0; h < 2 && !fin; h++) {
                const int b = 64 * h + lane;
                const bool inb = b < kMtRoundBlocks;
                const uint32_t vs = inb ? sh.sum[b][0] : 0u;
                uint32_t c = 0u, lo = 0u, hi = 0u;
                if (vs) { c = sh.sum[b][1]; lo = sh.win[b][0]; hi = sh.win[b][1]; }
                const int nb = kMtRoundBlocks - 64 * h < 64 ? kMtRoundBlocks - 64 * h : 64;
                int f = 0;
                while (f < nb) {
                    uint32_t t = lane >= f && vs ? c : 0u;
#pragma unroll
                    for (int dd = 1; dd < 64; dd <<= 1) {
                        const uint32_t p = (uint32_t)__shfl_up((int)t, dd);
                        if (lane >= dd) t += p;
                    }
                    const uint32_t sd = d + (t - (lane >= f && vs ? c : 0u));   // exclusive prefix
                    const bool ok = lane >= f && lane < nb && vs && sd < nd && sd >= lo && sd <= hi;
                    const uint64_t bad = __ballot(lane >= f && lane < nb && !ok);
                    const int g = bad ? __ffsll((long long)bad) - 1 : nb;
                    if (lane >= f && lane < g) { sh.start[b][0] = sd; sh.start[b][3] = 0u; }
                    if (g >= nb) {
                        d += (uint32_t)__builtin_amdgcn_readlane((int)t, nb - 1);
                        break;
                    }
                    d = (uint32_t)__builtin_amdgcn_readlane((int)sd, g);
                    const int bg = 64 * h + g;
                    if (d >= nd) {
                        for (int r = bg + lane; r < kMtRoundBlocks; r += 64) { sh.start[r][0] = d; sh.start[r][3] = 1u; }
                        fin = true;
                        break;
                    }
                    if (lane == 0) { sh.start[bg][0] = d; sh.start[bg][3] = 1u; }
                    const int q0 = mt_block_q0(bg), nval = mt_block_nval(bg);
                    d += draw_block(lane < nval ? tc[q0 + lane] : 0u, nval, d, nd, bound, emit);
                    f = g + 1;
                }
            }
            if (lane == 0) sh.state[0] = d;
        }
        __syncthreads();
        if (gen) {
            mt_gen_round(sh, cur, tn, 2 * kMtRound, 3 * kMtRound, lane);
        } else {
#pragma unroll
            for (int s = 0; s < kMtPerWave; s++) {
                const int b = wv + kMtConsumers * s;
                if (b >= kMtRoundBlocks) break;
                if (!sh.sum[b][0] || sh.start[b][3]) continue;
                const uint32_t d = sh.start[b][0] + (uint32_t)__popcll(__ballot(acck[s]) & below);
                if (acck[s] && d < nd) emit(d, rk[s]);
            }
        }
        __syncthreads();
    }
}

// ---- seeding many streams ahead of their draws ----------------------------------------------
// The wave-per-stream draw kernels used to seed in the wave itself: ~12K scalar instructions,
// and a CU's waves take turns on its scalar unit, so with several streams per CU the seeding
// was a large share of the launch.  k_mt_seed_streams instead runs init_by_array for
// kMtSeedLanes streams per wave, one per lane on vector registers, the loop-1 words of each in
// LDS for loop 2; the draw kernels then load the finished 624 words (mt_load).  Stream i's seed
// is epoch + zero_add for idx = first + i == 0, else epoch + (idx + off) * 10000 (V1:102,165-171:
// first = w_lo, off = 0, zero_add = 0; V2:107-109,147: first = 0, off = -1, zero_add = 2).
constexpr int kMtSeedLanes = 16;
constexpr int kMtSeedPitch = kMtSeedLanes + 1;   // LDS words per state word (conflict-free)

struct MtSeedSpec {
    int64_t epoch, first, off, zero_add;
    uint32_t n;   // streams
};

__device__ __forceinline__ int64_t mt_seed_of(const MtSeedSpec &sp, uint32_t i) {
    const int64_t idx = sp.first + (int64_t)i;
    return idx == 0 ? sp.epoch + sp.zero_add : sp.epoch + (idx + sp.off) * 10000;
}

constexpr int kMtSeedLdsWords = kMtN * kMtSeedPitch;

// streams [blk * kMtSeedLanes, ...) by one wave; t: kMtSeedLdsWords of LDS
__device__ __forceinline__ void mt_seed_streams_block(const MtSeedSpec &sp, uint32_t *__restrict__ st,
                                                      uint32_t *t, uint32_t blk) {
    const int lane = threadIdx.x & 63;
    const uint32_t s0 = blk * (uint32_t)kMtSeedLanes;
    if (lane < kMtSeedLanes) {
        const uint32_t si = s0 + (uint32_t)lane;
        const int64_t a = mt_seed_of(sp, si < sp.n ? si : s0);
        const uint64_t m = a < 0 ? (uint64_t)(-(a + 1)) + 1u : (uint64_t)a;
        const uint32_t key0 = (uint32_t)m, key1 = (uint32_t)(m >> 32);
        const uint32_t add_even = key0, add_odd = key1 ? key1 + 1u : key0;
        // loop 1: k = 0..622 at i = k + 1 (step k adds key[k % klen] + k % klen), then the wrap
        // (mt[0] = mt[623]) and k = 623 at i = 1; init_genrand(19650218)'s words g alongside
        uint32_t g = 19650218u, prev = g;
#pragma unroll 2
        for (int i = 1; i < kMtN; i++) {
            g = 1812433253u * (g ^ (g >> 30)) + (uint32_t)i;
            prev = (g ^ ((prev ^ (prev >> 30)) * 1664525u)) + (((i - 1) & 1) ? add_odd : add_even);
            t[i * kMtSeedPitch + lane] = prev;
        }
        const uint32_t v1 = (t[kMtSeedPitch + lane] ^ ((prev ^ (prev >> 30)) * 1664525u)) + add_odd;
        // loop 2: i = 2..623, the wrap, i = 1.  The loop-1 words come from LDS one block of 8
        // ahead of the chain (a read waited on at its use would put LDS latency on every step).
        prev = v1;
        constexpr int kAhead = 8;
        static_assert((kMtN - 2) % kAhead == 6, "the last block is short");
        uint32_t cur[kAhead], nxt[kAhead];
#pragma unroll
        for (int k = 0; k < kAhead; k++) cur[k] = t[(2 + k) * kMtSeedPitch + lane];
        for (int i0 = 2; i0 < kMtN; i0 += kAhead) {
#pragma unroll
            for (int k = 0; k < kAhead; k++) {
                const int i = i0 + kAhead + k;
                nxt[k] = i < kMtN ? t[i * kMtSeedPitch + lane] : 0u;
            }
#pragma unroll
            for (int k = 0; k < kAhead; k++) {
                const int i = i0 + k;
                if (i < kMtN) {
                    prev = (cur[k] ^ ((prev ^ (prev >> 30)) * 1566083941u)) - (uint32_t)i;
                    t[i * kMtSeedPitch + lane] = prev;
                }
            }
#pragma unroll
            for (int k = 0; k < kAhead; k++) cur[k] = nxt[k];
        }
        t[kMtSeedPitch + lane] = (v1 ^ ((prev ^ (prev >> 30)) * 1566083941u)) - 1u;
        t[lane] = 0x80000000u;
    }
    wave_lds_order();
    // each stream's 624 words: coalesced rows
    for (int l = 0; l < kMtSeedLanes; l++) {
        if (s0 + (uint32_t)l >= sp.n) break;
        uint32_t *dst = st + (size_t)(s0 + (uint32_t)l) * kMtN;
        for (int i = lane; i < kMtN; i += 64) dst[i] = t[i * kMtSeedPitch + l];
    }
}

__host__ __device__ __forceinline__ uint32_t mt_seed_blocks(uint32_t n) { return (n + kMtSeedLanes - 1) / kMtSeedLanes; }

__global__ __launch_bounds__(64) void k_mt_seed_streams(MtSeedSpec sp, uint32_t *__restrict__ st) {
    __shared__ uint32_t t[kMtSeedLdsWords];
    mt_seed_streams_block(sp, st, t, blockIdx.x);
}

__host__ __forceinline__ void launch_mt_seed_streams(const MtSeedSpec &sp, uint32_t *st, hipStream_t s) {
    if (sp.n)
        hipLaunchKernelGGL(k_mt_seed_streams, dim3(mt_seed_blocks(sp.n)), dim3(64), 0, s, sp, st);
}

// a stream's state seeded by k_mt_seed_streams, into the wave's LDS
__device__ __forceinline__ void mt_load(uint32_t *mt, const uint32_t *__restrict__ st) {
    const int lane = threadIdx.x & 63;
    for (int i = lane; i < kMtN; i += 64) mt[i] = st[i];
    wave_lds_order();
}

// The first _randbelow(n) draw of a freshly seeded stream, ONE SEED PER LANE (V2's tail steps
// reseed before every draw, V2:107-112, and use only its first word or few).  Seeding is
// init_by_array over the 1-2 key words (klen), two serial chains of 624 + 623 steps; draw word
// w < 227 of the first twist needs only s[w], s[w + 1] and s[w + 397] of the seeded state, so
// each lane runs the chains itself (loop 1 twice: once for its wrap value, once beside loop 2)
// and keeps s[0 .. kFirstWords] and s[397 .. 397 + kFirstWords).  Returns false when all
// kFirstWords words were rejected (probability < 2^-16 per lane): the caller then runs the
// wave path (mt_seed + mt_draws) for that lane's seed.  The init_genrand(19650218) chain is
// the same for every lane (scalar code).
constexpr int kFirstWords = 16;

__device__ __forceinline__ bool mt_first_draw_lane(uint32_t key0, uint32_t key1, int klen, uint32_t n,
                                                   uint32_t &out) {
    const uint32_t add_even = key0, add_odd = klen == 2 ? key1 + 1u : key0;
    auto f1 = [](uint32_t p) { return (p ^ (p >> 30)) * 1664525u; };
    auto f2 = [](uint32_t p) { return (p ^ (p >> 30)) * 1566083941u; };
    // pass 1: loop 1's chain a[1 .. 623] (a[i] = (g[i] ^ f1(a[i-1])) + key term, a[0] = g[0]),
    // then its wrap iteration (k = 623, i = 1): a'[1]
    uint32_t g = 19650218u, a = g, a1 = 0u;
    for (int i = 1; i < kMtN; i++) {
        g = 1812433253u * (g ^ (g >> 30)) + (uint32_t)i;
        a = (g ^ f1(a)) + (((i - 1) & 1) ? add_odd : add_even);
        if (i == 1) a1 = a;
    }
    const uint32_t a1w = (a1 ^ f1(a)) + add_odd;
    // pass 2: loop 2 (b[i] = (a[i] ^ f2(b[i-1])) - i, i = 2 .. 623, b[1] = a'[1]) with loop 1's
    // a[i] regenerated beside it
    g = 1812433253u * (19650218u ^ (19650218u >> 30)) + 1u;   // g[1]
    a = a1;
    uint32_t b = a1w;
    uint32_t lo[kFirstWords + 1], hi[kFirstWords];   // s[0 .. K], s[397 .. 397 + K)
    auto step = [&](int i) {
        g = 1812433253u * (g ^ (g >> 30)) + (uint32_t)i;
        a = (g ^ f1(a)) + (((i - 1) & 1) ? add_odd : add_even);
        b = (a ^ f2(b)) - (uint32_t)i;
    };
#pragma unroll
    for (int i = 2; i <= kFirstWords; i++) { step(i); lo[i] = b; }
    for (int i = kFirstWords + 1; i < kMtM; i++) step(i);
#pragma unroll
    for (int i = kMtM; i < kMtM + kFirstWords; i++) { step(i); hi[i - kMtM] = b; }
    for (int i = kMtM + kFirstWords; i < kMtN; i++) step(i);
    lo[1] = (a1w ^ f2(b)) - 1u;     // loop 2's wrap (i = 1, mt[0] = b[623])
    lo[0] = 0x80000000u;
    const uint32_t kbits = 32u - (uint32_t)__builtin_clz(n);   // n.bit_length()
    bool found = false;
    uint32_t r = 0;
#pragma unroll
    for (int w = 0; w < kFirstWords; w++) {
        const uint32_t y = mt_temper(mt_twist_word(lo[w], lo[w + 1], hi[w])) >> (32u - kbits);
        if (!found && y < n) { r = y; found = true; }
    }
    out = r;
    return found;
}
}  // namespace

}  // namespace pss
