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
// k2 indices [i2, i2 + 32], else the lanes' k2 indices are guessed and re-derived to the fixed
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
        const uint32_t Fp = (uint32_t)__shfl((int)Fx, lane > 0 ? lane - 1 : 0);
        role = lane ? role_apply(Fp, st) : st;
        const uint64_t m2 = __ballot(valid && role == 1u && a2);
        j = i2 + (uint32_t)__popcll(m2 & below);
    };
    // a block holds at most 32 k2 draws, so each lane's k2 index lies in [i2, i2 + 32]: where
    // every lane's k2 verdict is the same over that whole range (all but ~1 % of lanes), one
    // scan settles the block; otherwise iterate guess -> true index
    const uint32_t nhi = i2 < W ? W - i2 : 1u, nlo = i2 + 32u < W ? W - (i2 + 32u) : 1u;
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
    st = role_apply((uint32_t)__shfl((int)Fx, 63), st);
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

// The same draws on a workgroup of kMtWgThreads (10 waves) per stream, for long windows (C5's
// pool2 windows are 2^20 steps and there are only ~11 per rank: one wave per stream left most of
// the chip idle).  Per twist:
//   twist   the 624 new words in three barrier-separated phases of <= 227 words (new[k] needs
//           new[k - 227] from k = 227 on), double-buffered, tempered into tw[]
//   blocks  the ten 64-word blocks, wave w takes block w: where every k2 verdict
//           of a block is fixed over all k2 indices the block can see in this twist ([i2, i2 +
//           32 (b + 1)] for block b), its transfer -- the composed role map and the k1 / k2
//           acceptances for either start role -- comes from one role scan without knowing
//           where the block starts
//   combine wave 0 chains the transfers from the twist's start state up to the first block
//           that was not settled, then runs that block and all after it exactly (pair_block)
//   emit    each wave emits its settled blocks from their now known start states
constexpr int kMtWgThreads = 640;   // ten waves: one 64-word block each
constexpr int kMtBlocks = (kMtN + 63) / 64;   // 10: nine of 64 words, one of 48
constexpr int kMtWgWaves = kMtWgThreads / 64;
constexpr int kMtPerWave = (kMtBlocks + kMtWgWaves - 1) / kMtWgWaves;

struct MtWgShared {
    uint32_t mt[2][kMtN];           // state, double-buffered across the twist
    uint32_t tw[2][kMtN];           // tempered words: the current twist's and the next one's
    uint32_t sum[kMtBlocks][6];     // settled?, role map, c1(st = 0), c1(st = 1), c2(0), c2(1)
    uint32_t start[kMtBlocks][3];   // (st, i1, i2) at each block's start
    uint32_t state[4];              // st, i1, i2, first unsettled block
};

// Software pipeline of the workgroup draws: the twist that makes the NEXT 624 words runs on
// waves 4.. beside the current twist's three phases (blocks | combine | emit), one of its three
// dependent steps per phase, so a twist costs three barriers instead of six phases.  Step p
// computes new[k], k in [227 p, 227 p + 227) (new[k] needs new[k - 227] from k = 227 on), by
// thread tt = tid - kMtTwistLo; the tempered word goes to tw.
constexpr int kMtTwistLo = 256;
__device__ __forceinline__ void mt_twist_step(const uint32_t *o, uint32_t *nw, uint32_t *tw, int p,
                                              int tid) {
    constexpr int D = kMtN - kMtM;   // 227
    const uint32_t tt = (uint32_t)(tid - kMtTwistLo);
    const int k = (int)tt + D * p;
    if (tt >= (uint32_t)D || k >= kMtN) return;
    uint32_t v;
    if (p == 0) v = mt_twist_word(o[k], o[k + 1], o[k + kMtM]);
    else if (k < kMtN - 1) v = mt_twist_word(o[k], o[k + 1], nw[k - D]);
    else v = mt_twist_word(o[kMtN - 1], nw[0], nw[kMtM - 1]);
    nw[k] = v;
    tw[k] = mt_temper(v);
}

// the first twist of a stream (the pipeline's prologue): old = mt[cur] -> mt[cur ^ 1], tw
__device__ __forceinline__ void mt_twist_wg(MtWgShared &sh, int cur, uint32_t *tw) {
#pragma unroll
    for (int p = 0; p < 3; p++) {
        mt_twist_step(sh.mt[cur], sh.mt[cur ^ 1], tw, p, threadIdx.x);
        __syncthreads();
    }
}

template <class Emit>
__device__ void mt_draws_pair_wg(MtWgShared &sh, int cur, uint32_t W, uint32_t P, Emit emit) {
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const uint32_t kb1 = 32u - (uint32_t)__builtin_clz(P);
    const uint64_t below = lanemask_lt();
    if (tid == 0) { sh.state[0] = 0u; sh.state[1] = 0u; sh.state[2] = 0u; }
    mt_twist_wg(sh, cur, sh.tw[0]);   // (its first barrier also publishes state)
    cur ^= 1;
    for (int tb = 0;; tb ^= 1) {
        if (sh.state[2] >= W) break;   // (uniform: read after a barrier)
        // tc: this twist's tempered words; the next twist (old = mt[cur] -> mt[cur ^ 1], into
        // tw[tb ^ 1]) runs one step per phase beside it
        const uint32_t *tc = sh.tw[tb];
        const uint32_t *o = sh.mt[cur];
        uint32_t *nw = sh.mt[cur ^ 1], *tn = sh.tw[tb ^ 1];
        mt_twist_step(o, nw, tn, 0, tid);
        // ---- blocks: transfers of the settled ones
        const uint32_t i2_0 = sh.state[2];
        uint32_t Fkeep[kMtPerWave];
        bool a1k[kMtPerWave], a2k[kMtPerWave];
#pragma unroll
        for (int s = 0; s < kMtPerWave; s++) {
            Fkeep[s] = 0u; a1k[s] = false; a2k[s] = false;
            const int b = wv + kMtWgWaves * s;
            if (b >= kMtBlocks) break;
            const int q0 = 64 * b, nval = kMtN - q0 < 64 ? kMtN - q0 : 64;
            const bool valid = lane < nval;
            const uint32_t word = valid ? tc[q0 + lane] : 0u;
            const bool a1 = valid && (word >> (32u - kb1)) < P;
            const uint32_t jhi = i2_0 + 32u * (uint32_t)(b + 1);
            const uint32_t nhi = i2_0 < W ? W - i2_0 : 1u, nlo = jhi < W ? W - jhi : 1u;
            const uint32_t kbh = 32u - (uint32_t)__builtin_clz(nhi);
            const uint32_t rh = word >> (32u - kbh);
            const bool sure = kbh == 32u - (uint32_t)__builtin_clz(nlo) && (rh < nlo || rh >= nhi);
            const bool settled = __ballot(valid && !sure) == 0;
            if (settled) {
                const bool a2 = valid && rh < nlo;
                const uint32_t Fx = wave_role_scan(((a1 != a2) ? 2u : 0u) | (a1 ? 1u : 0u));
                const uint32_t Fp = (uint32_t)__shfl((int)Fx, lane > 0 ? lane - 1 : 0);
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
                    sh.sum[b][0] = 1u;
                    sh.sum[b][1] = F63;
                    sh.sum[b][2] = c[0]; sh.sum[b][3] = c[1]; sh.sum[b][4] = c[2]; sh.sum[b][5] = c[3];
                }
                Fkeep[s] = Fp;
                a1k[s] = a1;
                a2k[s] = a2;
            } else if (lane == 0) {
                sh.sum[b][0] = 0u;
            }
        }
        __syncthreads();
        mt_twist_step(o, nw, tn, 1, tid);
        // ---- combine (wave 0): chain the settled transfers, then the rest exactly.  Lane b holds
        // block b's summary; the chain reads it with readlane (no LDS round trip per block)
        if (wv == 0) {
            uint32_t st = sh.state[0], i1 = sh.state[1], i2 = sh.state[2];
            uint32_t vs = 0u, vF = 0u, v10 = 0u, v11 = 0u, v20 = 0u, v21 = 0u;
            if (lane < kMtBlocks) {
                vs = sh.sum[lane][0];
                if (vs) { vF = sh.sum[lane][1]; v10 = sh.sum[lane][2]; v11 = sh.sum[lane][3]; v20 = sh.sum[lane][4]; v21 = sh.sum[lane][5]; }
            }
            int b = 0;
            for (; b < kMtBlocks; b++) {
                if (lane == 0) { sh.start[b][0] = st; sh.start[b][1] = i1; sh.start[b][2] = i2; }
                if (!__builtin_amdgcn_readlane((int)vs, b)) break;
                i1 += (uint32_t)__builtin_amdgcn_readlane((int)(st ? v11 : v10), b);
                i2 += (uint32_t)__builtin_amdgcn_readlane((int)(st ? v21 : v20), b);
                st = role_apply((uint32_t)__builtin_amdgcn_readlane((int)vF, b), st);
            }
            const int fu = b;
            for (; b < kMtBlocks && i2 < W; b++) {
                const int q0 = 64 * b, nval = kMtN - q0 < 64 ? kMtN - q0 : 64;
                const bool valid = lane < nval;
                pair_block(valid ? tc[q0 + lane] : 0u, valid, W, P, kb1, st, i1, i2, emit);
            }
            if (lane == 0) { sh.state[0] = st; sh.state[1] = i1; sh.state[2] = i2; sh.state[3] = (uint32_t)fu; }
        }
        __syncthreads();
        mt_twist_step(o, nw, tn, 2, tid);
        cur ^= 1;
        // ---- emit the settled blocks before the first unsettled one
        const int fu = (int)sh.state[3];
#pragma unroll
        for (int s = 0; s < kMtPerWave; s++) {
            const int b = wv + kMtWgWaves * s;
            if (b >= fu) break;
            const int q0 = 64 * b, nval = kMtN - q0 < 64 ? kMtN - q0 : 64;
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
                    const uint32_t nhi = i2_0 < W ? W - i2_0 : 1u;
                    if (j < W) emit(true, j, word >> (32u - (32u - (uint32_t)__builtin_clz(nhi))));
                }
            }
        }
        __syncthreads();
    }
}

// mt_draws on a workgroup per stream (V1 windows beyond LDS: ~12 windows per rank at C5), for a
// non-increasing bound(d): the twist and the block transfers as in mt_draws_pair_wg -- a block
// whose every verdict is fixed over the bounds of all draw indices it can see in this twist
// ([d, d + 64 (b + 1)] for block b) makes exactly popc(accepted) draws wherever it starts.
template <class Bound, class Emit>
__device__ void mt_draws_wg(MtWgShared &sh, int cur, uint32_t nd, Bound bound, Emit emit) {
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const uint64_t below = lanemask_lt();
    if (tid == 0) sh.state[0] = 0u;
    mt_twist_wg(sh, cur, sh.tw[0]);   // pipelined as in mt_draws_pair_wg
    cur ^= 1;
    for (int tb = 0;; tb ^= 1) {
        if (sh.state[0] >= nd) break;
        const uint32_t *tc = sh.tw[tb];
        const uint32_t *o = sh.mt[cur];
        uint32_t *nw = sh.mt[cur ^ 1], *tn = sh.tw[tb ^ 1];
        mt_twist_step(o, nw, tn, 0, tid);
        const uint32_t d0 = sh.state[0];
        bool acck[kMtPerWave];
        uint32_t rk[kMtPerWave];
#pragma unroll
        for (int s = 0; s < kMtPerWave; s++) {
            acck[s] = false; rk[s] = 0u;
            const int b = wv + kMtWgWaves * s;
            if (b >= kMtBlocks) break;
            const int q0 = 64 * b, nval = kMtN - q0 < 64 ? kMtN - q0 : 64;
            const bool valid = lane < nval;
            const uint32_t word = valid ? tc[q0 + lane] : 0u;
            const uint32_t dlo = d0 < nd ? d0 : nd - 1u;
            const uint32_t dhi = d0 + 64u * (uint32_t)(b + 1) < nd ? d0 + 64u * (uint32_t)(b + 1) : nd - 1u;
            const uint32_t nhi = bound(dlo), nlo = bound(dhi);
            const uint32_t kbh = 32u - (uint32_t)__builtin_clz(nhi);
            const uint32_t r = word >> (32u - kbh);
            const bool sure = kbh == 32u - (uint32_t)__builtin_clz(nlo) && (r < nlo || r >= nhi);
            if (__ballot(valid && !sure) == 0) {
                const bool acc = valid && r < nlo;
                const uint32_t cnt = (uint32_t)__popcll(__ballot(acc));
                if (lane == 0) { sh.sum[b][0] = 1u; sh.sum[b][1] = cnt; }
                acck[s] = acc;
                rk[s] = r;
            } else if (lane == 0) {
                sh.sum[b][0] = 0u;
            }
        }
        __syncthreads();
        mt_twist_step(o, nw, tn, 1, tid);
        if (wv == 0) {
            uint32_t d = sh.state[0];
            uint32_t vs = 0u, vc = 0u;
            if (lane < kMtBlocks) { vs = sh.sum[lane][0]; vc = vs ? sh.sum[lane][1] : 0u; }
            int b = 0;
            for (; b < kMtBlocks; b++) {
                if (lane == 0) sh.start[b][0] = d;
                if (!__builtin_amdgcn_readlane((int)vs, b)) break;
                d += (uint32_t)__builtin_amdgcn_readlane((int)vc, b);
            }
            const int fu = b;
            for (; b < kMtBlocks && d < nd; b++) {
                const int q0 = 64 * b, nval = kMtN - q0 < 64 ? kMtN - q0 : 64;
                d += draw_block(lane < nval ? tc[q0 + lane] : 0u, nval, d, nd, bound, emit);
            }
            if (lane == 0) { sh.state[0] = d; sh.state[3] = (uint32_t)fu; }
        }
        __syncthreads();
        mt_twist_step(o, nw, tn, 2, tid);
        cur ^= 1;
        const int fu = (int)sh.state[3];
#pragma unroll
        for (int s = 0; s < kMtPerWave; s++) {
            const int b = wv + kMtWgWaves * s;
            if (b >= fu) break;
            const uint32_t d = sh.start[b][0] + (uint32_t)__popcll(__ballot(acck[s]) & below);
            if (acck[s] && d < nd) emit(d, rk[s]);
        }
        __syncthreads();
    }
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
