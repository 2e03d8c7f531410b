// pss_mt.h -- CPython 3.10 MT19937 on one wave (order mode PSS_ORDER_EXACT): seeding
// (`random_seed` -> init_by_array, _randommodule.c), the twist in LDS, tempering, and a
// speculative reader that turns the word stream into `_randbelow(n)` draws (random.py:239-249)
// 64 words at a time.  Shared by pss_v1exact.hip and pss_v2exact.hip.
#pragma once
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
__device__ void mt_seed(uint32_t *mt, uint32_t key0, uint32_t key1, int klen) {
    const int lane = threadIdx.x & 63;
    // loop 1: i = 1..623, then the wrap (mt[0] = mt[623]) and one more step at i = 1
    // init_genrand(19650218)'s words are generated alongside (an independent scalar chain,
    // cheaper than a scalar-cache load per step)
    uint32_t g = 19650218u;
    uint32_t prev = g;
    uint32_t first = 0;
    int j = 0;
    for (int i = 1; i < kMtN; i++) {
        g = 1812433253u * (g ^ (g >> 30)) + (uint32_t)i;
        const uint32_t v = (g ^ ((prev ^ (prev >> 30)) * 1664525u)) + (j ? key1 : key0) + (uint32_t)j;
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
template <class Bound, class Emit>
__device__ void mt_draws(uint32_t *mt, uint32_t nd, Bound bound, Emit emit) {
    const int lane = threadIdx.x & 63;
    uint32_t d0 = 0;
    while (d0 < nd) {
        mt_twist(mt);
        for (int q0 = 0; q0 < kMtN && d0 < nd; q0 += 64) {
            const int nval = kMtN - q0 < 64 ? kMtN - q0 : 64;
            const uint32_t word = lane < nval ? mt_temper(mt[q0 + lane]) : 0u;
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
            d0 += (uint32_t)__popcll(__ballot(acc));
        }
    }
}
}  // namespace

}  // namespace pss
