// pss_common.h -- counter-based schedule primitives shared by the gfx950 kernels and the
// product's CPU mode (pss_cpu.cpp): the Philox schedule of DESIGN.md §3.  Both compile these
// same definitions, so the CPU mode matches the GPU bit for bit by construction.
// oracle/pss_oracle.c restates the schedule independently in C as the test checker.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define PSS_HD __host__ __device__ __forceinline__
#else
#define PSS_HD static inline
#endif

namespace pss {

enum : uint32_t { DOM_V1_WIN = 1, DOM_V2_SLOT = 2, DOM_V2_INS = 3, DOM_V2_TAIL = 4, DOM_V2_INIT = 5 };

// Philox4x32-10 (Salmon et al., SC'11).  Each 64-bit product is one v_mad_u64_u32 on gfx950.
PSS_HD void philox4x32_10(uint32_t &c0, uint32_t &c1, uint32_t &c2, uint32_t &c3,
                          uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; r++) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
        const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        c0 = n0; c1 = (uint32_t)p1; c2 = n2; c3 = (uint32_t)p0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
}

// The same function as a rolled loop: small code for kernel prologues, where an unrolled
// Philox is long straight-line code that runs once and mostly costs instruction-cache misses.
PSS_HD void philox4x32_10_rolled(uint32_t &c0, uint32_t &c1, uint32_t &c2, uint32_t &c3,
                                 uint32_t k0, uint32_t k1) {
#pragma unroll 1
    for (int r = 0; r < 10; r++) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
        const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        c0 = n0; c1 = (uint32_t)p1; c2 = n2; c3 = (uint32_t)p0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
}

PSS_HD uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

PSS_HD uint64_t epoch_key(uint64_t seed, int64_t epoch) {
    return mix64(mix64(seed) ^ (uint64_t)epoch);
}

PSS_HD int ceil_log2_u64(uint64_t n) {  // smallest b with 2^b >= n (n >= 1)
    return n <= 1 ? 0 : 64 - __builtin_clzll(n - 1);
}

// Keyed bijection of [0, n): 6-round balanced Feistel over 2h bits + cycle walking.
// Round function: multiplicative hashing of the keyed right half (one multiply per round);
// halves of <= 5 bits take 8 rounds of a stronger mixer (feistel_fsmall, below).
constexpr int kFeistelRounds = 6;

// Round function for halves of h <= 10 bits (domains up to 2^20, C5's pool): the top h bits of
// the low 16 bits of (R ^ k) * 0x9E37 -- a 16-bit multiplicative hash, so two chains fit one
// 32-bit register and run on packed 16-bit ops (feistel2_pk16; round 3 widened this from
// h <= 8, halving the grouped replay's Feistel work at C5).  Wider halves (h in 11..16): bits
// [24 - h, 24) of ((R ^ k) mod 2^24) * 0x9E3779 -- a 24 x 24-bit product (one full-rate
// v_mul_u32_u24 on gfx950; a 32-bit v_mul_lo_u32 issues at quarter rate) and one v_bfe_u32.
// Both take the bits just below the product's width, where one input step moves the output by
// the golden-ratio fraction of the output range -- the top bits of a 32-bit product would move
// by only ~2.5 at h = 10, and neighbouring positions then map to neighbouring values
// (tests/test_schedule_quality.py measures the neighbour law at every width).
constexpr uint32_t kFeistelM16 = 0x9E37u, kFeistelM24 = 0x9E3779u;
constexpr uint32_t kFeistelH16 = 10;   // widest half on the 16-bit round function

PSS_HD uint32_t feistel_f24(uint32_t r, uint32_t k, uint32_t h) {
    return ((((r ^ k) & 0xFFFFFFu) * kFeistelM24) >> (24u - h)) & ((1u << h) - 1u);
}

// Halves of <= kFeistelSmallH bits (domains up to 1024 elements: V1 windows and V2 pools of
// B <= 1024, off the bandwidth-bound paths): the one-multiply round functions above are nearly
// linear in a 2..5-bit R and leave neighbouring images dependent (tests/test_schedule_quality.py
// measured z = 20-120 on the law of (pi(0), pi(1)) at n = 16..256).  These domains take 8 rounds
// of a full 32-bit mixer instead -- the top h bits of murmur3's fmix32(R ^ k_i), round key
// k_i = k[i mod 6] + i * 0x9E3779B9 (the same six key words) -- which leaves no measurable
// dependence (|z| < 3 down to n = 2).
constexpr uint32_t kFeistelSmallH = 5;
constexpr int kFeistelSmallRounds = 8;

PSS_HD uint32_t feistel_fsmall(uint32_t r, uint32_t k, uint32_t h) {
    uint32_t x = r ^ k;
    x ^= x >> 16;
    x *= 0x85EBCA6Bu;
    x ^= x >> 13;
    x *= 0xC2B2AE35u;
    x ^= x >> 16;
    return h ? x >> (32u - h) : 0u;   // h = 0: a one-element domain (feistel_once with n = 1)
}

PSS_HD uint32_t feistel_pass(uint32_t x, uint32_t h, const uint32_t *k) {
    const uint32_t mask = (1u << h) - 1u;
    uint32_t L = x >> h, R = x & mask;
    if (h <= kFeistelSmallH) {
        for (int i = 0; i < kFeistelSmallRounds; i++) {
            const uint32_t t = L ^ feistel_fsmall(R, k[i % kFeistelRounds] + (uint32_t)i * 0x9E3779B9u, h);
            L = R;
            R = t;
        }
    } else if (h <= kFeistelH16) {
        const uint32_t sh = 16u - h;
#pragma unroll
        for (int i = 0; i < kFeistelRounds; i++) {
            const uint32_t t = L ^ ((((R ^ k[i]) * kFeistelM16) & 0xFFFFu) >> sh);
            L = R;
            R = t;
        }
    } else {
#pragma unroll
        for (int i = 0; i < kFeistelRounds; i++) {
            const uint32_t t = L ^ feistel_f24(R, k[i], h);
            L = R;
            R = t;
        }
    }
    return (L << h) | R;
}

// the 16-bit packed forms (feistel2_pk16 / feistel4_pk16: two chains per register, the halves
// joined in 32 bits) serve every half on the 16-bit round function, (kFeistelSmallH, 10]
PSS_HD bool feistel_packed_ok(uint32_t h) { return h > kFeistelSmallH && h <= kFeistelH16; }

PSS_HD uint32_t feistel(uint32_t x, uint32_t n, uint32_t h, const uint32_t *k) {
    if (n <= 1) return 0;
    // x < n <= 2^(2h): the walk stays on x's cycle and meets a value < n after a few steps
    // (each step lands below n with probability >= 1/4).  The bound only guards against a
    // caller passing x >= 2^(2h), which would otherwise never terminate.
    int guard = 1 << 16;
    do {
        if (--guard < 0) break;
        x = feistel_pass(x, h, k);
    } while (x >= n);
    return x;
}

// One Feistel pass, for domains n == 2^(2h) where cycle walking never triggers.
PSS_HD uint32_t feistel_once(uint32_t x, uint32_t h, const uint32_t *k) {
    return feistel_pass(x, h, k);
}

PSS_HD uint32_t feistel_half_bits(uint32_t n) {
    const int bits = ceil_log2_u64(n);
    return (uint32_t)((bits + 1) >> 1);
}

// V2 slot draw of step t (t < 2^32: ns >= 2^32 is rejected).  A keyed 32-bit mixer: two
// multiply-xorshift rounds (16 / x 0xA2F0AD / 15 / x 0x5A2D97 / 15), keyed by (s0, s1) = the
// first two words of the Philox block (0, 0, rank, DOM_V2_SLOT) under the epoch key.  Each
// multiply takes the low 24 bits of its operand (after the xorshift above it has folded the top
// bits down) by a 24-bit odd constant: one full-rate v_mul_u32_u24 on gfx950, where a 32-bit
// multiply is quarter rate -- the replay and the last-occurrence pass evaluate this for every
// step.  tests/test_schedule_quality.py checks the slot law and that the V2 displacement law
// still matches the reference's.
PSS_HD uint32_t slot_hash(uint32_t t, uint32_t s0, uint32_t s1) {
    uint32_t x = t ^ s0;
    x ^= x >> 16;
    x = (x & 0xFFFFFFu) * 0xA2F0ADu;
    x ^= x >> 15;
    x ^= s1;
    x = (x & 0xFFFFFFu) * 0x5A2D97u;
    x ^= x >> 15;
    return x;
}

// Lemire multiply-shift: uniform-ish slot in [0, n) from one 32-bit word (bias <= n/2^32).
PSS_HD uint32_t scale32(uint32_t u, uint32_t n) {
    return (uint32_t)(((uint64_t)u * n) >> 32);
}

// Slot drawn at V2 step t.  P1 = 2^b with b <= 16 ("paired"): one hash serves two steps -- t
// and t + 64 of each 128-step block, the top b bits of its high and of its low half-word (both
// exactly uniform).  Otherwise every step hashes its own index and scales it to [0, P1).
PSS_HD bool slot_paired(uint32_t P1) { return P1 <= 65536u && (P1 & (P1 - 1u)) == 0u; }

PSS_HD uint32_t slot_pair_index(uint32_t t) { return ((t >> 7) << 6) | (t & 63u); }

PSS_HD uint32_t slot_draw(uint32_t t, uint32_t s0, uint32_t s1, uint32_t P1) {
    if (slot_paired(P1)) {
        if (P1 == 1u) return 0u;
        const uint32_t sh = 32u - (uint32_t)ceil_log2_u64(P1);
        uint32_t u = slot_hash(slot_pair_index(t), s0, s1);
        if (t & 64u) u <<= 16;
        return u >> sh;
    }
    return scale32(slot_hash(t, s0, s1), P1);
}

// ------------------------------------------------------------------------------------------
// V2 pools beyond LDS (P1 > kLdsSlotMax): grouped slot draws.  The P1 slots
// are split into G = ceil(P1 / 4096) groups of q or q + 1 consecutive slots (the first r = P1
// mod G groups have q + 1); steps come in bursts of 32, burst b = t / 32 belongs to group
// b mod G and draws uniformly inside it.  Every group is then an independent slot machine of
// <= 4096 slots fed by every G-th burst: one LDS-resident wave per (rank, group) replays it.
// An element still leaves pool1 with probability ~1/P1 per step (1/S_g per step of its group,
// one step in G), so the residence law of the reference's single pool is kept.
// ------------------------------------------------------------------------------------------
constexpr uint32_t kLdsSlotMax = 16384;   // largest V2 pool replayed as one LDS slot table
#ifndef PSS_GROUP_SLOTS
#define PSS_GROUP_SLOTS 4096
#endif
constexpr uint32_t kGroupSlots = PSS_GROUP_SLOTS;    // slots per group (at most)
#ifndef PSS_BURST
#define PSS_BURST 32
#endif
constexpr uint32_t kBurst = PSS_BURST;    // consecutive steps of one group (16 up to schedule 3;
                                          // other values: timing builds only)

struct Groups {
    uint32_t G, q, r;   // groups; q = P1 / G, r = P1 mod G (groups g < r have q + 1 slots)
};

PSS_HD Groups v2_groups(uint32_t P1) {
    Groups gr;
    gr.G = (P1 + kGroupSlots - 1) / kGroupSlots;
    gr.q = P1 / gr.G;
    gr.r = P1 % gr.G;
    return gr;
}
PSS_HD uint32_t group_base(const Groups &gr, uint32_t g) { return g * gr.q + (g < gr.r ? g : gr.r); }
PSS_HD uint32_t group_size(const Groups &gr, uint32_t g) { return gr.q + (g < gr.r ? 1u : 0u); }
PSS_HD uint32_t group_of_step(const Groups &gr, uint32_t t) { return (t / kBurst) % gr.G; }

// global step of sub-step u of group g's stream (its bursts are b = m * G + g, m = u / kBurst)
PSS_HD uint64_t group_step(const Groups &gr, uint32_t g, uint64_t u) {
    return ((u / kBurst) * gr.G + g) * kBurst + (u % kBurst);
}

// sub-step of step t inside its group's stream
PSS_HD uint64_t group_substep(const Groups &gr, uint64_t t) {
    return (t / kBurst / gr.G) * kBurst + t % kBurst;
}

// Slot, inside group g of size S, drawn by sub-step u (global step t).  Groups of 2^b slots
// pair sub-steps u and u + 64 (u mod 128 < 64): one hash of the lower one's step serves both,
// the lower takes the top b bits of its high half-word, the upper those of the low half-word
// (both exactly uniform).  Other sizes hash every step and scale it to [0, S).
PSS_HD uint32_t group_slot(const Groups &gr, uint32_t g, uint32_t S, uint64_t u, uint32_t t,
                           uint32_t s0, uint32_t s1) {
    if ((S & (S - 1u)) == 0u) {
        if (S == 1u) return 0u;
        const uint32_t sh = 32u - (uint32_t)ceil_log2_u64(S);
        if (u & 64u) return (slot_hash((uint32_t)group_step(gr, g, u - 64u), s0, s1) << 16) >> sh;
        return slot_hash(t, s0, s1) >> sh;
    }
    return scale32(slot_hash(t, s0, s1), S);
}

// slot (global index) drawn at step t of a grouped pool
PSS_HD uint32_t slot_draw_grouped(uint32_t t, uint32_t s0, uint32_t s1, const Groups &gr) {
    const uint32_t g = group_of_step(gr, t);
    const uint32_t S = group_size(gr, g);
    return group_base(gr, g) + group_slot(gr, g, S, group_substep(gr, t), t, s0, s1);
}

// Tail of a grouped pool: the final pool is drained in rounds; in each round every group emits
// its next (up to) kBurst elements, groups in order.  Group g emits its S_g elements in the order
// of its own Feistel bijection of [0, S_g) (keys round_keys8(g, rank, DOM_V2_TAIL)).  Position
// (after T) of group g's e-th element: full rounds while every group still has kBurst left,
// then one last round of the q mod kBurst (+1 for g < r) leftovers.
PSS_HD uint32_t group_tail_pos(const Groups &gr, uint32_t g, uint32_t e) {
    const uint32_t full = gr.q / kBurst;
    if (e < full * kBurst) return (e / kBurst) * kBurst * gr.G + g * kBurst + e % kBurst;
    const uint32_t c = gr.q % kBurst;
    return full * kBurst * gr.G + g * c + (g < gr.r ? g : gr.r) + (e - full * kBurst);
}

// number of the steps t < T that group g draws (its sub-stream length)
PSS_HD uint64_t group_steps(const Groups &gr, uint32_t g, uint64_t T) {
    const uint64_t full = T / kBurst, rem = T % kBurst;
    uint64_t n = (full / gr.G + (g < full % gr.G ? 1u : 0u)) * kBurst;
    if (rem && full % gr.G == g) n += rem;
    return n;
}

// ------------------------------------------------------------------------------------------
// Philox-derived keys (the counters of DESIGN.md §3's domain table), one definition for the
// kernels and the CPU mode
// ------------------------------------------------------------------------------------------
// 8 words = Philox blocks (c0, 0, c2, dom) and (c0, 1, c2, dom); Feistel uses the first 6
PSS_HD void round_keys8(uint32_t key0, uint32_t key1, uint32_t c0, uint32_t c2, uint32_t dom,
                        uint32_t k[8]) {
    for (uint32_t h = 0; h < 2; h++) {
        uint32_t a = c0, b = h, c = c2, d = dom;
        philox4x32_10_rolled(a, b, c, d, key0, key1);
        k[4 * h] = a; k[4 * h + 1] = b; k[4 * h + 2] = c; k[4 * h + 3] = d;
    }
}

}  // namespace pss
