// pss_device.h -- wave64 / workgroup primitives shared by the gfx950 kernels.
#pragma once
#include "pss_common.h"
#include "pss_kernels.h"
#include "pss_map.h"

namespace pss {

template <int CTRL, int ROWMASK>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t x) {
    // old = 0: lanes whose source is outside the row (or whose row is masked) read 0
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, ROWMASK, 0xF, false);
}

template <int CTRL, int ROWMASK>
__device__ __forceinline__ uint64_t dpp_u64(uint64_t x) {
    const uint32_t lo = dpp_u32<CTRL, ROWMASK>((uint32_t)x);
    const uint32_t hi = dpp_u32<CTRL, ROWMASK>((uint32_t)(x >> 32));
    return ((uint64_t)hi << 32) | lo;
}

// Inclusive wave64 scan: row_shr 1/2/4/8 inside each 16-lane row, then row_bcast15 and
// row_bcast31 carry the row totals across rows (gfx9 DPP; no LDS traffic).
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
    x += dpp_u32<0x111, 0xF>(x);
    x += dpp_u32<0x112, 0xF>(x);
    x += dpp_u32<0x114, 0xF>(x);
    x += dpp_u32<0x118, 0xF>(x);
    x += dpp_u32<0x142, 0xA>(x);
    x += dpp_u32<0x143, 0xC>(x);
    return x;
}

__device__ __forceinline__ uint64_t wave_incl_scan(uint64_t x) {
    x += dpp_u64<0x111, 0xF>(x);
    x += dpp_u64<0x112, 0xF>(x);
    x += dpp_u64<0x114, 0xF>(x);
    x += dpp_u64<0x118, 0xF>(x);
    x += dpp_u64<0x142, 0xA>(x);
    x += dpp_u64<0x143, 0xC>(x);
    return x;
}

__device__ __forceinline__ uint64_t wave_sum(uint64_t x) {
    x = wave_incl_scan(x);
    return __shfl(x, 63);
}

// Exclusive scan over a workgroup of NT threads; `tot` is NT/64 words of LDS.
template <int NT, typename T>
__device__ __forceinline__ T block_excl_scan(T x, T *tot, T &total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const T inc = wave_incl_scan(x);
    if (lane == 63) tot[wid] = inc;
    __syncthreads();
    T pre = 0, all = 0;
#pragma unroll
    for (int i = 0; i < NT / 64; i++) {
        const T v = tot[i];
        if (i < wid) pre += v;
        all += v;
    }
    __syncthreads();
    total = all;
    return pre + inc - x;
}

__device__ __forceinline__ int64_t wrap_id(int64_t id, int64_t N) { return id >= N ? id - N : id; }

// ------------------------------------------------------------------------------------------
// V2 helpers
// ------------------------------------------------------------------------------------------
// slot draw of step t = sb*256 + j*64 + lane (super-batch sb, sub-batch j): slot_hash under
// the rank's key (SlotKey, computed once per wave)
struct SlotKey { uint32_t s0, s1; };

__device__ __forceinline__ SlotKey slot_key(const Geometry &g, uint32_t rank) {
    uint32_t c0 = 0, c1 = 0, c2 = rank, c3 = DOM_V2_SLOT;
    philox4x32_10_rolled(c0, c1, c2, c3, g.key0, g.key1);
    return SlotKey{c0, c1};
}

// slots of the 4 steps sb*256 + 64 j + lane (j < 4) of super-batch sb
__device__ __forceinline__ void slot_ks(const SlotKey &sk, int64_t sb, int lane, uint32_t P1,
                                        uint32_t k[4]) {
    const uint32_t t0 = (uint32_t)sb * 256u + (uint32_t)lane;
#pragma unroll
    for (int j = 0; j < 4; j++) k[j] = slot_draw(t0 + 64u * j, sk.s0, sk.s1, P1);
}

// slot of a 32-bit draw: Lemire multiply-shift, or a plain shift when P1 is a power of two
// (exactly the same value: (u * 2^k) >> 32 == u >> (32 - k)), one quarter-rate multiply less
template <bool POW2>
__device__ __forceinline__ uint32_t slot_scale(uint32_t u, uint32_t P1, uint32_t sh) {
    return POW2 ? (u >> sh) : scale32(u, P1);
}

// slots of steps t, t + 64, t + 128, t + 192 (t = a lane's step of a 256-aligned super-batch):
// POW2 (P1 = 2^b <= 65536, paired draw) -- two hashes for the four steps
template <bool POW2>
__device__ __forceinline__ void slot4(uint32_t t, const SlotKey &sk, uint32_t P1, uint32_t sh,
                                      uint32_t k[4]) {
    if (POW2) {
#pragma unroll
        for (int j = 0; j < 4; j += 2) {
            const uint32_t u = slot_hash(slot_pair_index(t + 64u * j), sk.s0, sk.s1);
            k[j] = u >> sh;
            k[j + 1] = (u << 16) >> sh;
        }
    } else {
#pragma unroll
        for (int j = 0; j < 4; j++) k[j] = scale32(slot_hash(t + 64u * j, sk.s0, sk.s1), P1);
    }
}

// Two one-pass Feistel chains (feistel_pass with h <= kFeistelH16) in one register, on packed 16-bit ops:
// chain 0 in the low half-word, chain 1 in the high one; kp[i] = (k[i] & 0xFFFF) * 0x10001
// (both chains under the same round keys).  Same values as feistel_once on each chain.
typedef unsigned short pss_u16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void feistel2_pk16(uint32_t x0, uint32_t x1, uint32_t h, const uint32_t *kp,
                                              uint32_t &y0, uint32_t &y1) {
    const uint32_t mask = (1u << h) - 1u;
    uint32_t L = (x0 >> h) | ((x1 >> h) << 16);
    uint32_t R = (x0 & mask) | ((x1 & mask) << 16);
    const pss_u16x2 M = {(unsigned short)kFeistelM16, (unsigned short)kFeistelM16};
    const pss_u16x2 SH = {(unsigned short)(16u - h), (unsigned short)(16u - h)};
#pragma unroll
    for (int i = 0; i < kFeistelRounds; i++) {
        const pss_u16x2 a = __builtin_bit_cast(pss_u16x2, R ^ kp[i]);
        const pss_u16x2 f = (a * M) >> SH;
        const uint32_t t = L ^ __builtin_bit_cast(uint32_t, f);
        L = R;
        R = t;
    }
    y0 = ((L & 0xFFFFu) << h) | (R & 0xFFFFu);
    y1 = ((L >> 16) << h) | (R >> 16);
}

// feistel2_pk16 with each chain's own round keys (k0: the low half-word's chain, k1: the high's)
__device__ __forceinline__ void feistel2_pk16_k2(uint32_t x0, uint32_t x1, uint32_t h, const uint32_t *k0,
                                                 const uint32_t *k1, uint32_t &y0, uint32_t &y1) {
    const uint32_t mask = (1u << h) - 1u;
    uint32_t L = (x0 >> h) | ((x1 >> h) << 16);
    uint32_t R = (x0 & mask) | ((x1 & mask) << 16);
    const pss_u16x2 M = {(unsigned short)kFeistelM16, (unsigned short)kFeistelM16};
    const pss_u16x2 SH = {(unsigned short)(16u - h), (unsigned short)(16u - h)};
#pragma unroll
    for (int i = 0; i < kFeistelRounds; i++) {
        const uint32_t kp = (k0[i] & 0xFFFFu) | (k1[i] << 16);
        const pss_u16x2 a = __builtin_bit_cast(pss_u16x2, R ^ kp);
        const pss_u16x2 f = (a * M) >> SH;
        const uint32_t t = L ^ __builtin_bit_cast(uint32_t, f);
        L = R;
        R = t;
    }
    y0 = ((L & 0xFFFFu) << h) | (R & 0xFFFFu);
    y1 = ((L >> 16) << h) | (R >> 16);
}

// Four chains in two registers, rounds interleaved so that neither packed multiply waits on
// the other's result (no dependency stalls between the pk ops).  Same values as feistel2_pk16.
__device__ __forceinline__ void feistel4_pk16(const uint32_t x[4], uint32_t h, const uint32_t *kp,
                                              uint32_t y[4]) {
    const uint32_t mask = (1u << h) - 1u;
    uint32_t L0 = (x[0] >> h) | ((x[1] >> h) << 16), R0 = (x[0] & mask) | ((x[1] & mask) << 16);
    uint32_t L1 = (x[2] >> h) | ((x[3] >> h) << 16), R1 = (x[2] & mask) | ((x[3] & mask) << 16);
    const pss_u16x2 M = {(unsigned short)kFeistelM16, (unsigned short)kFeistelM16};
    const pss_u16x2 SH = {(unsigned short)(16u - h), (unsigned short)(16u - h)};
#pragma unroll
    for (int i = 0; i < kFeistelRounds; i++) {
        const pss_u16x2 a0 = __builtin_bit_cast(pss_u16x2, R0 ^ kp[i]);
        const pss_u16x2 a1 = __builtin_bit_cast(pss_u16x2, R1 ^ kp[i]);
        const pss_u16x2 f0 = (a0 * M) >> SH;
        const pss_u16x2 f1 = (a1 * M) >> SH;
        const uint32_t t0 = L0 ^ __builtin_bit_cast(uint32_t, f0);
        const uint32_t t1 = L1 ^ __builtin_bit_cast(uint32_t, f1);
        L0 = R0; R0 = t0;
        L1 = R1; R1 = t1;
    }
    y[0] = ((L0 & 0xFFFFu) << h) | (R0 & 0xFFFFu);
    y[1] = ((L0 >> 16) << h) | (R0 >> 16);
    y[2] = ((L1 & 0xFFFFu) << h) | (R1 & 0xFFFFu);
    y[3] = ((L1 >> 16) << h) | (R1 >> 16);
}

// Feistel round keys of pool2 window w: Philox blocks (w, 0, rank, INS) and (w, 1, rank, INS),
// 8 words of which the first kFeistelRounds are used
constexpr int kRoundKeyWords = 8;

__device__ __forceinline__ void window_round_keys(const Geometry &g, uint32_t rank, int64_t w,
                                                  uint32_t k[kRoundKeyWords]) {
#pragma unroll 1
    for (int h = 0; h < 2; h++) {
        uint32_t c0 = (uint32_t)w, c1 = (uint32_t)h, c2 = rank, c3 = DOM_V2_INS;
        philox4x32_10_rolled(c0, c1, c2, c3, g.key0, g.key1);
        k[4 * h] = c0; k[4 * h + 1] = c1; k[4 * h + 2] = c2; k[4 * h + 3] = c3;
    }
}

// Feistel keys of the final-pool drain (V2 tail): Philox blocks (0, 0|1, rank, DOM_V2_TAIL)
__device__ __forceinline__ void tail_round_keys(const Geometry &g, uint32_t rank,
                                                uint32_t k[kRoundKeyWords]) {
#pragma unroll 1
    for (int h = 0; h < 2; h++) {
        uint32_t c0 = 0, c1 = (uint32_t)h, c2 = rank, c3 = DOM_V2_TAIL;
        philox4x32_10_rolled(c0, c1, c2, c3, g.key0, g.key1);
        k[4 * h] = c0; k[4 * h + 1] = c1; k[4 * h + 2] = c2; k[4 * h + 3] = c3;
    }
}

// round keys of windows [w_lo, w_lo + nwin) into LDS (all threads of the block take part)
__device__ __forceinline__ void stage_keys(const Geometry &g, uint32_t rank, int64_t w_lo, int nwin,
                                           uint32_t *rk) {
    for (int j = threadIdx.x; j < nwin; j += blockDim.x)
        window_round_keys(g, rank, w_lo + j, rk + kRoundKeyWords * j);
}

// virtual index inserted at step t (pool2 window w = 1 + t/B in Feistel order), given the
// window's round keys
__device__ __forceinline__ uint32_t ins_value_k(const Geometry &g, int64_t t, const uint32_t *k) {
    const int64_t w = 1 + t / g.B;
    const int64_t p = t - (w - 1) * g.B;
    const int64_t rem = g.ns - w * g.B;
    const uint32_t len = (uint32_t)(rem < g.B ? rem : g.B);
    return (uint32_t)(w * g.B) + feistel((uint32_t)p, len, feistel_half_bits(len), k);
}

__device__ __forceinline__ int64_t v2_id(uint32_t v, const RankDesc &rd, const Geometry &g) {
    return wrap_id(((int64_t)v < 2 * g.B ? rd.old_start : rd.new_start) + (int64_t)v, g.N);
}

// value held by slot s after tile `tile` (walk back over tiles that never drew s)
__device__ __forceinline__ uint32_t slot_value_after(const uint32_t *VALr, int64_t P1,
                                                     int64_t tile, int64_t s) {
    for (int64_t gg = tile; gg >= 0; gg--) {
        const uint32_t v = VALr[gg * P1 + s];
        if (v != kNone) return v;
    }
    return (uint32_t)s;  // initial pool1 = window 0 in slot order
}

// At most two waves per SIMD.  The replay kernels are sized for eight waves per CU (LDS padding
// caps the CU), but with <= 128 VGPRs a SIMD could take three or four of them and another one
// or none; the waves sharing a SIMD then run at a fraction of the issue rate and set the
// kernel's time.  Claiming VGPRs through v180 (> 512 / 3) leaves room for two per SIMD only.
#define PSS_TWO_WAVES_PER_SIMD() asm volatile("" ::: "v180")

// Progress-based wave priority.  Co-resident waves with equal work are arbitrated by age, so
// the older one runs ahead and the younger finishes alone at half the issue rate.  A wave
// lowers its own priority as it passes 1/4, 1/2 and 3/4 of its work: whoever is behind wins
// arbitration, and the waves of a SIMD finish together.
#ifndef PSS_PACER_MODE
#define PSS_PACER_MODE 0
#endif
struct Pacer {
    uint32_t next, quarter;
    int stage;
    uint32_t total_;
    __device__ __forceinline__ explicit Pacer(uint32_t total) {
        total_ = total;
        quarter = total / 4 + 1;
#if PSS_PACER_MODE == 1
        next = total - total / 4;
#else
        next = quarter;
#endif
        stage = 0;
#if PSS_PACER_MODE != 2
        __builtin_amdgcn_s_setprio(3);
#endif
    }
    __device__ __forceinline__ void step(uint32_t done) {
#if PSS_PACER_MODE == 2
        return;
#endif
        if (done < next) return;
        stage++;
#if PSS_PACER_MODE == 1
        next = stage == 1 ? total_ - total_ / 16 : stage == 2 ? total_ - total_ / 64 : ~0u;
#else
        next += quarter;
#endif
        if (stage == 1) __builtin_amdgcn_s_setprio(2);
        else if (stage == 2) __builtin_amdgcn_s_setprio(1);
        else __builtin_amdgcn_s_setprio(0);
    }
};


// global id of virtual index v (NARROW: every id and id + ns fits in 32 bits)
template <bool NARROW>
__device__ __forceinline__ int64_t emit_id(uint32_t v, uint32_t twoB, uint32_t old32, uint32_t new32,
                                           uint32_t N32, const RankDesc &rd, const Geometry &g) {
    if (NARROW) {
        const uint32_t id = (v < twoB ? old32 : new32) + v;
        const uint32_t idw = id - N32;
        return (int64_t)(id < N32 ? id : idw);
    }
    return v2_id(v, rd, g);
}

// ---- fused (file, offset) output of the V2 replay kernels (pss_generate_mapped) ------------------
// A replay wave's ids come, with overwhelming probability, from one interval of ids: the pool2
// windows of its tile and the kSegBackWin before it (a value survives a window of steps in a pool
// of <= B slots with probability <= e^-1).  The wave cuts that interval into kSegBuckets equal
// buckets and keeps, per bucket, its first file, the bucket's one file boundary (if any) and
// the first file's start -- three parallel LDS arrays, one independent read each per id.
// Buckets holding two or more boundaries, ids outside the interval and ids past the scanned
// total (reflected) take the global bucketed map (map_one_bucketed_t): results equal pss_map's.
constexpr uint32_t kSegBuckets = 256, kSegBackWin = 40;
constexpr uint32_t kSegLdsWords = 3 * kSegBuckets;
constexpr uint32_t kSegMulti = 0xFFFFu;    // bucket with >= 2 boundaries: global path

// id -> (file position, int32 offset): when every file holds uL samples (MapArgs::uni) and
// id < T, the file is id / uL -- one multiply-high by the host's magic, no table read -- else the
// global bucketed map; the same values pss_map gives either way
__device__ __forceinline__ void map_id_fast(const MapArgs &ma, int64_t id, int32_t &f, int32_t &off) {
    if (ma.uni && (uint64_t)id < (uint64_t)ma.T) {
        const uint32_t q = udiv_apply((uint32_t)id, ma.um, ma.ul);
        f = (int32_t)q;
        off = (int32_t)((uint32_t)id - q * ma.uL);
    } else {
        int64_t o;
        map_one_bucketed_t(ma.prefix, ma.F, ma.T, ma.BT, ma.kb, ma.nb, id, f, o);
        off = (int32_t)o;
    }
}

// exact orders (pss_v1exact.hip, pss_v2exact.hip): the id into out[e], or -- ma.fpos set, the
// fused hand-off of pss_generate_mapped -- its (file position, offset) pair, the same values
// pss_map gives
__device__ __forceinline__ void put_id_or_pair(int64_t *out, const MapArgs &ma, int64_t e, int64_t id) {
    if (ma.fpos) {
        int32_t f, o;
        map_id_fast(ma, id, f, o);
        ma.fpos[e] = f;
        ma.off[e] = o;
    } else {
        out[e] = id;
    }
}

// the global map for the rare ids the LDS buckets miss
__device__ __forceinline__ void seg_global_map(const MapArgs &ma, int64_t T, int64_t id,
                                               int32_t &f, int32_t &off) {
    (void)T;   // (ma.T, the same total)
    map_id_fast(ma, id, f, off);
}

struct SegMap {
    MapArgs ma;
    int64_t T;          // prefix[F]
    int64_t id_lo;      // [id_lo, id_lo + len) maps through LDS
    uint32_t len, kbm;
    int32_t f0;
    const uint32_t *fw;  // LDS: file of the bucket's start (relative to f0) | files to the one after its boundary << 16
    const int32_t *sw;   // LDS: the boundary (relative id), or INT32_MAX
    const int32_t *bw;   // LDS: start of the bucket's first file (relative id, may be < 0)

    // one wave (the whole workgroup) builds it; lds: kSegLdsWords words
    __device__ __forceinline__ void build(const MapArgs &m, int64_t lo, int64_t hi, uint32_t *lds,
                                          int lane) {
        ma = m;
        T = m.prefix[m.F];
        id_lo = lo;
        len = 0;
        kbm = 0;
        f0 = 0;
        uint32_t *fww = lds;
        int32_t *sww = (int32_t *)(lds + kSegBuckets), *bww = (int32_t *)(lds + 2 * kSegBuckets);
        fw = fww; sw = sww; bw = bww;
        if (hi > T) hi = T;                       // past the total: reflected ids, global path
        if (hi <= lo || hi - lo >= ((int64_t)1 << 30)) return;
        int32_t fa;
        int64_t o;
        map_one_bucketed_t(m.prefix, m.F, T, m.BT, m.kb, m.nb, lo, fa, o);
        if (fa < 0) return;
        const uint32_t L = (uint32_t)(hi - lo);
        uint32_t k = 0;
        while (((L - 1u) >> k) >= kSegBuckets) k++;
        // four buckets per lane, their global lookups interleaved
#pragma unroll
        for (int q = 0; q < (int)(kSegBuckets / 64); q++) {
            const uint32_t b = (uint32_t)lane + 64u * q;
            const int64_t r0 = (int64_t)b << k, r1 = (r0 + ((int64_t)1 << k)) < (int64_t)L ? r0 + ((int64_t)1 << k) : L;
            uint32_t word = kSegMulti << 16;
            int32_t split = INT32_MAX, base = 0;
            if (r0 < (int64_t)L) {
                int32_t f;
                map_one_bucketed_t(m.prefix, m.F, T, m.BT, m.kb, m.nb, lo + r0, f, o);
                const int64_t pa = m.prefix[f] - lo;                 // start of the bucket's first file
                const int64_t pb = f + 1 < m.F ? m.prefix[f + 1] - lo : (int64_t)L;   // its end
                uint32_t df = 0;
                if (pb < r1) {                                       // a boundary inside the bucket
                    int32_t fb;
                    map_one_bucketed_t(m.prefix, m.F, T, m.BT, m.kb, m.nb, lo + pb, fb, o);  // skips empty files
                    const int64_t pc = fb + 1 < m.F ? m.prefix[fb + 1] - lo : (int64_t)L;
                    df = pc < r1 ? kSegMulti : (uint32_t)(fb - f);
                    split = (int32_t)pb;
                }
                if (f - fa >= 0xFFFF || df > 0xFFFEu) df = kSegMulti;
                word = (uint32_t)(f - fa) | (df << 16);
                base = (int32_t)pa;
            }
            fww[b] = word;
            sww[b] = split;
            bww[b] = base;
        }
        __syncthreads();
        f0 = fa;
        kbm = k;
        len = L;
    }

    __device__ __forceinline__ void map(int64_t id, int32_t &f, int32_t &off) const {
        const uint64_t rel = (uint64_t)(id - id_lo);
        bool hit = false;
        if (rel < (uint64_t)len) {
            const int32_t r = (int32_t)rel;
            const uint32_t b = (uint32_t)r >> kbm;
            const uint32_t w = fw[b];
            const int32_t split = sw[b], base = bw[b];
            const uint32_t df = w >> 16;
            if (df != kSegMulti) {
                const bool up = r >= split;
                f = f0 + (int32_t)(w & 0xFFFFu) + (up ? (int32_t)df : 0);
                off = r - (up ? split : base);
                hit = true;
            }
        }
        if (!hit) seg_global_map(ma, T, id, f, off);
    }
};

// ---- packed-pair slots of the exchange replay (MapArgs::pack, pss_generate_mapped) -----------
// The slot table carries the pair (file << pob) | offset instead of the id.  It is computed where
// a value is inserted -- the inserted values of pool2 window w are the ids a + y, y < B, of one
// id interval, which crosses at most two file boundaries when files are not much shorter than
// the window: y -> y + Q_k on segment k, three SGPR constants and two compares -- so emitting a
// value is a shift and a mask.  Values without a pair (windows that wrap at N, reach past the
// scanned total T, or cross three or more file boundaries; slot-table values older than
// kPairBack windows at a tile's start) carry kPairEsc | virtual index and take the global
// bucketed map when emitted.  Results equal pss_map's.
constexpr uint32_t kPairEsc = 0x80000000u;
constexpr uint32_t kPairBack = 8;       // windows before the tile's first with constants
constexpr uint32_t kPairWords = 5;      // per window: Q0, Q1, Q2, s1, s2 (Q0 = kNone: no pairs)

// The map of one contiguous id interval [a, a + len) (a window's ids) as at most three segments:
// y < s1 -> (f0, d0 + y), s1 <= y < s2 -> (f1, y - s1), y >= s2 -> (f2, y - s2) -- s = kNone
// where a segment is absent.  False when the interval reaches past the scanned total T (reflected
// ids) or crosses three or more file boundaries.  Empty files are skipped as the map skips them.
__device__ __forceinline__ bool window_map_segments(const MapArgs &ma, int64_t a, int64_t len, int32_t f[3],
                                                    uint32_t &d0, uint32_t s[2]) {
    s[0] = kNone; s[1] = kNone;
    if (a < 0 || a + len > ma.T) return false;
    int64_t o;
    map_one_bucketed_t(ma.prefix, ma.F, ma.T, ma.BT, ma.kb, ma.nb, a, f[0], o);
    if (f[0] < 0) return false;
    d0 = (uint32_t)o;
    f[1] = f[2] = f[0];
    {   // the usual case in one round trip: the next three prefix entries, non-empty files
        const int64_t f0 = f[0];
        const int64_t p1 = ma.prefix[f0 + 1];
        const int64_t p2 = f0 + 2 <= ma.F ? ma.prefix[f0 + 2] : p1;
        const int64_t p3 = f0 + 3 <= ma.F ? ma.prefix[f0 + 3] : p2;
        if (p1 - a >= len) return true;                       // one file
        if (p2 > p1) {                                        // file f0 + 1 not empty
            s[0] = (uint32_t)(p1 - a);
            f[1] = f[2] = (int32_t)(f0 + 1);
            if (p2 - a >= len) return true;                   // two files
            if (p3 > p2) {
                s[1] = (uint32_t)(p2 - a);
                f[2] = (int32_t)(f0 + 2);
                return p3 - a >= len;                         // three files, else a third boundary
            }
        }
        s[0] = kNone; s[1] = kNone;                           // empty files: the general walk
        f[1] = f[2] = f[0];
    }
    for (int k = 0; k < 3; k++) {
        const int64_t end = ma.prefix[f[k] + 1] - a;   // the next file boundary (prefix[F] = T)
        if (end >= len) return true;
        if (k == 2) return false;                      // a third boundary
        int64_t ob;
        map_one_bucketed_t(ma.prefix, ma.F, ma.T, ma.BT, ma.kb, ma.nb, a + end, f[k + 1], ob);
        if (k == 0) f[2] = f[1];
        s[k] = (uint32_t)end;
    }
    return true;
}

// constants of pool2 window w (virtual values [w B, w B + len)) of rank rd into c[kPairWords]
__device__ __forceinline__ void pair_window_consts(const MapArgs &ma, const RankDesc &rd, const Geometry &g,
                                                   uint32_t B, uint32_t twoB, uint32_t w, uint32_t *c) {
    c[0] = kNone; c[1] = 0u; c[2] = 0u; c[3] = kNone; c[4] = kNone;
    const int64_t v0 = (int64_t)w * B;
    if (v0 >= g.ns) return;
    const int64_t len = g.ns - v0 < (int64_t)B ? g.ns - v0 : (int64_t)B;
    if (v0 < (int64_t)twoB && v0 + len > (int64_t)twoB) return;   // (2B and ns are window ends)
    int64_t a = (v0 < (int64_t)twoB ? rd.old_start : rd.new_start) + v0;
    if (a >= g.N) a -= g.N;
    if (a + len > g.N) return;                                    // wraps inside the window
    int32_t f[3];
    uint32_t d0, s[2];
    if (!window_map_segments(ma, a, len, f, d0, s)) return;
    c[0] = ((uint32_t)f[0] << ma.pob) + d0;
    c[1] = ((uint32_t)f[1] << ma.pob) - s[0];
    c[2] = ((uint32_t)f[2] << ma.pob) - s[1];
    c[3] = s[0];
    c[4] = s[1];
}

// the pair of value y of a window with constants (Q0, Q1, Q2, s1, s2)
__device__ __forceinline__ uint32_t pair_of_y(uint32_t y, uint32_t Q0, uint32_t Q1, uint32_t Q2, uint32_t s1,
                                              uint32_t s2) {
    return y + (y < s1 ? Q0 : (y < s2 ? Q1 : Q2));
}

// The id interval staged for virtual values [v_lo, v_hi) of one rank: ids are base + v (base =
// old start below twoB, new start above) wrapped modulo N, so the values may map to two or three
// id intervals; the one holding the value v_pref (the tile's own first window) is staged.
__device__ __forceinline__ void seg_interval(uint32_t v_lo, uint32_t v_hi, uint32_t v_pref,
                                             uint32_t twoB, const RankDesc &rd, const Geometry &g,
                                             int64_t &lo, int64_t &hi) {
    lo = hi = 0;
    if (v_hi <= v_lo) return;
    if (v_lo < twoB && v_hi > twoB) {
        if (v_pref < twoB) v_hi = twoB;
        else v_lo = twoB;
    }
    const int64_t base = v_lo < twoB ? rd.old_start : rd.new_start;
    const int64_t a = base + v_lo, b = base + v_hi, p = base + v_pref;
    if (b <= g.N) { lo = a; hi = b; }
    else if (a >= g.N) { lo = a - g.N; hi = b - g.N; }
    else if (p >= g.N) { lo = 0; hi = b - g.N; }
    else { lo = a; hi = g.N; }
}

}  // namespace pss
