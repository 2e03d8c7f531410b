// pss_v2.hip -- the V2 two-pool shuffle buffer (V2:96-116) in slot-replacement form
// (DESIGN.md §3.3):
//
//   k_v2_lastocc     pass A, slot table in LDS: per tile the last step that drew each slot
//                    (order-independent ds_max) -> VAL[tile][s] = value inserted there
//   k_v2_emit        pass B: one wave replays a tile in step order, 64 steps per iteration;
//                    each step exchanges its insertion into the drawn slot (ds_wrxchg_rtn /
//                    global_atomic_swap) and emits what it held; lanes of one iteration that
//                    drew the same slot are chained through ds_bpermute instead
//   k_v2_emit_x      pass B on gfx950: one lane-ordered LDS exchange per step; the wave of a
//                    rank's last tile also drains the final pool (the tail) from LDS
//   k_v2_tail_f      the tail from the VAL tables, when the last tile is not replayed in the
//                    same launch (or on the probe path): final pool1 drained in the order of
//                    a keyed Feistel bijection of [0, P1)
// Pools beyond LDS (P1 > kLdsSlotMax) take the grouped schedule of pss_v2grp.hip.
#include <cstdlib>
#include <type_traits>
#include <vector>

#include "pss_device.h"

namespace pss {


static inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

__device__ __forceinline__ void tile_bounds(const V2Plan &pl, int64_t tile, int64_t &tlo,
                                            int64_t &thi) {
    tlo = tile * pl.L;
    thi = tlo + pl.L < pl.T ? tlo + pl.L : pl.T;
}

#ifdef PSS_STAMPS   // diagnostic build only (tools/stamp_v2.hip): per-workgroup phase clocks
__device__ uint64_t pss_stamps[1 << 16][8];
#define PSS_STAMP(i) do { if (threadIdx.x == 0 && blockIdx.x < (1u << 16)) pss_stamps[blockIdx.x][i] = __builtin_amdgcn_s_memtime(); } while (0)
#define PSS_STAMPW(i) do { if ((threadIdx.x & 63) == 0 && blockIdx.x < (1u << 16)) pss_stamps[blockIdx.x][i] = __builtin_amdgcn_s_memtime(); } while (0)
#ifndef PSS_STAMPS_EMIT_ONLY   // (a pass running beside the replay would overwrite its slots)
#define PSS_PASS_STAMPS 1
#else
#undef PSS_STAMP
#define PSS_STAMP(i) do { } while (0)
#endif
#else
#define PSS_STAMP(i) do { } while (0)
#endif

// ---- pass A, LDS ----------------------------------------------------------------------------
// Per tile: the last step (tile-local, +1) that drew each slot (ds_max in any order), then that
// step's inserted value.
template <int NT, bool POW2>
__global__ __launch_bounds__(NT) void k_v2_lastocc(Geometry g, V2Plan pl, int32_t rank_lo,
                                                   int64_t ng, uint32_t *__restrict__ VAL) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    PSS_STAMP(0);
    const int P1 = (int)pl.P1;
    uint32_t *lastT = smem, *rk = smem + P1;
    // 32-bit tile arithmetic from the plan's host-computed constants (T < 2^32)
    const uint32_t ngu = (uint32_t)ng, B = pl.B32;
    const int32_t rl = (int32_t)(blockIdx.x / ngu);
    const uint32_t tile = blockIdx.x - (uint32_t)rl * ngu;
    const uint32_t rank = (uint32_t)(rank_lo + rl);
    const uint32_t tlo = tile * pl.L32;
    const uint32_t thi = pl.T32 - tlo < pl.L32 ? pl.T32 : tlo + pl.L32;
    const uint32_t w_lo = 1 + tlo / B;
    const int nwin = (int)(1 + (thi - 1) / B - w_lo + 1);
#ifdef PSS_PASS_STAMPS
    if (threadIdx.x == 0) pss_stamps[blockIdx.x][4] = __builtin_amdgcn_s_memrealtime();
#endif
    for (int s = threadIdx.x; s < P1; s += NT) lastT[s] = 0;
    stage_keys(g, rank, w_lo, nwin, rk);
    const SlotKey sk = slot_key(g, rank);
    __syncthreads();
    PSS_STAMP(1);
    // whole blocks of 8*NT steps run branch-free with 8 independent hashes per thread
    const uint32_t n = (uint32_t)(thi - tlo), t0 = (uint32_t)tlo;
    const uint32_t sh = 32u - (uint32_t)ceil_log2_u64((uint64_t)P1);   // POW2 only
    constexpr uint32_t BLK = 8 * NT;
    const uint32_t nfull = n / BLK * BLK;
    // Loop counters are workgroup-uniform (base), never per-lane: with a per-lane trip count the
    // compiler may unroll per thread, and lanes would then run different steps in one store.
    Pacer pace(nfull);
    for (uint32_t base = 0; base < nfull; base += BLK) {
        pace.step(base);
        // thread -> 8 steps: (t, t + 64) pairs of 4 different 128-step groups, so that with
        // a paired draw (POW2) one hash serves two steps
        uint32_t st[8], k[8];
#pragma unroll
        for (int j = 0; j < 8; j++)
            st[j] = base + 128u * ((threadIdx.x >> 6) + (NT / 64) * (j >> 1)) + 64u * (j & 1) + (threadIdx.x & 63u);
        if (POW2) {
            // t0 + base is a multiple of 256, so the pair index of st[j] (j even) is
            // (t0 + base) / 2 + 64 (wave + NT/64 (j/2)) + lane: one add of a per-thread constant
            const uint32_t pb = (t0 + base) >> 1;
#pragma unroll
            for (int j = 0; j < 8; j += 2) {
                const uint32_t c = 64u * ((threadIdx.x >> 6) + (NT / 64) * (j >> 1)) + (threadIdx.x & 63u);
                const uint32_t u = slot_hash(pb + c, sk.s0, sk.s1);
                k[j] = u >> sh;
                k[j + 1] = (u & 0xFFFFu) >> (sh - 16u);
            }
        } else {
#pragma unroll
            for (int j = 0; j < 8; j++) k[j] = slot_draw(t0 + st[j], sk.s0, sk.s1, (uint32_t)P1);
        }
#pragma unroll
        for (int j = 0; j < 8; j++) atomicMax(&lastT[k[j]], st[j] + 1u);
    }
    for (uint32_t base = nfull; base < n; base += NT) {
        const uint32_t b = base + threadIdx.x;
        if (b < n) {
            const uint32_t kk = slot_draw(t0 + b, sk.s0, sk.s1, (uint32_t)P1);
            atomicMax(&lastT[kk], b + 1u);
        }
    }
    __syncthreads();
    PSS_STAMP(2);
    // last step -> inserted value, in 32-bit tile-local arithmetic (no 64-bit division)
    uint32_t *V = VAL + ((int64_t)rl * pl.G + tile) * P1;
    const uint32_t hB = pl.hB, w_last = pl.w_last, len_last = pl.len_last, h_last = pl.h_last;
    const uint32_t p_lo = tlo - (w_lo - 1) * B;                 // index of step tlo in window w_lo
    const bool walk_full = pl.walk_full;
    const float invB = 1.0f / (float)B;
    // 4 slots per thread per pass (independent chains); a whole pass takes the one-pass
    // Feistel unless one of its slots lies in the short last window or B needs cycle walking
    for (int s0 = threadIdx.x; s0 < P1; s0 += 4 * NT) {
        uint32_t lt[4], pp[4], dw[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int s = s0 + u * NT;
            lt[u] = s < P1 ? lastT[s] : 0u;
            const uint32_t p = p_lo + lt[u] - 1u;        // < L + B < 2^24: exact in float
            uint32_t d = (uint32_t)((float)p * invB);    // p / B to within one, then corrected
            int32_t r = (int32_t)(p - d * B);
            if (r < 0) { d--; r += (int32_t)B; }
            if (r >= (int32_t)B) { d++; r -= (int32_t)B; }
            pp[u] = (uint32_t)r;
            dw[u] = lt[u] ? d : 0u;
        }
        bool slow = walk_full;
#pragma unroll
        for (int u = 0; u < 4; u++) slow |= lt[u] && (uint32_t)w_lo + dw[u] == w_last;
        uint32_t x[4];
        if (!slow && feistel_packed_ok(hB)) {
            // two chains per register on the packed 16-bit round function, each with its own
            // window's keys (the slots' last steps lie in different windows)
            feistel2_pk16_k2(pp[0], pp[1], hB, rk + kRoundKeyWords * dw[0], rk + kRoundKeyWords * dw[1], x[0], x[1]);
            feistel2_pk16_k2(pp[2], pp[3], hB, rk + kRoundKeyWords * dw[2], rk + kRoundKeyWords * dw[3], x[2], x[3]);
        } else if (!slow) {
#pragma unroll
            for (int u = 0; u < 4; u++) x[u] = feistel_once(pp[u], hB, rk + kRoundKeyWords * dw[u]);
        } else {
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const bool lastw = (uint32_t)w_lo + dw[u] == w_last;
                x[u] = lt[u] ? feistel(pp[u], lastw ? len_last : B, lastw ? h_last : hB, rk + kRoundKeyWords * dw[u]) : 0u;
            }
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int s = s0 + u * NT;
            if (s < P1) V[s] = lt[u] ? ((uint32_t)w_lo + dw[u]) * B + x[u] : kNone;
        }
    }
    PSS_STAMP(3);
#ifdef PSS_PASS_STAMPS
    if (threadIdx.x == 0) {
        pss_stamps[blockIdx.x][5] = __builtin_amdgcn_s_memrealtime();
        pss_stamps[blockIdx.x][6] = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));
        pss_stamps[blockIdx.x][7] = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (15 << 11));
    }
#endif
}

// ---- pass B -------------------------------------------------------------------------------
// collision probe bytes live in LDS and are accessed volatile (the read-back must not be
// forwarded from the store); the explicit address space keeps them ds_write_b8/ds_read_u8
// (a generic volatile pointer lowers to flat sc0 sc1 accesses)
typedef __attribute__((address_space(3))) volatile uint8_t lds_vu8;

// FOLD (every virtual id < 2^24): the probe byte of slot k is the top byte of buf[k] itself
// (values live in bits 0..23), so the wave needs no separate probe array -- 16 KB of LDS per
// wave at P1 = 4096 instead of 20 KB, i.e. 8 instead of 7 waves per CU (2 per SIMD)
template <bool FOLD>
struct EmitCtx {   // per-tile constants of k_v2_emit + the running pool2 position (w0, p0)
    static constexpr uint32_t kValMask = FOLD ? 0x00FFFFFFu : 0xFFFFFFFFu;
    __device__ __forceinline__ static uint32_t probe_ix(uint32_t k) {
        return FOLD ? (k << 2) : (k & (uint32_t)(kMarkBytes - 1));
    }
    uint64_t lt_mask;
    uint32_t *buf;
    lds_vu8 *mark;
    const uint32_t *rk;
    int64_t *o;
    const Geometry *g;
    RankDesc rd;
    int lane;
    uint32_t P1, nvalid, e_lo, e_hi;
    uint32_t twoB, old32, new32, N32;
    uint32_t B, hB, w_last, len_last, h_last, w_lo;
    bool walk_full;
    uint32_t w0, p0;

    // One 64-step sub-batch (lane l = step tl) in two halves, so that the next sub-batch's
    // prep (ALU work + probe) can be issued while this one's LDS round trips are in flight.
    struct Step { uint32_t k, ins, probe; int32_t tl; bool valid; };

    // FAST: every step valid, B >= 64 (at most one window boundary per sub-batch) and no
    // step in the last (short) window or in a cycle-walking window -- straight-line code.
    template <bool FAST>
    __device__ __forceinline__ Step prep(uint32_t uword, int32_t tl) {
        Step s;
        s.tl = tl;
        s.valid = FAST || (uint32_t)tl < nvalid;
        s.k = uword;   // the step's slot (slot_ks)
        // collision probe: a lane that reads back another lane's id shares its probe byte
        // (slot & 4095) with a lane of this sub-batch
        const uint32_t hk = probe_ix(s.k);
        if (s.valid) mark[hk] = (uint8_t)lane;
        s.probe = mark[hk];
        // insertion of step t: window w, index p
        uint32_t p = p0 + (uint32_t)lane;
        uint32_t w = w0;
        if (FAST) {
            const bool cross = p >= B;
            p = cross ? p - B : p;
            w = cross ? w + 1 : w;
            s.ins = w * B + feistel_once(p, hB, rk + kRoundKeyWords * (w - w_lo));
        } else {
            while (p >= B) { p -= B; w++; }
            s.ins = 0;
            if (s.valid) {
                const bool lastw = w == w_last;
                s.ins = w * B + feistel(p, lastw ? len_last : B, lastw ? h_last : hB,
                                        rk + kRoundKeyWords * (w - w_lo));
            }
        }
        p0 += 64;
        if (FAST) {
            const bool c2 = p0 >= B;
            p0 = c2 ? p0 - B : p0;
            w0 = c2 ? w0 + 1 : w0;
        } else {
            while (p0 >= B) { p0 -= B; w0++; }
        }
        return s;
    }

    // Fast super-batch, first half: slots + probes of its 4 sub-batches (in order: the probe
    // of sub-batch j+1 is written after sub-batch j's read-back) ...
    __device__ __forceinline__ Step probe4(uint32_t uword, int32_t tl) {
        Step s;
        s.tl = tl;
        s.valid = true;
        s.k = uword;   // the step's slot (slot_ks)
        const uint32_t hk = probe_ix(s.k);
        mark[hk] = (uint8_t)lane;
        s.probe = mark[hk];
        return s;
    }
    // ... second half: insertion value of sub-batch j (B >= 256: at most one window boundary
    // inside the super-batch; no last / cycle-walking window).  Independent of the other
    // three, so the four Feistel chains interleave.
    __device__ __forceinline__ uint32_t ins4(int j) const {
        uint32_t p = p0 + (uint32_t)(64 * j + lane);
        const bool cross = p >= B;
        p = cross ? p - B : p;
        const uint32_t w = cross ? w0 + 1 : w0;
        return w * B + feistel_once(p, hB, rk + kRoundKeyWords * (w - w_lo));
    }
    __device__ __forceinline__ void advance256() {
        p0 += 256;
        const bool c2 = p0 >= B;
        p0 = c2 ? p0 - B : p0;
        w0 = c2 ? w0 + 1 : w0;
    }

    template <bool FAST, bool NARROW>
    __device__ __forceinline__ void finish(const Step &s) {
        const bool clash = s.valid && s.probe != (uint32_t)lane;
        uint64_t cm = __ballot(clash);
        uint32_t v;
        if (cm == 0) {
            // every valid lane drew a distinct slot: emit its content, insert in one op
            v = (FAST || s.valid) ? atomicExch(&buf[s.k], s.ins) & kValMask : 0u;
        } else {
            // peers = lanes that drew the same slot; the first of them exchanges the LAST
            // peer's insertion, the others take the previous peer's insertion
            uint64_t m = s.valid ? (1ull << lane) : 0ull;
            while (cm) {
                const int cl = __ffsll((long long)cm) - 1;
                const uint32_t sc = (uint32_t)__builtin_amdgcn_readlane((int)s.k, cl);
                const bool same = s.valid && s.k == sc;
                const uint64_t mm = __ballot(same);
                if (same) m = mm;
                cm &= ~mm;
            }
            const uint64_t lower = m & lt_mask;
            const int hi_lane = m ? 63 - __clzll((long long)m) : lane;
            const int prev_lane = lower ? 63 - __clzll((long long)lower) : lane;
            const uint32_t ins_last = (uint32_t)__shfl((int)s.ins, hi_lane);
            const uint32_t ins_prev = (uint32_t)__shfl((int)s.ins, prev_lane);
            v = (s.valid && !lower) ? atomicExch(&buf[s.k], ins_last) & kValMask : ins_prev;
        }
        if (FAST || ((uint32_t)s.tl >= e_lo && (uint32_t)s.tl < e_hi)) {
            if (NARROW) {
                uint32_t id = (v < twoB ? old32 : new32) + v;
                id = id >= N32 ? id - N32 : id;
                o[s.tl] = (int64_t)id;
            } else {
                o[s.tl] = v2_id(v, rd, *g);
            }
        }
    }
};

template <bool NARROW, bool FOLD>
__global__ __launch_bounds__(64) void k_v2_emit(Geometry g, V2Plan pl,
                                                const RankDesc *__restrict__ ranks,
                                                int32_t rank_lo, int64_t g_lo, int64_t ng,
                                                const uint32_t *__restrict__ VAL,
                                                int64_t pos_lo, int64_t count,
                                                int64_t *__restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    const int64_t P1 = pl.P1;
    const int64_t nwin_max = pl.L / g.B + 2;
    uint32_t *rk = smem;                                    // Feistel keys of the tile's windows
    // collision probe: kMarkBytes of its own, or (FOLD) the top byte of each slot word
    const int mark_words = FOLD ? 0 : kMarkBytes / 4;
    lds_vu8 *mark = (lds_vu8 *)(rk + kRoundKeyWords * nwin_max);
    const int lane = threadIdx.x;
    const int32_t rl = (int32_t)(blockIdx.x / ng);
    const int64_t tile = g_lo + (int64_t)(blockIdx.x % ng);
    const uint32_t rank = (uint32_t)(rank_lo + rl);
    const RankDesc rd = ranks[rank];
    int64_t tlo, thi;
    tile_bounds(pl, tile, tlo, thi);
    const int64_t w_lo = 1 + tlo / g.B;
    const int nwin = (int)(1 + (thi - 1) / g.B - w_lo + 1);
    uint32_t *buf;   // slot table: virtual ids held by the P1 slots at the tile's start
    {
        buf = (uint32_t *)(smem + kRoundKeyWords * nwin_max + mark_words);
        if (FOLD) mark = (lds_vu8 *)buf + 3;
        const uint32_t *VALr = VAL + (int64_t)rl * pl.G * P1;
        const uint32_t *prev = VALr + (tile - 1) * P1;
        for (int64_t s0 = lane; s0 < P1; s0 += 256) {       // 4 independent loads in flight
            uint32_t v[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int64_t s = s0 + 64 * u;
                v[u] = (tile > 0 && s < P1) ? prev[s] : kNone;
            }
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int64_t s = s0 + 64 * u;
                if (s < P1) buf[s] = v[u] != kNone ? v[u] : slot_value_after(VALr, P1, tile - 2, s);
            }
        }
    }
    stage_keys(g, rank, w_lo, nwin, rk);
    __syncthreads();
    EmitCtx<FOLD> c;
    c.lane = lane;
    c.lt_mask = (1ull << lane) - 1ull;
    c.P1 = (uint32_t)P1;
    c.buf = buf;
    c.mark = mark;
    c.rk = rk;
    const int64_t sb_lo = tlo >> 8, sb_hi = (thi - 1) >> 8;
    // tile-local 32-bit step index tl = t - tlo; the tile emits tl in [e_lo, e_hi)
    const int64_t pos_hi = pos_lo + count;
    c.nvalid = (uint32_t)(thi - tlo);
    c.e_lo = (uint32_t)(pos_lo > tlo ? (pos_lo - tlo < c.nvalid ? pos_lo - tlo : c.nvalid) : 0);
    c.e_hi = (uint32_t)(pos_hi < thi ? (pos_hi > tlo ? pos_hi - tlo : 0) : c.nvalid);
    c.o = out + (int64_t)rl * count + (tlo - pos_lo);
    // ids: v < 2B came from the OLD start, the rest from the NEW one
    c.twoB = (uint32_t)(2 * g.B < g.ns ? 2 * g.B : g.ns);
    c.old32 = (uint32_t)rd.old_start; c.new32 = (uint32_t)rd.new_start;
    c.N32 = (uint32_t)g.N;
    c.rd = rd;
    c.g = &g;
    // pool2 window bookkeeping without per-step division: (w0, p0) = window and insertion
    // index of the sub-batch's first step t0, advanced by 64 per sub-batch.
    c.B = (uint32_t)g.B;
    c.hB = feistel_half_bits(c.B);
    c.walk_full = c.B != (1u << (2 * c.hB));      // full windows need cycle walking
    c.w_last = (uint32_t)(1 + (pl.T - 1) / g.B);  // last pool2 window (may be short)
    c.len_last = (uint32_t)(g.ns - (int64_t)c.w_last * g.B);
    c.h_last = feistel_half_bits(c.len_last);
    c.w_lo = (uint32_t)w_lo;
    const int64_t t_first = sb_lo * 256;
    c.w0 = (uint32_t)(1 + t_first / g.B);
    c.p0 = (uint32_t)(t_first - (int64_t)(c.w0 - 1) * g.B);
    // fast super-batches: fully valid and emitted, B >= 256, and no window touched that is
    // the last one or needs cycle walking (windows w0 .. w0 + 1)
    const bool fast_tile = c.e_lo == 0 && c.e_hi == c.nvalid && c.B >= 256 && !c.walk_full;
    int32_t tl0 = (int32_t)(t_first - tlo);   // negative while the super-batch starts before the tile
    const SlotKey sk = slot_key(g, rank);
    uint32_t u[4];
    slot_ks(sk, sb_lo, lane, c.P1, u);
    for (int64_t sb = sb_lo; sb <= sb_hi; sb++, tl0 += 256) {
        uint32_t un[4];   // next super-batch's slot words, computed under this one's work
        if (fast_tile && tl0 >= 0 && (uint32_t)tl0 + 256 <= c.nvalid && c.w0 + 1 < c.w_last) {
            // one branch-free block: 4 probes, 4 independent Feistel chains and the next
            // Philox block interleave; then the 4 sub-batches finish in step order
            typename EmitCtx<FOLD>::Step s[4];
#pragma unroll
            for (int j = 0; j < 4; j++) s[j] = c.probe4(u[j], tl0 + 64 * j + lane);
#pragma unroll
            for (int j = 0; j < 4; j++) s[j].ins = c.ins4(j);
            slot_ks(sk, sb + 1, lane, c.P1, un);
            c.advance256();
#pragma unroll
            for (int j = 0; j < 4; j++) c.template finish<true, NARROW>(s[j]);
        } else {
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const typename EmitCtx<FOLD>::Step s = c.template prep<false>(u[j], tl0 + j * 64 + lane);
                c.template finish<false, NARROW>(s);
            }
            slot_ks(sk, sb + 1, lane, c.P1, un);
        }
#pragma unroll
        for (int j = 0; j < 4; j++) u[j] = un[j];
    }
}

// ---- pass B, exchange-ordered (the default on gfx950) --------------------------------------
// One ds_wrxchg_rtn_b32 whose lanes hit the same LDS word behaves on gfx950 like the lanes
// exchanging one after another in ascending lane order (checked at start-up by
// k_xchg_order_check below, and tools/lds_xchg_order.hip): lane l gets the value the highest
// lower lane on that slot inserted, the lowest gets the slot's content, the slot ends with the
// highest lane's insertion.  That is exactly the sequential replay of 64 consecutive steps, so
// each step is ONE exchange -- no probe, no ballot, no per-clash fix-up -- and the four
// exchanges of a super-batch issue back to back behind a single wait.
// MAPPED: (int32 file position, int32 offset) into ma.fpos / ma.off instead of int64 ids into
// out -- PAIR: the slot table carries packed pairs (MapArgs::pack, pair_window_consts), emitting
// is a shift and a mask; else through the wave's LDS segment map (SegMap, pss_device.h)
template <bool NARROW, bool POW2, bool MAPPED, bool PAIR = false>
__global__ __launch_bounds__(64) void k_v2_emit_x(Geometry g, V2Plan pl,
                                                  const RankDesc *__restrict__ ranks,
                                                  int32_t rank_lo, int64_t g_lo, int64_t ng,
                                                  const uint32_t *__restrict__ VAL,
                                                  int64_t pos_lo, int64_t count, int do_tail,
                                                  int64_t *__restrict__ out, MapArgs ma, RankArgs ra,
                                                  int use_ra) {
    static_assert(MAPPED || !PAIR, "pair slots are a form of the mapped replay");
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    PSS_TWO_WAVES_PER_SIMD();
#ifdef PSS_STAMPS
    if (threadIdx.x == 0 && blockIdx.x < (1u << 16)) pss_stamps[blockIdx.x][2] = __builtin_amdgcn_s_memrealtime();
#endif
    const uint32_t P1 = (uint32_t)pl.P1;
    const uint32_t B = pl.B32;
    const uint32_t nwin_max = pl.L32 / B + 2;
    // slot table at LDS offset 0 (exchange addresses are 4 * slot, no base add), then the
    // Feistel keys of the tile's windows (MAPPED: then the segment map)
    uint32_t *buf = smem;
    uint32_t *rk = smem + ((P1 + 3u) & ~3u);
    const int lane = threadIdx.x;
    // 32-bit tile arithmetic from the plan's host-computed constants (T < 2^32)
    const uint32_t ngu = (uint32_t)ng;
    const int32_t rl = (int32_t)(blockIdx.x / ngu);
#ifdef PSS_DIAG_TILE_SWAP   // (diagnostic build, tools/stamp_v2x.hip: adjacent tiles trade XCDs)
    const uint32_t tile = (uint32_t)g_lo + ((blockIdx.x - (uint32_t)rl * ngu) ^ 1u);
#else
    const uint32_t tile = (uint32_t)g_lo + (blockIdx.x - (uint32_t)rl * ngu);
#endif
    const uint32_t rank = (uint32_t)(rank_lo + rl);
    const RankDesc rd = use_ra ? ra.r[rl] : ranks[rank];   // (kernel argument: a scalar load)
    const uint32_t twoB = pl.twoB;
    const uint32_t old32 = (uint32_t)rd.old_start, new32 = (uint32_t)rd.new_start;
    const uint32_t N32 = (uint32_t)g.N;
    const uint32_t tlo = tile * pl.L32;
    const uint32_t thi = pl.T32 - tlo < pl.L32 ? pl.T32 : tlo + pl.L32;
    const uint32_t w_lo = 1 + tlo / B;
    const int nwin = (int)(1 + (thi - 1) / B - w_lo + 1);
    // PAIR: the pair constants of the tile's windows and the kPairBack before them (after the
    // round keys), one lane per window
    uint32_t *pw = rk + kRoundKeyWords * nwin_max;
    const uint32_t wc_lo = w_lo > kPairBack ? w_lo - kPairBack : 0u;
    const uint32_t nwc = w_lo + (uint32_t)nwin - wc_lo;
    const uint32_t pob = ma.pob, omask = (1u << pob) - 1u;
    // (computed while the slot table's loads are in flight: both are chains of global loads)
    auto pair_consts = [&]() {
        if constexpr (PAIR) {
            for (uint32_t i = lane; i < nwc; i += 64) pair_window_consts(ma, rd, g, B, twoB, wc_lo + i, pw + kPairWords * i);
            __syncthreads();
        }
    };
    const float invB = 1.0f / (float)B;
    // PAIR, one lane: the pair of virtual value v from its window's constants, else an escape
    auto pair_lookup = [&](uint32_t v) -> uint32_t {
        uint32_t w = (uint32_t)((float)v * invB);     // v / B to within one (v < 2^31), corrected
        int32_t y = (int32_t)(v - w * B);
        if (y < 0) { w--; y += (int32_t)B; }
        if (y >= (int32_t)B) { w++; y -= (int32_t)B; }
        const uint32_t i = w - wc_lo;
        if (i < nwc) {
            const uint32_t *c = pw + kPairWords * i;
            const uint32_t Q0 = c[0];
            if (Q0 != kNone) return pair_of_y((uint32_t)y, Q0, c[1], c[2], c[3], c[4]);
        }
        return kPairEsc | v;
    };
    // NARROW: the slot table holds final ids (converted on insertion, emitted as they come out
    // of the exchange); PAIR: (file, offset) pairs (or escaped virtual indices); otherwise
    // virtual indices, converted on emission
    auto to_slot = [&](uint32_t v) -> uint32_t {
        if constexpr (PAIR) return pair_lookup(v);
        else if constexpr (NARROW) return (uint32_t)emit_id<true>(v, twoB, old32, new32, N32, rd, g);
        else return v;
    };
    auto from_slot = [&](uint32_t x) -> int64_t {
        if constexpr (NARROW && !PAIR) return (int64_t)x;
        else return emit_id<false>(x, twoB, old32, new32, N32, rd, g);
    };
    const SlotKey sk = slot_key(g, rank);
    {   // slot table at the tile's start: 16-byte loads, up to 16 per lane in flight (the whole
        // 16 KB table of P1 = 4096 in one round trip); slots the previous tile never drew walk
        // back further (probability e^-(L/P1))
        const uint32_t *VALr = VAL + (int64_t)rl * pl.G * pl.P1;
        const uint32_t *prev = VALr + ((int64_t)tile - 1) * pl.P1;   // tile 0: never read
        if (tile == 0) {
            pair_consts();
            for (uint32_t s = lane; s < P1; s += 64) buf[s] = to_slot(s);
        } else if ((P1 & 4095u) == 0) {
            // rounds of 16 x 64 quads, every load of a round in flight at once (P1 % 4096 == 0:
            // whole rounds -- round 5 took this path for P1 % 1024 == 0 and, at P1 = 1024 / 2048
            // / 3072 / 5120 ..., read the next tile's table and wrote past this one in LDS; those
            // pools now take the loop below)
            const uint4 *p4 = (const uint4 *)prev;
            for (uint32_t q0 = 0; q0 < P1 / 4; q0 += 1024) {
                uint4 v[16];
#pragma unroll
                for (int u = 0; u < 16; u++) v[u] = p4[q0 + 64u * u + lane];
                if (q0 == 0) pair_consts();
#pragma unroll
                for (int u = 0; u < 16; u++) {
                    const uint32_t q = q0 + 64u * u + lane;
                    uint32_t w[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
                    for (int c = 0; c < 4; c++)
                        w[c] = to_slot(w[c] != kNone ? w[c] : slot_value_after(VALr, pl.P1, (int64_t)tile - 2, 4 * q + c));
                    *(uint4 *)(buf + 4 * q) = make_uint4(w[0], w[1], w[2], w[3]);
                }
            }
        } else {
            pair_consts();
            for (uint32_t s0 = lane; s0 < P1; s0 += 256) {
                uint32_t v[4];
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const uint32_t s = s0 + 64 * u;
                    v[u] = s < P1 ? prev[s] : kNone;
                }
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const uint32_t s = s0 + 64 * u;
                    if (s < P1) buf[s] = to_slot(v[u] != kNone ? v[u] : slot_value_after(VALr, pl.P1, (int64_t)tile - 2, s));
                }
            }
        }
    }
    stage_keys(g, rank, w_lo, nwin, rk);
    __syncthreads();
    // tile-local step tl = t - tlo (tlo is a multiple of 256); the tile emits tl in [e_lo, e_hi)
    const int64_t pos_hi = pos_lo + count;
    const uint32_t nvalid = thi - tlo;
    const uint32_t e_lo = (uint32_t)(pos_lo > tlo ? (pos_lo - tlo < nvalid ? pos_lo - tlo : nvalid) : 0);
    const uint32_t e_hi = (uint32_t)(pos_hi < thi ? (pos_hi > tlo ? pos_hi - tlo : 0) : nvalid);
    int64_t *o = out + (int64_t)rl * count + ((int64_t)tlo - pos_lo);
    const int64_t ebase = (int64_t)rl * count + ((int64_t)tlo - pos_lo);   // element index of tl = 0
    SegMap sm;
    if constexpr (MAPPED && !PAIR) {
        // ids of the tile's windows and the kSegBackWin before them
        const uint32_t vl = w_lo > kSegBackWin ? (w_lo - kSegBackWin) * B : 0u;
        const int64_t vh64 = (int64_t)(w_lo + (uint32_t)nwin) * B;
        const uint32_t vh = (uint32_t)(vh64 < g.ns ? vh64 : g.ns);
        int64_t lo, hi;
        seg_interval(vl, vh, w_lo * B, twoB, rd, g, lo, hi);
        sm.build(ma, lo, hi, rk + kRoundKeyWords * nwin_max, lane);
    }
    auto put_m = [&](int64_t e, int64_t id) {
        int32_t f, of;
#ifdef PSS_DIAG_MAP_NONE   // (timing-only build: the stores of the mapped form without the map)
        f = (int32_t)id; of = (int32_t)(id >> 3);
#else
        sm.map(id, f, of);
#endif
        ma.fpos[e] = f;
        ma.off[e] = of;
    };
    // emit slot value x at element e: MAPPED + PAIR the pair itself (an escaped value through the
    // global bucketed map), MAPPED its id through the segment map, else the id
    auto emit_m = [&](int64_t e, uint32_t x) {
        if constexpr (PAIR) {
            int32_t f, of;
            if (x & kPairEsc) {
                map_id_fast(ma, from_slot(x & ~kPairEsc), f, of);
            } else {
                f = (int32_t)(x >> pob);
                of = (int32_t)(x & omask);
            }
            ma.fpos[e] = f;
            ma.off[e] = of;
        } else if constexpr (MAPPED) {
            put_m(e, from_slot(x));
        } else {
            out[e] = from_slot(x);
        }
    };
    const uint32_t hB = pl.hB;
    const bool walk_full = pl.walk_full;                     // full windows need cycle walking
    const uint32_t w_last = pl.w_last;                       // last pool2 window (may be short)
    const uint32_t len_last = pl.len_last, h_last = pl.h_last;
    const uint32_t wl = w_lo;
    const uint32_t t0 = tlo;
    const uint32_t sh = 32u - (uint32_t)ceil_log2_u64((uint64_t)P1);   // POW2 only
#ifdef PSS_STAMPS
    const uint64_t st_clk = __builtin_amdgcn_s_memtime(), st_rt = __builtin_amdgcn_s_memrealtime();
    if (lane == 0 && blockIdx.x < (1u << 16)) pss_stamps[blockIdx.x][3] = st_rt;
#endif
    // pool2 position (w0, p0) of the super-batch's first step, advanced without division
    uint32_t w0 = w_lo;
    uint32_t p0 = tlo - (w0 - 1) * B;
    // fast super-batches: every step valid and emitted, B >= 256 (at most one window boundary
    // per super-batch), neither window short nor cycle-walking
    const bool fast_tile = e_lo == 0 && e_hi == nvalid && B >= 256 && !walk_full;
    Pacer pace(nvalid);
    uint32_t tl0 = 0;
    if (fast_tile && (B & 255u) == 0 && w_last > w_lo + 1 && feistel_packed_ok(hB) && hB <= 8) {
        // (hB <= 8: the keyed-carry form below joins the halves inside 16-bit lanes)
        // Fast phase: whole super-batches of windows w_lo .. w_last - 2 (full, no cycle walk),
        // as one counted loop per window with the window's round keys in SGPRs.  B % 256 == 0
        // and tlo % 256 == 0 put every super-batch inside one window.
        const uint32_t avail = (w_last - 1 - w_lo) * B - p0;     // steps before window w_last-1
        uint32_t left = (avail < nvalid ? avail : nvalid) >> 8;  // super-batches
        if constexpr ((NARROW || PAIR) && POW2) {
            // Keyed-carry form of the packed Feistel (feistel4_pk16's values): with
            // A_i = R_i ^ K_i, A_{i+1} = A_{i-1} ^ F(A_i) ^ (K_{i-1} ^ K_{i+1}), one 3-input xor
            // per round; the output is L = A_5 ^ K_5, R = A_4 ^ F(A_5) ^ K_4.  p0 is a multiple
            // of 256 >= 2^hB, so R_0 = (64 j + lane) & mask is loop-invariant, L_0 = (p0 >> hB)
            // | ((64 j + lane) >> hB) has disjoint halves, and A_0, F(A_0) are per-window
            // constants: A_1 = C ^ (p0 >> hB) costs one xor.  The paired slot hashes take
            // (pb | 64 q | lane) ^ s0 with pb = (t0 + tl0) / 2, again one xor of a constant.
            const uint32_t h = hB, mask = (1u << h) - 1u;
            const uint32_t j1 = 64u + lane, j2 = 128u + lane, j3 = 192u + lane;
            const uint32_t Li0 = ((uint32_t)lane >> h) | ((j1 >> h) << 16);
            const uint32_t Li1 = (j2 >> h) | ((j3 >> h) << 16);
            const uint32_t Ri0 = ((uint32_t)lane & mask) | ((j1 & mask) << 16);
            const uint32_t Ri1 = (j2 & mask) | ((j3 & mask) << 16);
            const uint32_t hx0 = (uint32_t)lane ^ sk.s0, hx2 = (64u | (uint32_t)lane) ^ sk.s0;
            const pss_u16x2 M = {(unsigned short)kFeistelM16, (unsigned short)kFeistelM16};
            const pss_u16x2 SH = {(unsigned short)(16u - h), (unsigned short)(16u - h)};
            const pss_u16x2 HS = {(unsigned short)h, (unsigned short)h};
            auto F = [&](uint32_t a) -> uint32_t {
                return __builtin_bit_cast(uint32_t, (__builtin_bit_cast(pss_u16x2, a) * M) >> SH);
            };
            auto hash2 = [&](uint32_t x) -> uint32_t {   // slot_hash after the s0 xor
                x ^= x >> 16;
                x = (x & 0xFFFFFFu) * 0xA2F0ADu;
                x ^= x >> 15;
                x ^= sk.s1;
                x = (x & 0xFFFFFFu) * 0x5A2D97u;
                x ^= x >> 15;
                return x;
            };
            while (left) {
                const uint32_t room = (B - p0) >> 8;
                // wave-uniform trip count (readfirstlane: a scalar loop, not an exec-masked one)
                const uint32_t n = __builtin_amdgcn_readfirstlane(left < room ? left : room);
                uint32_t kw[kFeistelRounds];
#pragma unroll
                for (int i = 0; i < kFeistelRounds; i++)
                    kw[i] = (__builtin_amdgcn_readfirstlane(rk[kRoundKeyWords * (w0 - wl) + i]) & 0xFFFFu) * 0x10001u;
                const uint32_t K02 = kw[0] ^ kw[2], K13 = kw[1] ^ kw[3];
                const uint32_t K24 = kw[2] ^ kw[4], K35 = kw[3] ^ kw[5];
                const uint32_t KY = kw[4] ^ ((((kw[5] & 0xFFFFu) << h) & 0xFFFFu) * 0x10001u);
                const uint32_t A00 = Ri0 ^ kw[0], A01 = Ri1 ^ kw[0];
                const uint32_t C0 = Li0 ^ F(A00) ^ kw[1], C1 = Li1 ^ F(A01) ^ kw[1];
                // ids of the window's values wB + y: one add when the window maps contiguously
                // (PAIR: the window's pair constants in SGPRs, y -> y + Q_k on segment k)
                const uint32_t wB = w0 * B;
                uint32_t id_first = 0, PQ0 = 0, PQ1 = 0, PQ2 = 0, Ps1 = 0, Ps2 = 0;
                bool contiguous;
                if constexpr (PAIR) {
                    const uint32_t *c = pw + kPairWords * (w0 - wc_lo);
                    PQ0 = __builtin_amdgcn_readfirstlane(c[0]);
                    PQ1 = __builtin_amdgcn_readfirstlane(c[1]);
                    PQ2 = __builtin_amdgcn_readfirstlane(c[2]);
                    Ps1 = __builtin_amdgcn_readfirstlane(c[3]);
                    Ps2 = __builtin_amdgcn_readfirstlane(c[4]);
                    contiguous = PQ0 != kNone;
                } else {
                    id_first = to_slot(wB);
                    const uint32_t id_last = to_slot(wB + B - 1);
                    contiguous = __builtin_amdgcn_readfirstlane(
                        id_last - id_first == B - 1 && ((wB < twoB) == (wB + B - 1 < twoB)));
                }
                pace.step(tl0);
                // one 256-step super-batch at (tlx, px): its 4 slots and 4 inserted values
                auto batch = [&](auto contig, uint32_t tlx, uint32_t px, uint32_t (&k)[4], uint32_t (&ins)[4]) {
                    const uint32_t pb = (t0 + tlx) >> 1;
                    const uint32_t u0 = hash2(hx0 ^ pb), u2 = hash2(hx2 ^ pb);
                    k[0] = u0 >> sh; k[1] = (u0 << 16) >> sh; k[2] = u2 >> sh; k[3] = (u2 << 16) >> sh;
                    const uint32_t s = (px >> h) * 0x10001u;
                    const uint32_t A10 = C0 ^ s, A11 = C1 ^ s;
                    const uint32_t F10 = F(A10), F11 = F(A11);
                    const uint32_t A20 = A00 ^ F10 ^ K02, A21 = A01 ^ F11 ^ K02;
                    const uint32_t F20 = F(A20), F21 = F(A21);
                    const uint32_t A30 = A10 ^ F20 ^ K13, A31 = A11 ^ F21 ^ K13;
                    const uint32_t F30 = F(A30), F31 = F(A31);
                    const uint32_t A40 = A20 ^ F30 ^ K24, A41 = A21 ^ F31 ^ K24;
                    const uint32_t F40 = F(A40), F41 = F(A41);
                    const uint32_t A50 = A30 ^ F40 ^ K35, A51 = A31 ^ F41 ^ K35;
                    const uint32_t F50 = F(A50), F51 = F(A51);
                    const uint32_t S0 = __builtin_bit_cast(uint32_t, __builtin_bit_cast(pss_u16x2, A50) << HS);
                    const uint32_t S1 = __builtin_bit_cast(uint32_t, __builtin_bit_cast(pss_u16x2, A51) << HS);
                    const uint32_t Y0 = S0 ^ (A40 ^ F50 ^ KY), Y1 = S1 ^ (A41 ^ F51 ^ KY);
                    const uint32_t y[4] = {Y0 & 0xFFFFu, Y0 >> 16, Y1 & 0xFFFFu, Y1 >> 16};
                    // contig: 0 = the window's values through to_slot (PAIR: escaped), else one
                    // add -- PAIR: on 1, 2 or 3 file segments (the window's boundaries)
                    constexpr int M = decltype(contig)::value;
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        if constexpr (PAIR) {
                            if constexpr (M == 0) ins[j] = kPairEsc | (wB + y[j]);
                            else if constexpr (M == 1) ins[j] = y[j] + PQ0;
                            else if constexpr (M == 2) ins[j] = y[j] + (y[j] < Ps1 ? PQ0 : PQ1);
                            else ins[j] = pair_of_y(y[j], PQ0, PQ1, PQ2, Ps1, Ps2);
                        } else {
                            ins[j] = M ? id_first + y[j] : to_slot(wB + y[j]);
                        }
                    }
                };
                auto emit4 = [&](uint32_t tlx, const uint32_t (&v)[4]) {
                    if constexpr (PAIR) {
                        // branch-free unless some lane holds an escaped value (one wave-uniform
                        // test per super-batch, not an exec-masked branch per value)
                        const uint32_t any = (v[0] | v[1] | v[2] | v[3]) & kPairEsc;
                        if (__builtin_amdgcn_ballot_w64(any != 0u) == 0u) {
#ifdef PSS_DIAG_PAIR_INTERLEAVED   // (timing-only build: one 8-byte (file, offset) store per pair into fpos)
                            if (true) {
#pragma unroll
                                for (int j = 0; j < 4; j++) {
                                    const int64_t e = ebase + tlx + 64u * j + lane;
                                    ((int2 *)ma.fpos)[e] = make_int2((int)(v[j] >> pob), (int)(v[j] & omask));
                                }
#else
                            if (false) {
#endif
                            } else {
#pragma unroll
                                for (int j = 0; j < 4; j++) {
                                    const int64_t e = ebase + tlx + 64u * j + lane;
                                    ma.fpos[e] = (int32_t)(v[j] >> pob);
                                    ma.off[e] = (int32_t)(v[j] & omask);
                                }
                            }
                        } else {
#pragma unroll
                            for (int j = 0; j < 4; j++) emit_m(ebase + tlx + 64u * j + lane, v[j]);
                        }
                    } else if constexpr (MAPPED) {
#pragma unroll
                        for (int j = 0; j < 4; j++) emit_m(ebase + tlx + 64u * j + lane, v[j]);
                    } else {
                        int64_t *ob = o + tlx;
#pragma unroll
                        for (int j = 0; j < 4; j++) ob[64u * j + lane] = (int64_t)v[j];
                    }
                };
                auto run = [&](auto contig) {
                    uint32_t i = 0;
                    for (; i < n; i++) {
                        uint32_t k[4], ins[4], v[4];
                        batch(contig, tl0, p0, k, ins);
#pragma unroll
                        for (int j = 0; j < 4; j++) v[j] = atomicExch(&buf[k[j]], ins[j]);
                        emit4(tl0, v);
                        tl0 += 256;
                        p0 += 256;
                    }
                };
                if constexpr (PAIR) {
                    if (!contiguous) run(std::integral_constant<int, 0>{});
                    else if (Ps1 == kNone) run(std::integral_constant<int, 1>{});
                    else if (Ps2 == kNone) run(std::integral_constant<int, 2>{});
                    else run(std::integral_constant<int, 3>{});
                } else {
                    if (contiguous) run(std::integral_constant<int, 1>{});
                    else run(std::integral_constant<int, 0>{});
                }
                left -= n;
                if (p0 == B) { p0 = 0; w0++; }
            }
        } else {
            while (left) {
                const uint32_t room = (B - p0) >> 8;
                const uint32_t n = left < room ? left : room;
                uint32_t kw[kFeistelRounds];   // window w0's round keys, packed twice into 16 bits
#pragma unroll
                for (int i = 0; i < kFeistelRounds; i++)
                    kw[i] = (__builtin_amdgcn_readfirstlane(rk[kRoundKeyWords * (w0 - wl) + i]) & 0xFFFFu) * 0x10001u;
                const uint32_t wB = w0 * B;
                uint32_t PQ[5] = {kNone, 0u, 0u, kNone, kNone};   // PAIR: the window's constants
                if constexpr (PAIR) {
#pragma unroll
                    for (int i = 0; i < 5; i++) PQ[i] = __builtin_amdgcn_readfirstlane(pw[kPairWords * (w0 - wc_lo) + i]);
                }
                pace.step(tl0);
                for (uint32_t i = 0; i < n; i++) {
                    uint32_t k[4], ins[4], v[4];
                    slot4<POW2>(t0 + tl0 + lane, sk, P1, sh, k);
                    const uint32_t x[4] = {p0 + lane, p0 + 64u + lane, p0 + 128u + lane, p0 + 192u + lane};
                    feistel4_pk16(x, hB, kw, ins);
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        uint32_t sv;
                        if constexpr (PAIR)
                            sv = PQ[0] != kNone ? pair_of_y(ins[j], PQ[0], PQ[1], PQ[2], PQ[3], PQ[4]) : kPairEsc | (wB + ins[j]);
                        else
                            sv = to_slot(wB + ins[j]);
                        v[j] = atomicExch(&buf[k[j]], sv);
                    }
                    // wave-uniform base: the stores take (lane * 8 + 512 j) as offset
                    if constexpr (MAPPED) {
#pragma unroll
                        for (int j = 0; j < 4; j++) emit_m(ebase + tl0 + 64u * j + lane, v[j]);
                    } else {
                        int64_t *ob = o + tl0;
#pragma unroll
                        for (int j = 0; j < 4; j++) ob[64u * j + lane] = from_slot(v[j]);
                    }
                    tl0 += 256;
                    p0 += 256;
                }
                left -= n;
                if (p0 == B) { p0 = 0; w0++; }
            }
        }
    }
    for (; tl0 < nvalid; tl0 += 256) {
        pace.step(tl0);
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const uint32_t tl = tl0 + 64u * j + lane;
            if (tl < nvalid) {
                const uint32_t kk = slot_draw(t0 + tl, sk.s0, sk.s1, P1);
                uint32_t p = p0 + 64u * j + lane, w = w0;
                while (p >= B) { p -= B; w++; }
                const bool lastw = w == w_last;
                const uint32_t in = w * B + feistel(p, lastw ? len_last : B, lastw ? h_last : hB,
                                                    rk + kRoundKeyWords * (w - wl));
                const uint32_t vv = atomicExch(&buf[kk], to_slot(in));
                if (tl >= e_lo && tl < e_hi) {
                    if constexpr (MAPPED) emit_m(ebase + tl, vv);
                    else o[tl] = from_slot(vv);
                }
            }
        }
        p0 += 256;
        while (p0 >= B) { p0 -= B; w0++; }
    }
#ifdef PSS_STAMPS
    if (lane == 0 && blockIdx.x < (1u << 16)) {
        pss_stamps[blockIdx.x][0] = __builtin_amdgcn_s_memtime() - st_clk;
        pss_stamps[blockIdx.x][1] = __builtin_amdgcn_s_memrealtime() - st_rt;
        pss_stamps[blockIdx.x][4] = __builtin_amdgcn_s_memrealtime();
        pss_stamps[blockIdx.x][6] = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));   // HW_ID
        pss_stamps[blockIdx.x][7] = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (15 << 11));  // XCC_ID
    }
#endif
    if (do_tail && (int64_t)tile == pl.G - 1) {
        // the rank's final pool is this wave's slot table: drain it in tail order (positions
        // T + j, j < P1).  One wave: its own LDS exchanges above are complete in order.  The
        // last tile is short, so its wave reaches this point while its SIMD partner still runs
        // at a higher Pacer priority: take the top priority, the tail is on the critical path.
        __builtin_amdgcn_s_setprio(3);
        __syncthreads();
        uint32_t tk[kRoundKeyWords];
        tail_round_keys(g, rank, tk);
        const uint32_t hT = feistel_half_bits(P1);
        int64_t *ot = out + (int64_t)rl * count - pos_lo + pl.T;
        const int64_t etail = (int64_t)rl * count - pos_lo + pl.T;
        const bool whole = pl.T >= pos_lo && pl.T + pl.P1 <= pos_hi;
        if (whole && (P1 & 255u) == 0 && feistel_packed_ok(hT) && P1 == (1u << (2 * hT))) {
            // P1 = 4^hT: no cycle walking; four independent chains per lane, packed in pairs
            uint32_t kp[kFeistelRounds];
#pragma unroll
            for (int i = 0; i < kFeistelRounds; i++) kp[i] = (tk[i] & 0xFFFFu) * 0x10001u;
            for (uint32_t j0 = 0; j0 < P1; j0 += 256) {
                uint32_t y[4];
                feistel2_pk16(j0 + lane, j0 + 64u + lane, hT, kp, y[0], y[1]);
                feistel2_pk16(j0 + 128u + lane, j0 + 192u + lane, hT, kp, y[2], y[3]);
                uint32_t v[4];
#pragma unroll
                for (int u = 0; u < 4; u++) v[u] = buf[y[u]];
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    if constexpr (MAPPED) emit_m(etail + j0 + 64u * u + lane, v[u]);
                    else ot[j0 + 64u * u + lane] = from_slot(v[u]);
                }
            }
        } else {
            for (uint32_t j = lane; j < P1; j += 64) {
                const int64_t pos = pl.T + j;
                if (pos < pos_lo || pos >= pos_hi) continue;
                if constexpr (MAPPED) emit_m(etail + j, buf[feistel(j, P1, hT, tk)]);
                else ot[j] = from_slot(buf[feistel(j, P1, hT, tk)]);
            }
        }
    }
#ifdef PSS_STAMPS
    if (lane == 0 && blockIdx.x < (1u << 16)) pss_stamps[blockIdx.x][5] = __builtin_amdgcn_s_memrealtime();
#endif
}

// Start-up check of the exchange order k_v2_emit_x relies on: random slot patterns (heavy
// collisions at 64 slots in blocks 0..63, sparse at 4096 in blocks 64..127) against the
// sequential lane-order model.  Once per device per process, on the first V2 replay.
__global__ __launch_bounds__(64) void k_xchg_order_check(int iters, uint32_t *bad) {
    const uint32_t P = blockIdx.x < 64 ? 64u : 4096u;
    bad += blockIdx.x < 64 ? 0 : 1;
    // two exchanges and two plain stores per iteration, back to back (no wait in between), as
    // the replay kernels issue them; the model replays them in (instruction, lane) order
    __shared__ uint32_t buf[4096];
    __shared__ uint32_t model[4096];
    __shared__ uint32_t wbuf[4096];
    __shared__ uint32_t cnt[4096];
    __shared__ uint32_t mcnt[4096];
    const int lane = threadIdx.x;
    for (uint32_t s = lane; s < P; s += 64) {
        buf[s] = 0xF0000000u | s; model[s] = buf[s]; wbuf[s] = buf[s]; cnt[s] = 0; mcnt[s] = 0;
    }
    __syncthreads();
    uint32_t nbad = 0, nbadw = 0, nbada = 0;
    for (int it = 0; it < iters; it++) {
        uint32_t ks[2], ins[2], got[2];
#pragma unroll
        for (int q = 0; q < 2; q++) {
            ks[q] = scale32(slot_hash((uint32_t)((blockIdx.x * iters + it) * 2 + q) * 64u + lane, 0x9E3779B9u, 0x7F4A7C15u), P);
            ins[q] = ((uint32_t)it << 9) ^ ((uint32_t)q << 8) ^ (uint32_t)lane;
        }
        uint32_t pos[2];
#pragma unroll
        for (int q = 0; q < 2; q++) got[q] = atomicExch(&buf[ks[q]], ins[q]);
#pragma unroll
        for (int q = 0; q < 2; q++) wbuf[ks[q]] = ins[q];
#pragma unroll
        for (int q = 0; q < 2; q++) pos[q] = atomicAdd(&cnt[ks[q]], 1u);
        __syncthreads();
        uint32_t expect[2] = {0, 0}, expc[2] = {0, 0};
        for (int q = 0; q < 2; q++) {
            for (int l = 0; l < 64; l++) {      // lane 0 replays the exchanges / adds in lane order
                const uint32_t kl = (uint32_t)__shfl((int)ks[q], l);
                const uint32_t il = (uint32_t)__shfl((int)ins[q], l);
                uint32_t old = 0, oc = 0;
                if (lane == 0) { old = model[kl]; model[kl] = il; oc = mcnt[kl]; mcnt[kl] = oc + 1; }
                old = (uint32_t)__shfl((int)old, 0);
                oc = (uint32_t)__shfl((int)oc, 0);
                if (lane == l) { expect[q] = old; expc[q] = oc; }
            }
        }
        __syncthreads();
        nbad += (got[0] != expect[0]) + (got[1] != expect[1]);
        nbada += (pos[0] != expc[0]) + (pos[1] != expc[1]);
    }
    for (uint32_t s = lane; s < P; s += 64) {
        nbad += buf[s] != model[s];
        nbadw += wbuf[s] != model[s];
    }
    for (uint32_t s = lane; s < P; s += 64) nbada += cnt[s] != mcnt[s];
    if (nbad) atomicAdd(bad, nbad);
    if (nbadw) atomicAdd(bad + 2, nbadw);
    if (nbada) atomicAdd(bad + 4, nbada);
}

// ---- tail ---------------------------------------------------------------------------------
// position T + j of a rank emits the final pool1 slot pi(j), pi = Feistel bijection of [0, P1)
// keyed by tail_round_keys; the final content of a slot is the VAL walk-back from the last tile
__global__ __launch_bounds__(256) void k_v2_tail_f(Geometry g, V2Plan pl,
                                                  const RankDesc *__restrict__ ranks,
                                                  int32_t rank_lo, const uint32_t *__restrict__ VAL,
                                                  int64_t pos_lo, int64_t count,
                                                  int64_t *__restrict__ out, MapArgs ma,
                                                  RankArgs ra, int use_ra) {
    const int32_t rl = (int32_t)blockIdx.y;
    const uint32_t rank = (uint32_t)(rank_lo + rl);
    // ranks by value (the whole-stream calls that touch no shared device table) or the table
    const RankDesc rd = use_ra ? ra.r[rl] : ranks[rank];
    const uint32_t P1 = (uint32_t)pl.P1;
    uint32_t tk[kRoundKeyWords];
    tail_round_keys(g, rank, tk);
    const uint32_t hT = feistel_half_bits(P1);
    const uint32_t *VALr = VAL + (int64_t)rl * pl.G * pl.P1;
    int64_t *o = out + (int64_t)rl * count - pos_lo;
    const int64_t pos_hi = pos_lo + count;
    for (uint32_t j = blockIdx.x * 256u + threadIdx.x; j < P1; j += gridDim.x * 256u) {
        const int64_t pos = pl.T + j;
        if (pos < pos_lo || pos >= pos_hi) continue;
        const uint32_t s = feistel(j, P1, hT, tk);
        const int64_t id = v2_id(slot_value_after(VALr, pl.P1, pl.G - 1, s), rd, g);
        if (ma.fpos) {      // mapped output: the global bucketed map (P1 ids per rank)
            int32_t f, of;
            map_id_fast(ma, id, f, of);
            const int64_t e = (int64_t)rl * count - pos_lo + pos;
            ma.fpos[e] = f;
            ma.off[e] = of;
        } else {
            o[pos] = id;
        }
    }
}

// ------------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------------
static int device_cus() {
    static int cache[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
    if (!cache[dev]) {
        int n = 0;
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
            n = 256;
        cache[dev] = n;
    }
    return cache[dev];
}

constexpr int64_t kCuLdsBytes = 160 * 1024;
constexpr int64_t kMaxTileMult = 16;   // tile length <= 16 * P1 steps (Feistel key table bound)
constexpr int64_t kMinTileMult = 4;    // >= 4 * P1: VAL traffic <= 2 B/step, walk-back <= e^-4

V2Plan v2_plan(const Geometry &g, int32_t nr) {
    V2Plan p{};
    p.P1 = g.B < g.ns ? g.B : g.ns;
    p.T = g.ns - p.P1;
    p.fold = g.ns <= (int64_t)1 << 24;
    // emit wave LDS: Feistel keys of up to kMaxTileMult + 2 windows, the slot table, the probe
    const int64_t keys = (int64_t)kRoundKeyWords * 4 * (kMaxTileMult + 2);
    const int64_t lds = keys + p.P1 * 4 + (p.fold ? 0 : kMarkBytes);
    // waves per CU the LDS admits, rounded down to whole SIMD quads (balanced SIMDs), <= 16
    int64_t wpc = kCuLdsBytes / lds;
    wpc = wpc > 16 ? 16 : wpc;
    if (wpc >= 4) wpc &= ~3;
    // No LDS padding: k_v2_emit_x claims VGPRs for two waves per SIMD (PSS_TWO_WAVES_PER_SIMD),
    // which caps a CU at eight replay waves, and the LDS left over (25 KB at P1 = 4096) takes a
    // last-occurrence workgroup of the next epoch's lookahead beside them (round 2: C2 487-496
    // -> 511-516 G idx/s against round 1's LDS padding, same box).
    p.emit_lds = lds;
    // one round of waves: tiles = waves per CU x CUs spread over the nr streams
    const int64_t waves = wpc * device_cus();
    const int64_t per_rank = cdiv(waves, nr > 0 ? nr : 1);
    int64_t L = p.T > 0 ? cdiv(p.T, per_rank) : p.P1;
    const int64_t lo = kMinTileMult * p.P1, hi = kMaxTileMult * p.P1;
    L = L < lo ? lo : (L > hi ? hi : L);
    p.L = cdiv(L, 256) * 256;
    p.G = p.T > 0 ? cdiv(p.T, p.L) : 0;
    p.B32 = (uint32_t)g.B;
    p.L32 = (uint32_t)p.L;
    p.T32 = (uint32_t)p.T;
    p.hB = feistel_half_bits(p.B32);
    p.walk_full = p.B32 != (1u << (2 * p.hB));
    p.w_last = p.T > 0 ? (uint32_t)(1 + (p.T - 1) / g.B) : 0;
    p.len_last = p.T > 0 ? (uint32_t)(g.ns - (int64_t)p.w_last * g.B) : 0;
    p.h_last = feistel_half_bits(p.len_last > 0 ? p.len_last : 1);
    p.twoB = (uint32_t)(2 * g.B < g.ns ? 2 * g.B : g.ns);
    return p;
}

size_t v2_val_bytes(const Geometry &g, int32_t nr) {
    if (v2_grouped(g)) return v2_grp_val_bytes(g, nr);
    const V2Plan p = v2_plan(g, nr);
    return (size_t)nr * (size_t)p.G * (size_t)p.P1 * sizeof(uint32_t);
}

size_t v2_buf_bytes(const Geometry &, int32_t) {
    return 0;   // no HBM slot tables: small pools replay in LDS, big ones in LDS groups
}

// pss_generate_mapped fuses the map into the V2 replay for pools that fit LDS, on the exchange
// path: a tile's ids then span ~(L / B + kSegBackWin) windows, a few hundred files at most.  A
// grouped replay wave covers its rank's whole stream (too many files to stage): generate + map.
bool v2_mapped_fused(const Geometry &g, int emit_path) {
    // the exchange replays map in-kernel: the small-pool one through its per-tile LDS segment
    // map, the grouped one through the global bucketed map
    (void)g;
    if (emit_path == EMIT_AUTO) emit_path = lds_xchg_ordered() ? EMIT_XCHG : EMIT_PROBE;
    return emit_path == EMIT_XCHG;
}

size_t v2_sort_bytes(const Geometry &, int32_t) {
    return 0;   // the tail order is a Feistel bijection: no sort workspace
}

hipError_t launch_v2_tail_vals(const Geometry &g, const V2Plan &pl, const RankDesc *ranks,
                               int32_t rank_lo, int32_t nr, const uint32_t *VAL, int64_t pos_lo,
                               int64_t count, int64_t *out, hipStream_t s, const MapArgs *mapped,
                               const RankArgs *rank_args) {
    const dim3 grid((uint32_t)cdiv(pl.P1 < 65536 ? pl.P1 : 65536, 256), (uint32_t)nr);
    const MapArgs ma = mapped ? *mapped : MapArgs{};
    RankArgs ra;
    if (rank_args) ra = *rank_args;
    hipLaunchKernelGGL(k_v2_tail_f, grid, dim3(256), 0, s, g, pl, ranks, rank_lo, VAL, pos_lo,
                       count, out, ma, ra, rank_args ? 1 : 0);
    return hipGetLastError();
}

bool v2_ranks_by_value(const Geometry &g, int32_t nr, int emit_path) {
    if (emit_path == EMIT_AUTO) emit_path = lds_xchg_ordered() ? EMIT_XCHG : EMIT_PROBE;
    return emit_path == EMIT_XCHG && nr >= 1 && nr <= kArgRanks;   // k_v2_emit_x, k_g_emit
}

bool v2_stage_split(const Geometry &g, int32_t nr, int emit_path) {
    if (emit_path == EMIT_AUTO) emit_path = lds_xchg_ordered() ? EMIT_XCHG : EMIT_PROBE;
    // grouped pools always split: their pre-pass (key table, last occurrences of tiled
    // streams) runs a step ahead on the side stream; in line the C5 step was 0.264 ms against
    // 0.233 ms split (round 2, profiles/r02/c5_split_ab.txt)
    if (v2_grouped(g)) return true;
    return emit_path == EMIT_XCHG;
}

hipError_t launch_v2(const Geometry &g, const RankDesc *ranks, int32_t rank_lo, int32_t nr,
                     int64_t pos_lo, int64_t count, int64_t *out, uint32_t *VAL, uint32_t *gbuf,
                     uint32_t *sort_ws, int32_t *err, hipStream_t s, const Marker &mk,
                     int emit_path, int stage, const MapArgs *mapped, const RankArgs *rank_args) {
    if (emit_path == EMIT_AUTO) emit_path = lds_xchg_ordered() ? EMIT_XCHG : EMIT_PROBE;
    if (mapped && !v2_mapped_fused(g, emit_path)) return hipErrorNotSupported;
    if (rank_args && !v2_ranks_by_value(g, nr, emit_path)) return hipErrorInvalidValue;
    // stage: V2_STAGE_ALL, or the split the runtime pipelines over two streams --
    // V2_STAGE_PRE (key table + last-occurrence pass, writes VAL) then V2_STAGE_EMIT (replay +
    // tail, reads VAL).  Only the LDS exchange path splits; everything else runs whole in the
    // PRE call and the EMIT call is a no-op.
    if (!v2_stage_split(g, nr, emit_path)) {
        if (stage == V2_STAGE_EMIT) return hipSuccess;
        stage = V2_STAGE_ALL;
    }
    const bool do_pre = stage != V2_STAGE_EMIT, do_emit = stage != V2_STAGE_PRE;
    if (v2_grouped(g))   // pools beyond LDS: the grouped slot machine (pss_v2grp.hip)
        return launch_v2_grp(g, ranks, rank_lo, nr, pos_lo, count, out, VAL, s, mk,
                             emit_path == EMIT_XCHG, stage, rank_args, mapped);
    (void)err; (void)sort_ws; (void)gbuf;
    const V2Plan pl = v2_plan(g, nr);
    const int64_t pos_hi = pos_lo + count < g.ns ? pos_lo + count : g.ns;
    if (nr <= 0 || pos_hi <= pos_lo) return hipSuccess;
    const int64_t nwin_max = pl.L / g.B + 2;
    const size_t lds_keys = (size_t)kRoundKeyWords * nwin_max * sizeof(uint32_t);
    const bool need_tail = pos_hi > pl.T;
    bool tail_fused = false;   // drained by the last tile's k_v2_emit_x wave
    if (pl.G > 0) {
        // pass A over every tile up to the last one emitted (the tail needs all of them);
        // VAL is indexed (rl*G + tile), tile < g_need
        const int64_t last_emit = pos_lo < pl.T ? ((pos_hi < pl.T ? pos_hi : pl.T) - 1) / pl.L : -1;
        const int64_t g_need = need_tail ? pl.G : last_emit + 1;
        if (g_need > 0 && do_pre) {
            mk(K_V2_LASTOCC, s);
            // 256 threads per workgroup: 512 shortens this pass (0.066 -> 0.060 ms) but the
            // replay beside it slows by as much (power-limited, same-box A/B in rounds 2 and 4);
            // a one-wave pass with ordered plain stores instead of ds_max was 15 % slower
            const size_t lds = (size_t)pl.P1 * 4 + lds_keys;
            const bool pow2 = pl.P1 >= 2 && slot_paired((uint32_t)pl.P1);   // paired draws
            const dim3 grid((uint32_t)(nr * g_need));
            if (pow2) hipLaunchKernelGGL((k_v2_lastocc<256, true>), grid, dim3(256), lds, s, g, pl, rank_lo, g_need, VAL);
            else hipLaunchKernelGGL((k_v2_lastocc<256, false>), grid, dim3(256), lds, s, g, pl, rank_lo, g_need, VAL);
        }
        if (do_pre && !do_emit) mk(-1, s);
        if (last_emit >= 0 && do_emit) {
            const int64_t g_lo = pos_lo / pl.L;
            const int64_t ng = last_emit - g_lo + 1;
            // 32-bit id arithmetic whenever every id (and id + ns before the wrap) fits
            const bool narrow = g.N + g.ns < (int64_t)UINT32_MAX;
            const dim3 grid((uint32_t)(nr * ng));
            if (emit_path == EMIT_XCHG) {
                mk(K_V2_EMIT, s);
                // mapped: pair slots (MapArgs::pack) with their window constants, else the
                // segment map, after the keys
                const bool pair = mapped && mapped->pack;
                const size_t need = lds_keys + (size_t)((pl.P1 + 3) & ~3) * 4 +
                                    (pair ? (size_t)kPairWords * (size_t)(nwin_max + kPairBack) * 4
                                          : mapped ? (size_t)kSegLdsWords * 4 : 0);
                const size_t lds = need > (size_t)pl.emit_lds ? need : (size_t)pl.emit_lds;
                tail_fused = need_tail && last_emit == pl.G - 1;
                const int dt = tail_fused ? 1 : 0;
                const bool pow2 = pl.P1 >= 2 && slot_paired((uint32_t)pl.P1);   // paired draws
                const MapArgs ma = mapped ? *mapped : MapArgs{};
                RankArgs ra;
                const int use_ra = rank_args ? 1 : 0;
                if (rank_args) ra = *rank_args;
#define PSS_EX(N, P2) do { if (pair) hipLaunchKernelGGL((k_v2_emit_x<N, P2, true, true>), grid, dim3(64), lds, s, g, pl, ranks, rank_lo, \
                                         g_lo, ng, (const uint32_t *)VAL, pos_lo, count, dt, out, ma, ra, use_ra); \
                           else if (mapped) hipLaunchKernelGGL((k_v2_emit_x<N, P2, true>), grid, dim3(64), lds, s, g, pl, ranks, rank_lo, \
                                         g_lo, ng, (const uint32_t *)VAL, pos_lo, count, dt, out, ma, ra, use_ra); \
                           else hipLaunchKernelGGL((k_v2_emit_x<N, P2, false>), grid, dim3(64), lds, s, g, pl, ranks, rank_lo, \
                                         g_lo, ng, (const uint32_t *)VAL, pos_lo, count, dt, out, ma, ra, use_ra); } while (0)
                if (narrow && pow2) PSS_EX(true, true);
                else if (narrow) PSS_EX(true, false);
                else if (pow2) PSS_EX(false, true);
                else PSS_EX(false, false);
#undef PSS_EX
            } else {   // probe path (EMIT_PROBE)
                mk(K_V2_EMIT, s);
                const size_t need = lds_keys + (size_t)pl.P1 * 4 + (pl.fold ? 0 : kMarkBytes);
                const size_t lds = need > (size_t)pl.emit_lds ? need : (size_t)pl.emit_lds;
#define PSS_EMIT(N, F) hipLaunchKernelGGL((k_v2_emit<N, F>), grid, dim3(64), lds, s, g, pl, ranks, rank_lo, \
                                          g_lo, ng, (const uint32_t *)VAL, pos_lo, count, out)
                if (pl.fold && narrow) PSS_EMIT(true, true);
                else if (pl.fold) PSS_EMIT(false, true);
                else if (narrow) PSS_EMIT(true, false);
                else PSS_EMIT(false, false);
#undef PSS_EMIT
            }
        }
    }
    if (!do_emit) return hipGetLastError();
    if (need_tail && !tail_fused) {
        // ranks that came by value go to the tail kernel by value too: a whole-stream call
        // touches no shared device table (the runtime skips its cross-stream ordering for it)
        mk(K_V2_TAIL, s);
        hipError_t e = launch_v2_tail_vals(g, pl, ranks, rank_lo, nr, VAL, pos_lo, count, out, s, mapped,
                                           rank_args);
        if (e != hipSuccess) return e;
    }
    mk(-1, s);
    return hipGetLastError();
}

static signed char g_xchg_ordered[64];   // per device: 0 unknown, 1 ordered, -1 not
static signed char g_write_ordered[64];
static signed char g_add_ordered[64];

// The exchange replay (k_v2_emit_x, one lane-ordered exchange per step) against the
// collision-probe replay (k_v2_emit: probe bytes + ballots, no ordering assumption) on small real
// geometries -- a power-of-two pool (paired draws, the C2 kernel) and a multiply-shift one, 3 ranks,
// several tiles, a wrapping block, the tail.  Run once per device after the synthetic pattern
// check passes: the ordering is then confirmed on the kernel and the shapes it serves, and a
// difference anywhere sends every replay down the probe path.  same = every id equal.
static hipError_t xchg_replay_crosscheck(bool &same) {
    same = false;
    struct Shape { int64_t ns, B; };
    const Shape shapes[2] = {{6 * 4 * 4096 + 4096 + 777, 4096}, {5 * 4 * 3000 + 3000 + 321, 3000}};
    const int32_t R = 3;
    for (const Shape &sh : shapes) {
        Geometry g{};
        g.ns = sh.ns; g.R = R; g.N = sh.ns * R - 2; g.B = sh.B; g.version = 2; g.shuffle = 1;
        g.key0 = 0x9E3779B9u; g.key1 = 0x7F4A7C15u;
        RankDesc hr[R];
        for (int32_t r = 0; r < R; r++) hr[r] = {(int64_t)r * g.ns, (int64_t)((r + 2) % R) * g.ns};
        const size_t nval = v2_val_bytes(g, R), nbuf = v2_buf_bytes(g, R), nsort = v2_sort_bytes(g, R);
        const size_t nout = (size_t)R * (size_t)g.ns * sizeof(int64_t);
        char *mem = nullptr;
        const size_t total = sizeof(hr) + 16 + nval + nbuf + nsort + 2 * nout + 64;
        hipError_t e = hipMalloc((void **)&mem, total);
        if (e != hipSuccess) return e;
        auto at = [&](size_t off) { return mem + ((off + 15) & ~(size_t)15); };
        size_t off = 0;
        RankDesc *dr = (RankDesc *)at(off); off = (size_t)((char *)dr - mem) + sizeof(hr);
        int32_t *err = (int32_t *)at(off); off = (size_t)((char *)err - mem) + 16;
        uint32_t *val = (uint32_t *)at(off); off = (size_t)((char *)val - mem) + nval;
        uint32_t *buf = nbuf ? (uint32_t *)at(off) : nullptr; off = (size_t)((char *)at(off) - mem) + nbuf;
        uint32_t *srt = nsort ? (uint32_t *)at(off) : nullptr; off = (size_t)((char *)at(off) - mem) + nsort;
        int64_t *o1 = (int64_t *)at(off); off = (size_t)((char *)o1 - mem) + nout;
        int64_t *o2 = (int64_t *)at(off);
        std::vector<int64_t> h1((size_t)R * g.ns), h2((size_t)R * g.ns);
        e = hipMemcpy(dr, hr, sizeof(hr), hipMemcpyHostToDevice);
        if (e == hipSuccess) e = hipMemset(err, 0, 16);
        if (e == hipSuccess) e = launch_v2(g, dr, 0, R, 0, g.ns, o1, val, buf, srt, err, 0, Marker(), EMIT_XCHG, V2_STAGE_ALL);
        if (e == hipSuccess) e = launch_v2(g, dr, 0, R, 0, g.ns, o2, val, buf, srt, err, 0, Marker(), EMIT_PROBE, V2_STAGE_ALL);
        if (e == hipSuccess) e = hipMemcpy(h1.data(), o1, nout, hipMemcpyDeviceToHost);
        if (e == hipSuccess) e = hipMemcpy(h2.data(), o2, nout, hipMemcpyDeviceToHost);
        (void)hipFree(mem);
        if (e != hipSuccess) return e;
        if (h1 != h2) return hipSuccess;   // same stays false
    }
    same = true;
    return hipSuccess;
}

hipError_t check_lds_xchg_order() {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    if (dev < 0 || dev >= 64 || g_xchg_ordered[dev]) return hipSuccess;
    // bad[0..1]: exchange mismatches at 64 / 4096 slots; bad[2..3]: plain-store mismatches;
    // bad[4..5]: returning-add mismatches
    uint32_t *bad = nullptr, hbad[6] = {1, 1, 1, 1, 1, 1};
    e = hipMalloc((void **)&bad, sizeof(hbad));
    if (e != hipSuccess) return e;
    e = hipMemset(bad, 0, sizeof(hbad));
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_xchg_order_check, dim3(128), dim3(64), 0, 0, 24, bad);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpy(hbad, bad, sizeof(hbad), hipMemcpyDeviceToHost);
    (void)hipFree(bad);
    if (e != hipSuccess) return e;
    g_write_ordered[dev] = (hbad[2] == 0 && hbad[3] == 0) ? 1 : -1;
    g_add_ordered[dev] = (hbad[4] == 0 && hbad[5] == 0) ? 1 : -1;
    if (hbad[0] != 0 || hbad[1] != 0) {
        g_xchg_ordered[dev] = -1;
        return hipSuccess;
    }
    // the pattern check passed: confirm it on the replay kernels themselves (the cross-check
    // launches explicit paths, so it does not recurse into this function)
    bool same = false;
    e = xchg_replay_crosscheck(same);
    if (e != hipSuccess) return e;
    g_xchg_ordered[dev] = same ? 1 : -1;
    return hipSuccess;
}

bool lds_add_ordered() {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return false;
    if (!g_add_ordered[dev] && check_lds_xchg_order() != hipSuccess) return false;
    return g_add_ordered[dev] > 0;
}

bool lds_write_ordered() {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return false;
    if (!g_write_ordered[dev] && check_lds_xchg_order() != hipSuccess) return false;
    return g_write_ordered[dev] > 0;
}

bool lds_xchg_ordered() {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return false;
    if (!g_xchg_ordered[dev] && check_lds_xchg_order() != hipSuccess) return false;
    return g_xchg_ordered[dev] > 0;
}

hipError_t init_kernel_attributes_v2() {
    const int big = 160 * 1024;
    // the exchange-order check runs lazily, on the first query (lds_*_ordered): V1-only
    // handles never pay for it, V2 ones once per device per process
    hipError_t e = init_kernel_attributes_v2grp();
#define PSS_ATTR(fn) { hipError_t x = hipFuncSetAttribute((const void *)(fn), hipFuncAttributeMaxDynamicSharedMemorySize, big); if (x != hipSuccess) e = x; }
    PSS_ATTR((k_v2_lastocc<256, true>));
    PSS_ATTR((k_v2_lastocc<256, false>));
    PSS_ATTR((k_v2_emit_x<true, true, false>));
    PSS_ATTR((k_v2_emit_x<true, false, false>));
    PSS_ATTR((k_v2_emit_x<false, true, false>));
    PSS_ATTR((k_v2_emit_x<false, false, false>));
    PSS_ATTR((k_v2_emit_x<true, true, true>));
    PSS_ATTR((k_v2_emit_x<true, false, true>));
    PSS_ATTR((k_v2_emit_x<false, true, true>));
    PSS_ATTR((k_v2_emit_x<false, false, true>));
    PSS_ATTR((k_v2_emit_x<true, true, true, true>));
    PSS_ATTR((k_v2_emit_x<true, false, true, true>));
    PSS_ATTR((k_v2_emit_x<false, true, true, true>));
    PSS_ATTR((k_v2_emit_x<false, false, true, true>));
    PSS_ATTR((k_v2_emit<true, false>));
    PSS_ATTR((k_v2_emit<false, false>));
    PSS_ATTR((k_v2_emit<true, true>));
    PSS_ATTR((k_v2_emit<false, true>));
#undef PSS_ATTR
    return e;
}

}  // namespace pss
