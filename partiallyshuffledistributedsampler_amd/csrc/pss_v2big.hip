// pss_v2big.hip -- V2 with pools too large for one LDS slot table (P1 > 16384, e.g. B = 2^20,
// BASELINE configs[4]): the slot-replacement replay of pss_v2.hip, split by SLOT instead of by
// time.
//
// Slots are cut into chunks of 4096 (16 KB of LDS).  A step touches exactly one slot, so the
// steps that draw chunk c form an independent sub-stream: replaying it in step order with a
// 4096-entry table gives exactly the values the full replay gives for those steps.  Per time
// tile (L = mult * P1 steps) and rank:
//
//   k_bk_count     one wave per segment of 4096 steps: histogram of the chunk of every step
//   k_bk_scan_*    per tile: exclusive scan of the (chunk, segment) counts, chunk-major
//   k_bk_scatter   per segment: each step's tile-local index into its chunk's list, in step
//                  order (lane-ordered ds_add_rtn, checked at start-up: stable)
//   k_bk_lastocc   per (tile, chunk): last step of each slot (plain stores in list order) ->
//                  VAL[tile][slot] = inserted value or NONE
//   k_bk_emit      per (tile, chunk): slot table from VAL[tile-1] (+ walk-back), replay of the
//                  chunk's list with one lane-ordered LDS exchange per step, ids written at
//                  their stream positions (scattered 8 B stores inside the tile's output)
//   k_v2_tail_f    (pss_v2.hip) the final pool from the VAL walk-back
//
// Same schedule as the LDS path: the output is bit-identical.
#include <cstdio>
#include <cstdlib>

#include "pss_device.h"

namespace pss {

namespace {

constexpr uint32_t kChunkBits = 12;
constexpr uint32_t kChunk = 1u << kChunkBits;     // slots per chunk (LDS table)
constexpr uint32_t kSeg = 4096;                   // steps per bucketing wave
constexpr int64_t kBigMaxP1 = (int64_t)1 << 22;   // <= 1024 chunks; counts <= 16 MB per tile

inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

struct BigPlan {
    int64_t P1, T, L, G, C, nseg;   // nseg = segments per (full) tile
};

BigPlan big_plan(const Geometry &g, int32_t nr) {
    BigPlan p{};
    p.P1 = g.B < g.ns ? g.B : g.ns;
    p.T = g.ns - p.P1;
    p.C = cdiv(p.P1, kChunk);
    // tiles of mult * P1 steps: long enough that a slot is rarely untouched by a whole tile
    // (walk-back e^-mult), short enough that nr * G * C jobs fill the chip
    static const int64_t mult_env = [] {   // tuning knob
        const char *e = getenv("PSS_V2BIG_MULT");
        const long v = e ? atol(e) : 0;
        return (int64_t)(v >= 1 && v <= 4 ? v : 0);
    }();
    int64_t mult = mult_env ? mult_env : 4;
    for (;;) {
        if (mult_env) break;
        const int64_t L = cdiv(mult * p.P1, kSeg) * kSeg;
        const int64_t G = p.T > 0 ? cdiv(p.T, L) : 0;
        if (mult == 2 || (int64_t)nr * G * p.C >= 4096) break;
        mult--;
    }
    p.L = cdiv(mult * p.P1, kSeg) * kSeg;
    p.G = p.T > 0 ? cdiv(p.T, p.L) : 0;
    p.nseg = p.L / kSeg;
    return p;
}

struct BigWS {   // carved from one workspace; [rank][tile] blocks of fixed stride
    uint32_t *cnt;    // [nr][G][C][nseg]  counts, then exclusive offsets (chunk-major)
    uint32_t *cst;    // [nr][G][C + 1]    start of each chunk's list inside the tile's list
    uint32_t *list;   // [nr][G][L]        tile-local step indices, grouped by chunk
    uint32_t *val;    // [nr][G][P1]       per-tile last inserted value per slot, or kNone
    int32_t *err;     // device error flag (bounds guards; the handle's pss_check reports it)
};

size_t big_bytes(const BigPlan &p, int32_t nr) {
    const size_t t = (size_t)nr * (size_t)p.G;
    return 4 * (t * p.nseg * p.C + t * (p.C + 1) + t * p.L + t * p.P1) + 256;
}

BigWS big_ws(void *base, const BigPlan &p, int32_t nr) {
    const size_t t = (size_t)nr * (size_t)p.G;
    BigWS w;
    w.cnt = (uint32_t *)base;
    w.cst = w.cnt + t * p.nseg * p.C;
    w.list = w.cst + t * (p.C + 1);
    w.val = w.list + t * p.L;
    w.err = nullptr;
    return w;
}

struct TileInfo {
    int32_t rl;
    uint32_t tile, tlo, n, rank;
};

__device__ __forceinline__ TileInfo tile_info(const BigPlan &p, int32_t rank_lo, uint32_t rt) {
    TileInfo ti;
    ti.rl = (int32_t)(rt / (uint32_t)p.G);
    ti.tile = rt - (uint32_t)ti.rl * (uint32_t)p.G;
    ti.tlo = ti.tile * (uint32_t)p.L;
    ti.n = (uint32_t)(p.T - ti.tlo < p.L ? p.T - ti.tlo : p.L);
    ti.rank = (uint32_t)(rank_lo + ti.rl);
    return ti;
}

__device__ __forceinline__ uint32_t slot_of(uint32_t t, const SlotKey &sk, uint32_t P1) {
    return slot_draw(t, sk.s0, sk.s1, P1);
}

// ---- bucketing ------------------------------------------------------------------------------
// grid: (nr * G) * nseg one-wave blocks; block b -> (rank-tile rt, segment sg)
__global__ __launch_bounds__(64) void k_bk_count(Geometry g, BigPlan p, int32_t rank_lo, BigWS w) {
    extern __shared__ uint32_t hist[];    // C counters
    const uint32_t rt = blockIdx.x / (uint32_t)p.nseg, sg = blockIdx.x - rt * (uint32_t)p.nseg;
    const TileInfo ti = tile_info(p, rank_lo, rt);
    const uint32_t C = (uint32_t)p.C, P1 = (uint32_t)p.P1;
    for (uint32_t c = threadIdx.x; c < C; c += 64) hist[c] = 0;
    __syncthreads();
    const SlotKey sk = slot_key(g, ti.rank);
    const uint32_t lo = sg * kSeg, hi = lo + kSeg < ti.n ? lo + kSeg : ti.n;
    for (uint32_t base = lo; base < hi; base += 256) {
        uint32_t ch[4];
#pragma unroll
        for (int j = 0; j < 4; j++) ch[j] = slot_of(ti.tlo + base + 64u * j + threadIdx.x, sk, P1) >> kChunkBits;
#pragma unroll
        for (int j = 0; j < 4; j++)
            if (base + 64u * j + threadIdx.x < hi) atomicAdd(&hist[ch[j]], 1u);
    }
    __syncthreads();
    uint32_t *cnt = w.cnt + (size_t)rt * p.nseg * C + sg;
    for (uint32_t c = threadIdx.x; c < C; c += 64) cnt[(size_t)c * p.nseg] = hist[c];
}

// Two-level scan of the (chunk, segment) counts:
//   k_bk_scan_seg   one 256-thread block per (rank-tile, chunk): exclusive scan over the
//                   chunk's segments in place; the chunk's total -> cst[c]
//   k_bk_scan_chunk one block per rank-tile: exclusive scan of the chunk totals (cst[0..C])
// k_bk_scatter then starts segment sg of chunk c at cst[c] + cnt[c][sg].
__global__ __launch_bounds__(256) void k_bk_scan_seg(BigPlan p, BigWS w) {
    __shared__ uint32_t tot[4];
    const uint32_t C = (uint32_t)p.C, S = (uint32_t)p.nseg;
    const uint32_t rt = blockIdx.x / C, c = blockIdx.x - rt * C;
    uint32_t *cnt = w.cnt + ((size_t)rt * C + c) * S;
    const uint32_t per = (S + 255) / 256;
    const uint32_t lo = threadIdx.x * per < S ? threadIdx.x * per : S;
    const uint32_t hi = lo + per < S ? lo + per : S;
    uint32_t sum = 0;
    for (uint32_t i = lo; i < hi; i++) sum += cnt[i];
    uint32_t total;
    uint32_t run = block_excl_scan<256>(sum, tot, total);
    for (uint32_t i = lo; i < hi; i++) {
        const uint32_t v = cnt[i];
        cnt[i] = run;
        run += v;
    }
    if (threadIdx.x == 0) w.cst[(size_t)rt * (C + 1) + c] = total;
}

__global__ __launch_bounds__(1024) void k_bk_scan_chunk(BigPlan p, BigWS w) {
    __shared__ uint32_t tot[16];
    const uint32_t C = (uint32_t)p.C;
    uint32_t *cst = w.cst + (size_t)blockIdx.x * (C + 1);
    const uint32_t per = (C + 1023) / 1024;
    const uint32_t lo = threadIdx.x * per < C ? threadIdx.x * per : C;
    const uint32_t hi = lo + per < C ? lo + per : C;
    uint32_t sum = 0;
    for (uint32_t i = lo; i < hi; i++) sum += cst[i];
    uint32_t total;
    uint32_t run = block_excl_scan<1024>(sum, tot, total);
    for (uint32_t i = lo; i < hi; i++) {
        const uint32_t v = cst[i];
        cst[i] = run;
        run += v;
    }
    if (threadIdx.x == 0) cst[C] = total;
}

// grid as k_bk_count; one wave writes its segment's steps in order: the returning LDS add is
// served in lane order, so each chunk's list stays sorted by step
__global__ __launch_bounds__(64) void k_bk_scatter(Geometry g, BigPlan p, int32_t rank_lo, BigWS w) {
    extern __shared__ uint32_t off[];     // C cursors
    const uint32_t rt = blockIdx.x / (uint32_t)p.nseg, sg = blockIdx.x - rt * (uint32_t)p.nseg;
    const TileInfo ti = tile_info(p, rank_lo, rt);
    const uint32_t C = (uint32_t)p.C, P1 = (uint32_t)p.P1;
    const uint32_t *cnt = w.cnt + (size_t)rt * p.nseg * C + sg;
    const uint32_t *cst = w.cst + (size_t)rt * (C + 1);
    for (uint32_t c = threadIdx.x; c < C; c += 64) off[c] = cst[c] + cnt[(size_t)c * p.nseg];
    __syncthreads();
    const SlotKey sk = slot_key(g, ti.rank);
    uint32_t *list = w.list + (size_t)rt * p.L;
    const uint32_t lo = sg * kSeg, hi = lo + kSeg < ti.n ? lo + kSeg : ti.n;
    for (uint32_t base = lo; base < hi; base += 256) {
        uint32_t ch[4];
#pragma unroll
        for (int j = 0; j < 4; j++) ch[j] = slot_of(ti.tlo + base + 64u * j + threadIdx.x, sk, P1) >> kChunkBits;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const uint32_t t = base + 64u * j + threadIdx.x;
            if (t < hi) {
                const uint32_t pos = atomicAdd(&off[ch[j]], 1u);
                if (pos < ti.n) list[pos] = t;
                else if (w.err) atomicOr(w.err, 16);   // counts and scatter disagree
            }
        }
    }
}

// ---- per (tile, chunk) ------------------------------------------------------------------------
struct WindowCtx {   // pool2 windows touched by a tile: round keys staged in LDS
    uint32_t B, hB, w_lo, p_lo, w_last, len_last, h_last;
    bool walk_full;
    float invB;
};

__device__ __forceinline__ WindowCtx window_ctx(const Geometry &g, const BigPlan &p, uint32_t tlo,
                                                uint32_t n, uint32_t rank, uint32_t *rk) {
    WindowCtx wc;
    wc.B = (uint32_t)g.B;
    wc.hB = feistel_half_bits(wc.B);
    wc.w_lo = 1 + tlo / wc.B;
    wc.p_lo = tlo - (wc.w_lo - 1) * wc.B;
    wc.w_last = (uint32_t)(1 + (p.T - 1) / g.B);
    wc.len_last = (uint32_t)(g.ns - (int64_t)wc.w_last * g.B);
    wc.h_last = feistel_half_bits(wc.len_last);
    wc.walk_full = wc.B != (1u << (2 * wc.hB));
    wc.invB = 1.0f / (float)wc.B;
    const uint32_t nwin = (wc.p_lo + n - 1) / wc.B + 1;
    for (uint32_t j = threadIdx.x; j < nwin; j += blockDim.x)
        window_round_keys(g, rank, wc.w_lo + j, rk + kRoundKeyWords * j);
    return wc;
}

// value inserted at tile-local step t
__device__ __forceinline__ uint32_t ins_at(const WindowCtx &wc, const uint32_t *rk, uint32_t t) {
    uint32_t p = wc.p_lo + t;                              // < L + B < 2^25
    uint32_t d = (uint32_t)((float)p * wc.invB);           // p / B to within one, corrected
    int32_t r = (int32_t)(p - d * wc.B);
    if (r < 0) { d--; r += (int32_t)wc.B; }
    if (r >= (int32_t)wc.B) { d++; r -= (int32_t)wc.B; }
    const uint32_t w = wc.w_lo + d;
    const uint32_t *k = rk + kRoundKeyWords * d;
    uint32_t x;
    if (w != wc.w_last && !wc.walk_full) x = feistel_once((uint32_t)r, wc.hB, k);
    else {
        const bool lastw = w == wc.w_last;
        x = feistel((uint32_t)r, lastw ? wc.len_last : wc.B, lastw ? wc.h_last : wc.hB, k);
    }
    return w * wc.B + x;
}

constexpr int kMaxTileWindows = 8;    // tile <= 4 * P1 <= 4 * B steps -> <= 6 windows

// grid: (nr * G) * C one-wave blocks
__global__ __launch_bounds__(64) void k_bk_lastocc(Geometry g, BigPlan p, int32_t rank_lo, BigWS w) {
    __shared__ uint32_t lastT[kChunk];
    __shared__ uint32_t rk[kRoundKeyWords * kMaxTileWindows];
    const uint32_t C = (uint32_t)p.C, P1 = (uint32_t)p.P1;
    const uint32_t rt = blockIdx.x / C, c = blockIdx.x - rt * C;
    const TileInfo ti = tile_info(p, rank_lo, rt);
    const uint32_t s_lo = c << kChunkBits;
    const uint32_t ns_c = P1 - s_lo < kChunk ? P1 - s_lo : kChunk;
    for (uint32_t s = threadIdx.x; s < kChunk; s += 64) lastT[s] = 0;
    const WindowCtx wc = window_ctx(g, p, ti.tlo, ti.n, ti.rank, rk);
    const SlotKey sk = slot_key(g, ti.rank);
    __syncthreads();
    const uint32_t *cst = w.cst + (size_t)rt * (C + 1);
    const uint32_t *list = w.list + (size_t)rt * p.L;
    uint32_t a = cst[c], b = cst[c + 1];
    if (a > b || b > ti.n) {                       // bounds guard: never walk outside the list
        if (threadIdx.x == 0 && w.err) atomicOr(w.err, 32);
        a = b = 0;
    }
    // the list is in step order and one wave walks it in order: a later store wins (the
    // highest lane inside one store), so each slot ends with its last step
    for (uint32_t base = a; base < b; base += 256) {
        uint32_t t[4], s[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const uint32_t i = base + 64u * j + threadIdx.x;
            t[j] = i < b ? list[i] : 0u;
            s[j] = slot_of(ti.tlo + t[j], sk, P1) - s_lo;
        }
#pragma unroll
        for (int j = 0; j < 4; j++)
            if (base + 64u * j + threadIdx.x < b) lastT[s[j]] = t[j] + 1u;
    }
    __syncthreads();
    uint32_t *V = w.val + (size_t)rt * p.P1 + s_lo;
    for (uint32_t s = threadIdx.x; s < ns_c; s += 64) {
        const uint32_t lt = lastT[s];
        V[s] = lt ? ins_at(wc, rk, lt - 1u) : kNone;
    }
}

template <bool NARROW, bool XG>
__global__ __launch_bounds__(64) void k_bk_emit(Geometry g, BigPlan p, int32_t rank_lo, BigWS w,
                                                const RankDesc *__restrict__ ranks, uint32_t g_lo,
                                                uint32_t ng, int64_t pos_lo, int64_t count,
                                                int64_t *__restrict__ out) {
    __shared__ uint32_t buf[kChunk];
    __shared__ uint32_t rk[kRoundKeyWords * kMaxTileWindows];
    const uint32_t C = (uint32_t)p.C, P1 = (uint32_t)p.P1;
    // block -> (rank r, emitted tile g_lo + tt, chunk c).  Workgroups go to the 8 XCDs round
    // robin by index; when the tiles divide evenly, every chunk of a tile is placed on the
    // same XCD (tile rtt on XCD rtt % 8), so the ids the tile's 256 chunk waves scatter over
    // its positions meet in one L2 and leave it as whole lines.
    uint32_t rtt, c;
    if (XG) {   // host checked: nr * ng tiles divide by 8
        const uint32_t x = blockIdx.x & 7u, k = blockIdx.x >> 3;
        rtt = (k / C) * 8u + x;
        c = k - (k / C) * C;
    } else {
        rtt = blockIdx.x / C;
        c = blockIdx.x - rtt * C;
    }
    const uint32_t r = rtt / ng, tt = rtt - r * ng;
    const uint32_t rt = r * (uint32_t)p.G + g_lo + tt;
    const TileInfo ti = tile_info(p, rank_lo, rt);
    const RankDesc rd = ranks[ti.rank];
    const uint32_t s_lo = c << kChunkBits;
    const uint32_t ns_c = P1 - s_lo < kChunk ? P1 - s_lo : kChunk;
    {   // slot table at the tile's start: last values of the earlier tiles
        const uint32_t *VALr = w.val + (size_t)ti.rl * p.G * p.P1;
        for (uint32_t s = threadIdx.x; s < ns_c; s += 64)
            buf[s] = slot_value_after(VALr, p.P1, (int64_t)ti.tile - 1, s_lo + s);
    }
    const WindowCtx wc = window_ctx(g, p, ti.tlo, ti.n, ti.rank, rk);
    const SlotKey sk = slot_key(g, ti.rank);
    __syncthreads();
    const uint32_t twoB = (uint32_t)(2 * g.B < g.ns ? 2 * g.B : g.ns);
    const uint32_t old32 = (uint32_t)rd.old_start, new32 = (uint32_t)rd.new_start;
    const uint32_t N32 = (uint32_t)g.N;
    const int64_t pos_hi = pos_lo + count;
    // positions of this tile that the launch emits, tile-local: [e_lo, e_hi)
    const uint32_t e_lo = (uint32_t)(pos_lo > ti.tlo ? (pos_lo - ti.tlo < ti.n ? pos_lo - ti.tlo : ti.n) : 0);
    const uint32_t e_hi = (uint32_t)(pos_hi < (int64_t)ti.tlo + ti.n ? (pos_hi > ti.tlo ? pos_hi - ti.tlo : 0) : ti.n);
    int64_t *o = out + (int64_t)ti.rl * count + ((int64_t)ti.tlo - pos_lo);
    const uint32_t *cst = w.cst + (size_t)rt * (C + 1);
    const uint32_t *list = w.list + (size_t)rt * p.L;
    uint32_t a = cst[c], b = cst[c + 1];
    if (a > b || b > ti.n) {                       // bounds guard: never walk outside the list
        if (threadIdx.x == 0 && w.err) atomicOr(w.err, 64);
        a = b = 0;
    }
    Pacer pace(b - a);
    for (uint32_t base = a; base < b; base += 256) {
        pace.step(base - a);
        uint32_t t[4], s[4], ins[4], v[4] = {0, 0, 0, 0};
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const uint32_t i = base + 64u * j + threadIdx.x;
            t[j] = i < b ? list[i] : 0u;
            s[j] = slot_of(ti.tlo + t[j], sk, P1) - s_lo;
            ins[j] = ins_at(wc, rk, t[j]);
        }
#pragma unroll
        for (int j = 0; j < 4; j++)
            if (base + 64u * j + threadIdx.x < b) v[j] = atomicExch(&buf[s[j]], ins[j]);
#pragma unroll
        for (int j = 0; j < 4; j++)
            if (base + 64u * j + threadIdx.x < b && t[j] >= e_lo && t[j] < e_hi)
                o[t[j]] = emit_id<NARROW>(v[j], twoB, old32, new32, N32, rd, g);
    }
}

}  // namespace

bool v2_big_applicable(const Geometry &g) {
    const int64_t P1 = g.B < g.ns ? g.B : g.ns;
    return P1 > kLdsSlotMax && P1 <= kBigMaxP1 && lds_xchg_ordered() && lds_write_ordered() &&
           lds_add_ordered();
}

size_t v2_big_bytes(const Geometry &g, int32_t nr) {
    return big_bytes(big_plan(g, nr), nr);
}

hipError_t launch_v2_big(const Geometry &g, const RankDesc *ranks, int32_t rank_lo, int32_t nr,
                         int64_t pos_lo, int64_t count, int64_t *out, void *ws, int32_t *err,
                         hipStream_t s, const Marker &mk, int stage) {
    // stage V2_STAGE_PRE: the bucketing + last-occurrence kernels (they read only the epoch key
    // and write `ws`); V2_STAGE_EMIT: the replay and the tail, from that `ws`
    const bool do_pre = stage != V2_STAGE_EMIT, do_emit = stage != V2_STAGE_PRE;
    const BigPlan p = big_plan(g, nr);
    BigWS w = big_ws(ws, p, nr);
    w.err = err;
    static const bool dbg = getenv("PSS_DEBUG_SYNC") != nullptr;   // diagnostic: sync per kernel
    auto chk = [&](const char *what) -> hipError_t {
        if (!dbg) return hipSuccess;
        const hipError_t e = hipStreamSynchronize(s);
        fprintf(stderr, "[pss debug] %s: %s (P1 %lld L %lld G %lld C %lld)\n", what, hipGetErrorString(e),
                (long long)p.P1, (long long)p.L, (long long)p.G, (long long)p.C);
        return e;
    };
    const int64_t pos_hi = pos_lo + count < g.ns ? pos_lo + count : g.ns;
    if (nr <= 0 || pos_hi <= pos_lo) return hipSuccess;
    const bool need_tail = pos_hi > p.T;
    if (p.G > 0) {
        // every tile of every rank is bucketed and scanned (the tail needs the last VAL);
        // emit runs over the tiles that hold requested positions
        const uint32_t rts = (uint32_t)(nr * p.G);
        const size_t lds_c = (size_t)p.C * 4;
        hipError_t e;
        if (do_pre) {
        mk(K_V2_LASTOCC, s);
        hipLaunchKernelGGL(k_bk_count, dim3(rts * (uint32_t)p.nseg), dim3(64), lds_c, s, g, p, rank_lo, w);
        if ((e = chk("k_bk_count")) != hipSuccess) return e;
        hipLaunchKernelGGL(k_bk_scan_seg, dim3(rts * (uint32_t)p.C), dim3(256), 0, s, p, w);
        if ((e = chk("k_bk_scan_seg")) != hipSuccess) return e;
        hipLaunchKernelGGL(k_bk_scan_chunk, dim3(rts), dim3(1024), 0, s, p, w);
        if ((e = chk("k_bk_scan_chunk")) != hipSuccess) return e;
        hipLaunchKernelGGL(k_bk_scatter, dim3(rts * (uint32_t)p.nseg), dim3(64), lds_c, s, g, p, rank_lo, w);
        if ((e = chk("k_bk_scatter")) != hipSuccess) return e;
        hipLaunchKernelGGL(k_bk_lastocc, dim3(rts * (uint32_t)p.C), dim3(64), 0, s, g, p, rank_lo, w);
        if ((e = chk("k_bk_lastocc")) != hipSuccess) return e;
        }
        if (!do_emit) { mk(-1, s); return hipGetLastError(); }
        const int64_t last_emit = pos_lo < p.T ? ((pos_hi < p.T ? pos_hi : p.T) - 1) / p.L : -1;
        if (last_emit >= 0) {
            mk(K_V2_EMIT, s);
            const int64_t g_lo = pos_lo / p.L;
            const bool narrow = g.N + g.ns < (int64_t)UINT32_MAX;
            const uint32_t ng = (uint32_t)(last_emit - g_lo + 1);
            const dim3 grid((uint32_t)nr * ng * (uint32_t)p.C);
            static const int xcd_group = [] {   // A/B knob: 0 = chunks of a tile spread over XCDs
                const char *e = getenv("PSS_V2BIG_XCD");
                return e ? atoi(e) : 1;
            }();
            // the mapping is a template parameter chosen here: with the choice made inside the
            // kernel (a runtime branch on gridDim), hipcc 7.2 reused a clobbered SGPR for the
            // block index on the fallback path and the chunk index ran outside the tile
            const bool xg = xcd_group && ((uint32_t)nr * ng) % 8u == 0;
            auto kern = narrow ? (xg ? k_bk_emit<true, true> : k_bk_emit<true, false>)
                               : (xg ? k_bk_emit<false, true> : k_bk_emit<false, false>);
            hipLaunchKernelGGL(kern, grid, dim3(64), 0, s, g, p, rank_lo, w, ranks, (uint32_t)g_lo, ng,
                               pos_lo, count, out);
            if ((e = chk("k_bk_emit")) != hipSuccess) return e;
        }
    }
    if (!do_emit) return hipGetLastError();
    if (need_tail) {
        mk(K_V2_TAIL, s);
        V2Plan vp{};
        vp.P1 = p.P1; vp.T = p.T; vp.L = p.L; vp.G = p.G; vp.global_buf = 1;
        hipError_t e = launch_v2_tail_vals(g, vp, ranks, rank_lo, nr, w.val, pos_lo, count, out, s, KeyTab{nullptr, 0});
        if (e != hipSuccess) return e;
        if ((e = chk("k_v2_tail_f")) != hipSuccess) return e;
    }
    mk(-1, s);
    return hipGetLastError();
}

hipError_t init_kernel_attributes_v2big() {
    const int big = 160 * 1024;
    hipError_t e = hipSuccess;
#define PSS_ATTR(fn) { hipError_t x = hipFuncSetAttribute((const void *)(fn), hipFuncAttributeMaxDynamicSharedMemorySize, big); if (x != hipSuccess) e = x; }
    PSS_ATTR(k_bk_count);
    PSS_ATTR(k_bk_scatter);
#undef PSS_ATTR
    return e;
}

}  // namespace pss
