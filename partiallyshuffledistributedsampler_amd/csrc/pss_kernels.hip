// pss_kernels.hip -- gfx950 (MI355X / CDNA4) kernels of the partial-shuffle sampler.
//
// The hot path of the reference (index generation, V1:157-172 / V2:96-116, and the id ->
// (file, offset) scan, V1:181-221) is restated as integer, HBM-write-bound kernels:
//
//   k_scan_prefix      exclusive scan of files_len over the shuffled file order (wave64 DPP)
//   k_part_*           balanced file -> rank partition (segments of each rank's id block)
//   k_v1_lds<EPT>      V1: one workgroup per (rank, window); pool permutation = stable sort
//                      of Philox keys in LDS (12..14-bit bucket pass + in-bucket fix-up)
//   k_v2_lastocc       V2 pass A: per tile, last occurrence of every slot (LDS ds_max)
//   k_v2_emit          V2 pass B: one wave per tile replays the TF-style shuffle buffer
//                      (slot table in LDS, wave-ballot conflict resolution)
//   k_v2_tail<EPT>     V2: final buffer drained in a Philox-sorted order
//   k_map, k_digest    id -> (file position, offset); coverage digest for the RCCL check
//
// Schedule definitions live in DESIGN.md §3 and are restated on the CPU in
// oracle/pss_oracle.c (orc_v1_philox_stream / orc_v2_philox_stream): both must agree bit for
// bit.  No MFMA anywhere -- this is integer, memory/latency-bound work.
#include "pss_common.h"
#include "pss_kernels.h"

#include <cstdlib>

namespace pss {

// ------------------------------------------------------------------------------------------
// wave64 / workgroup primitives
// ------------------------------------------------------------------------------------------
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
// scan + partition (V1:27-53,181-190 / V2:27-49,184-193)
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void k_scan_prefix(const int64_t *__restrict__ lens,
                                                      const int32_t *__restrict__ order,
                                                      int64_t F, int64_t *__restrict__ prefix) {
    __shared__ uint64_t tot[16];
    const int64_t per = (F + 1023) / 1024;
    int64_t lo = (int64_t)threadIdx.x * per;
    if (lo > F) lo = F;
    const int64_t hi = lo + per < F ? lo + per : F;
    uint64_t s = 0;
    for (int64_t f = lo; f < hi; f++) s += (uint64_t)lens[order[f]];
    uint64_t total;
    uint64_t run = block_excl_scan<1024>(s, tot, total);
    for (int64_t f = lo; f < hi; f++) {
        prefix[f] = (int64_t)run;
        run += (uint64_t)lens[order[f]];
    }
    if (threadIdx.x == 0) prefix[F] = (int64_t)total;
}

// largest f in [0, F) with prefix[f] <= id  (the file holding id; empty files are skipped
// because an empty file shares its prefix with the next one)
__device__ __forceinline__ int64_t file_of(const int64_t *prefix, int64_t F, int64_t id) {
    int64_t lo = 0, hi = F;
    while (hi - lo > 1) {
        const int64_t mid = (lo + hi) >> 1;
        if (prefix[mid] <= id) lo = mid; else hi = mid;
    }
    return lo;
}

// The id ranges a rank reads in one epoch, in stream order, wrapped at N and clipped to the
// scanned total T = prefix[F] (ids >= T are reflected by the host, V1:191-196).
struct Ranges { int64_t lo[4], hi[4]; int n; };

__device__ void rank_ranges(const Geometry &g, const RankDesc &rd, int64_t T, Ranges &r) {
    int64_t plo[2], plen[2];
    int np = 0;
    if (g.version == 1) {
        plo[0] = rd.new_start; plen[0] = g.ns; np = 1;
    } else {
        const int64_t a = 2 * g.B < g.ns ? 2 * g.B : g.ns;
        plo[0] = rd.old_start; plen[0] = a; np = 1;
        if (g.ns > a) { plo[1] = rd.new_start + a; plen[1] = g.ns - a; np = 2; }
    }
    r.n = 0;
    for (int i = 0; i < np; i++) {
        int64_t lo = plo[i] % g.N, len = plen[i];
        while (len > 0) {
            const int64_t take = (g.N - lo) < len ? (g.N - lo) : len;
            int64_t h = lo + take;
            int64_t l = lo;
            if (h > T) h = T;
            if (l < h) { r.lo[r.n] = l; r.hi[r.n] = h; r.n++; }
            len -= take;
            lo = 0;
        }
    }
}

__global__ void k_part_count(Geometry g, const RankDesc *ranks, int32_t rank_lo, int32_t nr,
                             const int64_t *prefix, int64_t F, int64_t *seg_off) {
    const int64_t T = prefix[F];
    for (int32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nr; i += gridDim.x * blockDim.x) {
        Ranges rr;
        rank_ranges(g, ranks[rank_lo + i], T, rr);
        int64_t c = 0;
        for (int k = 0; k < rr.n; k++) {
            const int64_t f0 = file_of(prefix, F, rr.lo[k]);
            const int64_t f1 = file_of(prefix, F, rr.hi[k] - 1);
            for (int64_t f = f0; f <= f1; f++) c += prefix[f + 1] > prefix[f];
        }
        seg_off[i + 1] = c;
    }
}

__global__ __launch_bounds__(1024) void k_excl_scan_inplace(int64_t *a, int64_t n) {
    // a[0] := 0, a[1..n] := inclusive scan of counts stored in a[1..n]
    __shared__ uint64_t tot[16];
    const int64_t per = (n + 1023) / 1024;
    int64_t lo = (int64_t)threadIdx.x * per;
    if (lo > n) lo = n;
    const int64_t hi = lo + per < n ? lo + per : n;
    uint64_t s = 0;
    for (int64_t i = lo; i < hi; i++) s += (uint64_t)a[i + 1];
    uint64_t total;
    uint64_t run = block_excl_scan<1024>(s, tot, total);
    for (int64_t i = lo; i < hi; i++) { run += (uint64_t)a[i + 1]; a[i + 1] = (int64_t)run; }
    if (threadIdx.x == 0) a[0] = 0;
}

__global__ void k_part_emit(Geometry g, const RankDesc *ranks, int32_t rank_lo, int32_t nr,
                            const int64_t *prefix, int64_t F, const int64_t *seg_off,
                            int32_t *seg_file, int64_t *seg_lo, int64_t *seg_hi,
                            int64_t seg_cap, int32_t *err) {
    const int64_t T = prefix[F];
    for (int32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nr; i += gridDim.x * blockDim.x) {
        Ranges rr;
        rank_ranges(g, ranks[rank_lo + i], T, rr);
        int64_t o = seg_off[i];
        if (seg_off[i + 1] > seg_cap) { atomicOr(err, 1); continue; }
        for (int k = 0; k < rr.n; k++) {
            const int64_t f0 = file_of(prefix, F, rr.lo[k]);
            const int64_t f1 = file_of(prefix, F, rr.hi[k] - 1);
            for (int64_t f = f0; f <= f1; f++) {
                if (prefix[f + 1] <= prefix[f]) continue;
                const int64_t a = rr.lo[k] > prefix[f] ? rr.lo[k] : prefix[f];
                const int64_t b = rr.hi[k] < prefix[f + 1] ? rr.hi[k] : prefix[f + 1];
                seg_file[o] = (int32_t)f;
                seg_lo[o] = a - prefix[f];
                seg_hi[o] = b - prefix[f];
                o++;
            }
        }
    }
}

// id -> (file position, offset) over the shuffled order (V1:181-221).  Ids at or past the
// scanned total are reflected exactly as V1:191-196 does; the host moves those to the end of
// their batch (they are flagged by a negative file position: fpos = -1 - f).
__global__ void k_map(const int64_t *__restrict__ prefix, int64_t F,
                      const int64_t *__restrict__ ids, int64_t n, int32_t *__restrict__ fpos,
                      int64_t *__restrict__ off) {
    const int64_t T = prefix[F];
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        int64_t id = ids[i];
        bool refl = false;
        if (id >= T) {
            id = 2 * T - id;
            if (id == T) id = T - 1;
            refl = true;
        }
        if (id < 0) { fpos[i] = INT32_MIN; off[i] = ids[i]; continue; }
        const int64_t f = file_of(prefix, F, id);
        fpos[i] = refl ? (int32_t)(-1 - f) : (int32_t)f;
        off[i] = id - prefix[f];
    }
}

__global__ void k_digest(const int64_t *__restrict__ ids, int64_t n, uint64_t *acc) {
    uint64_t s = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        s += mix64((uint64_t)ids[i]);
    s = wave_sum(s);
    if ((threadIdx.x & 63) == 0) atomicAdd((unsigned long long *)acc, (unsigned long long)s);
}

__global__ void k_digest_range(int64_t lo, int64_t hi, uint64_t *acc) {
    uint64_t s = 0;
    for (int64_t i = lo + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < hi;
         i += (int64_t)gridDim.x * blockDim.x)
        s += mix64((uint64_t)i);
    s = wave_sum(s);
    if ((threadIdx.x & 63) == 0) atomicAdd((unsigned long long *)acc, (unsigned long long)s);
}

__global__ void k_debug_wave_scan(const uint64_t *in, uint64_t *out, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t x = i < n ? in[i] : 0;
    const uint64_t y = wave_incl_scan(x);
    const uint32_t y32 = wave_incl_scan((uint32_t)x);
    if (i < n) { out[2 * i] = y; out[2 * i + 1] = y32; }
}

// ------------------------------------------------------------------------------------------
// LDS pool permutation: perm = stable argsort of Philox keys (i>>2, c1, rank, dom)[i&3].
// One 256-thread workgroup, n <= 256*EPT.  Keys stay in registers; LDS holds a 2^hb-bucket
// histogram (hb = ceil(log2 n), i.e. the keys' top hb bits) and the n packed slots
// (low 32-hb key bits << hb | i).  A bucket averages one element, so the in-bucket fix-up is
// a short insertion sort.  Result: S[p] & (2^hb - 1) = index of the p-th smallest key.
// ------------------------------------------------------------------------------------------
template <int EPT>
__device__ __forceinline__ int block_sort_keys(uint32_t k0, uint32_t k1, uint32_t c1,
                                               uint32_t rank, uint32_t dom, int n,
                                               uint32_t *S, uint32_t *hist, uint32_t *tot) {
    constexpr int NQ = EPT / 4;
    const int tid = threadIdx.x;
    const int hb = n > 1 ? ceil_log2_u64((uint64_t)n) : 0;
    const int nb = 1 << hb;
    uint32_t key[NQ][4];
#pragma unroll
    for (int j = 0; j < NQ; j++) {
        uint32_t c0 = (uint32_t)(tid + 256 * j), cc1 = c1, c2 = rank, c3 = dom;
        philox4x32_10(c0, cc1, c2, c3, k0, k1);
        key[j][0] = c0; key[j][1] = cc1; key[j][2] = c2; key[j][3] = c3;
    }
    for (int i = tid; i < nb; i += 256) hist[i] = 0;
    __syncthreads();
    const int sh = 32 - hb;
#pragma unroll
    for (int j = 0; j < NQ; j++)
#pragma unroll
        for (int w = 0; w < 4; w++) {
            const int i = 4 * (tid + 256 * j) + w;
            if (i < n) atomicAdd(&hist[hb ? key[j][w] >> sh : 0], 1u);
        }
    __syncthreads();
    const int per = nb >= 256 ? nb / 256 : 1;
    const int blo = tid * per < nb ? tid * per : nb;
    const int bhi = blo + per < nb ? blo + per : nb;
    uint32_t s = 0;
    for (int b = blo; b < bhi; b++) s += hist[b];
    uint32_t total;
    uint32_t run = block_excl_scan<256>(s, tot, total);
    for (int b = blo; b < bhi; b++) { const uint32_t c = hist[b]; hist[b] = run; run += c; }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < NQ; j++)
#pragma unroll
        for (int w = 0; w < 4; w++) {
            const int i = 4 * (tid + 256 * j) + w;
            if (i < n) {
                const uint32_t k = key[j][w];
                const uint32_t pos = atomicAdd(&hist[hb ? k >> sh : 0], 1u);
                S[pos] = hb ? ((k << hb) | (uint32_t)i) : 0u;
            }
        }
    __syncthreads();
    for (int b = blo; b < bhi; b++) {  // hist[b] is now the END of bucket b
        const int e = (int)hist[b];
        const int st = b ? (int)hist[b - 1] : 0;
        for (int x = st + 1; x < e; x++) {
            const uint32_t v = S[x];
            int y = x - 1;
            while (y >= st && S[y] > v) { S[y + 1] = S[y]; y--; }
            S[y + 1] = v;
        }
    }
    __syncthreads();
    return hb;
}

template <int EPT>
constexpr size_t sort_lds_bytes() { return (size_t)(2 * 256 * EPT + 16) * sizeof(uint32_t); }

// ------------------------------------------------------------------------------------------
// V1 (V1:157-172): window w of rank r -> ids start + w*B + perm_w[p], wrap at N
// ------------------------------------------------------------------------------------------
template <int EPT>
__global__ __launch_bounds__(256) void k_v1_lds(Geometry g, const RankDesc *__restrict__ ranks,
                                               int32_t rank_lo, int64_t w_lo, int64_t nw,
                                               int64_t pos_lo, int64_t count,
                                               int64_t *__restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    uint32_t *S = smem, *hist = smem + 256 * EPT, *tot = hist + 256 * EPT;
    const int32_t rl = (int32_t)(blockIdx.x / nw);
    const int64_t w = w_lo + (int64_t)(blockIdx.x % nw);
    const int32_t rank = rank_lo + rl;
    const int64_t wb = w * g.B;
    const int n = (int)(g.ns - wb < g.B ? g.ns - wb : g.B);
    const int64_t base = ranks[rank].new_start + wb;
    int hb = 0;
    if (g.shuffle) hb = block_sort_keys<EPT>(g.key0, g.key1, (uint32_t)w, (uint32_t)rank, DOM_V1_WIN, n, S, hist, tot);
    const uint32_t mask = (1u << hb) - 1u;
    int64_t *o = out + (int64_t)rl * count - pos_lo;
    int p0 = 0, p1 = n;
    if (wb < pos_lo) p0 = (int)(pos_lo - wb);
    if (wb + n > pos_lo + count) p1 = (int)(pos_lo + count - wb);
    for (int p = p0 + threadIdx.x; p < p1; p += 256) {
        const uint32_t idx = g.shuffle ? (S[p] & mask) : (uint32_t)p;
        o[wb + p] = wrap_id(base + idx, g.N);
    }
}

// ------------------------------------------------------------------------------------------
// V2 slot machine (V2:96-116 in slot-replacement form)
// ------------------------------------------------------------------------------------------
struct InsCtx {             // Feistel round keys of the pool2 windows a tile inserts
    const uint32_t *rk;     // LDS: 4 words per window, window w at rk[4*(w - w_lo)]
    int64_t w_lo;
};

__device__ __forceinline__ uint32_t ins_value(const Geometry &g, const InsCtx &c, int64_t t) {
    const int64_t w = 1 + t / g.B;           // pool2 window being drained at step t
    const int64_t p = t - (w - 1) * g.B;     // its p-th insertion
    const int64_t rem = g.ns - w * g.B;
    const uint32_t len = (uint32_t)(rem < g.B ? rem : g.B);
    const uint32_t *k = c.rk + 4 * (w - c.w_lo);
    return (uint32_t)(w * g.B) + feistel((uint32_t)p, len, feistel_half_bits(len), k[0], k[1], k[2], k[3]);
}

__device__ __forceinline__ int64_t v2_id(uint32_t v, const RankDesc &rd, const Geometry &g) {
    return wrap_id(((int64_t)v < 2 * g.B ? rd.old_start : rd.new_start) + (int64_t)v, g.N);
}

__device__ __forceinline__ void stage_round_keys(const Geometry &g, uint32_t rank, int64_t w_lo,
                                                 int nwin, uint32_t *rk) {
    for (int j = threadIdx.x; j < nwin; j += blockDim.x) {
        uint32_t c0 = (uint32_t)(w_lo + j), c1 = 0, c2 = rank, c3 = DOM_V2_INS;
        philox4x32_10(c0, c1, c2, c3, g.key0, g.key1);
        rk[4 * j] = c0; rk[4 * j + 1] = c1; rk[4 * j + 2] = c2; rk[4 * j + 3] = c3;
    }
}

__device__ __forceinline__ void tile_windows(const Geometry &g, int64_t tlo, int64_t thi,
                                             int64_t &w_lo, int &nwin) {
    w_lo = 1 + tlo / g.B;
    nwin = (int)(1 + (thi - 1) / g.B - w_lo + 1);
}

// slot draw of step t: super-batch sb = t>>8 holds 256 steps; lane l of a wave draws the
// Philox block (sb*64 + l) and its word j is the slot of step sb*256 + j*64 + l.
__device__ __forceinline__ void slot_words(const Geometry &g, uint32_t rank, int64_t sb, int lane,
                                           uint32_t u[4]) {
    const uint64_t c = (uint64_t)sb * 64u + (uint64_t)lane;
    uint32_t c0 = (uint32_t)c, c1 = (uint32_t)(c >> 32), c2 = rank, c3 = DOM_V2_SLOT;
    philox4x32_10(c0, c1, c2, c3, g.key0, g.key1);
    u[0] = c0; u[1] = c1; u[2] = c2; u[3] = c3;
}

// Pass A: last occurrence of every slot inside tile `tile` -> VAL[tile][s] = value inserted
// there (virtual index), or kNone if the tile never draws s.  Order-independent (ds_max).
__global__ __launch_bounds__(256) void k_v2_lastocc(Geometry g, V2Plan pl, int32_t rank_lo,
                                                    int64_t ng, uint32_t *__restrict__ VAL) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    const int P1 = (int)pl.P1;
    uint32_t *lastT = smem, *rk = smem + P1;
    const int32_t rl = (int32_t)(blockIdx.x / ng);
    const int64_t tile = (int64_t)(blockIdx.x % ng);
    const uint32_t rank = (uint32_t)(rank_lo + rl);
    const int64_t tlo = tile * pl.L;
    const int64_t thi = tlo + pl.L < pl.T ? tlo + pl.L : pl.T;
    int64_t w_lo; int nwin;
    tile_windows(g, tlo, thi, w_lo, nwin);
    for (int s = threadIdx.x; s < P1; s += 256) lastT[s] = 0;
    stage_round_keys(g, rank, w_lo, nwin, rk);
    __syncthreads();
    const int64_t sb_lo = tlo >> 8, sb_hi = (thi - 1) >> 8;
    const int64_t ncnt = (sb_hi - sb_lo + 1) * 64;
    for (int64_t ci = threadIdx.x; ci < ncnt; ci += 256) {
        const int64_t sb = sb_lo + (ci >> 6);
        const int lane = (int)(ci & 63);
        uint32_t u[4];
        slot_words(g, rank, sb, lane, u);
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int64_t t = sb * 256 + j * 64 + lane;
            if (t >= tlo && t < thi) atomicMax(&lastT[scale32(u[j], (uint32_t)P1)], (uint32_t)(t - tlo + 1));
        }
    }
    __syncthreads();
    InsCtx ic{rk, w_lo};
    uint32_t *V = VAL + ((int64_t)rl * pl.G + tile) * P1;
    for (int s = threadIdx.x; s < P1; s += 256) {
        const uint32_t lt = lastT[s];
        V[s] = lt ? ins_value(g, ic, tlo + (int64_t)lt - 1) : kNone;
    }
}

// value held by slot s after tile `tile` (walk back over tiles that never drew s)
__device__ __forceinline__ uint32_t slot_value_after(const uint32_t *VALr, const V2Plan &pl,
                                                     int64_t tile, int s) {
    for (int64_t gg = tile; gg >= 0; gg--) {
        const uint32_t v = VALr[gg * pl.P1 + s];
        if (v != kNone) return v;
    }
    return (uint32_t)s;  // initial pool1 = window 0 in slot order
}

// Pass B: one wave replays tile `tile` in step order.
__global__ __launch_bounds__(64) void k_v2_emit(Geometry g, V2Plan pl,
                                                const RankDesc *__restrict__ ranks,
                                                int32_t rank_lo, int64_t g_lo, int64_t ng,
                                                const uint32_t *__restrict__ VAL,
                                                int64_t pos_lo, int64_t count,
                                                int64_t *__restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    const int P1 = (int)pl.P1;
    uint32_t *buf = smem;                                   // slot table: P1 virtual ids
    uint32_t *rk = smem + P1;                               // Feistel keys of the tile's windows
    const int64_t nwin_max = pl.L / g.B + 2;
    // collision probe, P1 bytes; volatile so the read-back is never forwarded from the store,
    // and explicitly in LDS (a generic volatile pointer would lower to flat sc0 sc1 accesses)
    typedef __attribute__((address_space(3))) volatile uint8_t lds_vu8;
    lds_vu8 *mark = (lds_vu8 *)(rk + 4 * nwin_max);
    const int lane = threadIdx.x;
    const int32_t rl = (int32_t)(blockIdx.x / ng);
    const int64_t tile = g_lo + (int64_t)(blockIdx.x % ng);
    const uint32_t rank = (uint32_t)(rank_lo + rl);
    const RankDesc rd = ranks[rank];
    const int64_t tlo = tile * pl.L;
    const int64_t thi = tlo + pl.L < pl.T ? tlo + pl.L : pl.T;
    int64_t w_lo; int nwin;
    tile_windows(g, tlo, thi, w_lo, nwin);
    const uint32_t *VALr = VAL + (int64_t)rl * pl.G * P1;
    for (int s = lane; s < P1; s += 64) buf[s] = slot_value_after(VALr, pl, tile - 1, s);
    stage_round_keys(g, rank, w_lo, nwin, rk);
    __syncthreads();
    const uint64_t lt_mask = (1ull << lane) - 1ull;
    const uint64_t gt_mask = ~lt_mask << 1;
    const int64_t sb_lo = tlo >> 8, sb_hi = (thi - 1) >> 8;
    // tile-local 32-bit step index tl = t - tlo; the tile emits tl in [e_lo, e_hi)
    const int64_t pos_hi = pos_lo + count;
    const uint32_t nvalid = (uint32_t)(thi - tlo);
    const uint32_t e_lo = (uint32_t)(pos_lo > tlo ? (pos_lo - tlo < nvalid ? pos_lo - tlo : nvalid) : 0);
    const uint32_t e_hi = (uint32_t)(pos_hi < thi ? (pos_hi > tlo ? pos_hi - tlo : 0) : nvalid);
    int64_t *o = out + (int64_t)rl * count + (tlo - pos_lo);
    // ids: v < 2B came from the OLD start, the rest from the NEW one; 32-bit when N allows
    const bool narrow = g.N + g.ns < (int64_t)UINT32_MAX;
    const uint32_t twoB = (uint32_t)(2 * g.B < g.ns ? 2 * g.B : g.ns);
    const uint32_t old32 = (uint32_t)rd.old_start, new32 = (uint32_t)rd.new_start;
    const uint32_t N32 = (uint32_t)g.N;
    // pool2 window bookkeeping without per-step division: (w0, p0) = window and insertion
    // index of the sub-batch's first step t0, advanced by 64 per sub-batch.
    const uint32_t B = (uint32_t)g.B;
    const uint32_t hB = feistel_half_bits(B);
    const uint32_t w_last = (uint32_t)(1 + (pl.T - 1) / g.B);     // last pool2 window (may be short)
    const uint32_t len_last = (uint32_t)(g.ns - (int64_t)w_last * g.B);
    const uint32_t h_last = feistel_half_bits(len_last);
    const uint32_t w_lo32 = (uint32_t)w_lo;
    const int64_t t_first = sb_lo * 256;
    uint32_t w0 = (uint32_t)(1 + t_first / g.B);
    uint32_t p0 = (uint32_t)(t_first - (int64_t)(w0 - 1) * g.B);
    int32_t tl0 = (int32_t)(t_first - tlo);   // negative while the super-batch starts before the tile
    for (int64_t sb = sb_lo; sb <= sb_hi; sb++, tl0 += 256) {
        uint32_t u[4];
        slot_words(g, rank, sb, lane, u);
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int32_t tl = tl0 + j * 64 + lane;
            const bool valid = (uint32_t)tl < nvalid;
            const uint32_t k = scale32(u[j], (uint32_t)P1);
            // insertion of step t: window w, index p (p0 + lane crosses at most one window
            // boundary when B >= 64; smaller pools loop)
            uint32_t p = p0 + (uint32_t)lane;
            uint32_t w = w0;
            if (p >= B) {
                p -= B; w++;
                while (p >= B) { p -= B; w++; }
            }
            uint32_t ins = 0;
            if (valid) {
                const bool lastw = w == w_last;
                const uint32_t *kk = rk + 4 * (w - w_lo32);
                ins = w * B + feistel(p, lastw ? len_last : B, lastw ? h_last : hB,
                                      kk[0], kk[1], kk[2], kk[3]);
            }
            // collision probe: every valid lane writes its lane id to mark[k]; a lane that
            // reads back another id shares its slot with a lane of this sub-batch
            if (valid) mark[k] = (uint8_t)lane;
            const bool clash = valid && mark[k] != (uint8_t)lane;
            // peers of each clashing slot: one compare + ballot per distinct slot
            uint64_t cm = __ballot(clash);
            uint64_t lower = 0;
            bool last = true;
            while (cm) {
                const int c = __ffsll((long long)cm) - 1;
                const uint32_t sc = (uint32_t)__builtin_amdgcn_readlane((int)k, c);
                const bool same = valid && k == sc;
                const uint64_t m = __ballot(same);
                if (same) { lower = m & lt_mask; last = (m & gt_mask) == 0; }
                cm &= ~m;
            }
            const int src = lower ? 63 - __clzll((long long)lower) : lane;
            const uint32_t from_peer = (uint32_t)__shfl((int)ins, src);
            const uint32_t from_buf = buf[k];
            const uint32_t v = lower ? from_peer : from_buf;
            if (valid && last) buf[k] = ins;
            if ((uint32_t)tl >= e_lo && (uint32_t)tl < e_hi) {
                if (narrow) {
                    uint32_t id = (v < twoB ? old32 : new32) + v;
                    id = id >= N32 ? id - N32 : id;
                    o[tl] = (int64_t)id;
                } else {
                    o[tl] = v2_id(v, rd, g);
                }
            }
            p0 += 64;
            while (p0 >= B) { p0 -= B; w0++; }
        }
    }
}

// Tail: the final pool1 drained in the order of a stable sort of Philox keys.
template <int EPT>
__global__ __launch_bounds__(256) void k_v2_tail(Geometry g, V2Plan pl,
                                                const RankDesc *__restrict__ ranks,
                                                int32_t rank_lo, const uint32_t *__restrict__ VAL,
                                                int64_t pos_lo, int64_t count,
                                                int64_t *__restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    uint32_t *S = smem, *hist = smem + 256 * EPT, *tot = hist + 256 * EPT;
    const int32_t rl = (int32_t)blockIdx.x;
    const uint32_t rank = (uint32_t)(rank_lo + rl);
    const RankDesc rd = ranks[rank];
    const int P1 = (int)pl.P1;
    const int hb = block_sort_keys<EPT>(g.key0, g.key1, 0u, rank, DOM_V2_TAIL, P1, S, hist, tot);
    const uint32_t mask = (1u << hb) - 1u;
    const uint32_t *VALr = VAL + (int64_t)rl * pl.G * P1;
    int64_t *o = out + (int64_t)rl * count - pos_lo;
    const int64_t pos_hi = pos_lo + count;
    for (int j = threadIdx.x; j < P1; j += 256) {
        const int64_t pos = pl.T + j;
        if (pos < pos_lo || pos >= pos_hi) continue;
        const int s = (int)(S[j] & mask);
        o[pos] = v2_id(slot_value_after(VALr, pl, pl.G - 1, s), rd, g);
    }
}

// ------------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------------
static inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

V2Plan v2_plan(const Geometry &g) {
    V2Plan p{};
    p.P1 = g.B < g.ns ? g.B : g.ns;
    p.T = g.ns - p.P1;
    p.global_buf = p.P1 > kLdsSlotMax;
    static const int64_t mult = [] {
        const char *e = getenv("PSS_V2_TILE_MULT");   // tuning knob: tile = mult * P1 steps
        const long v = e ? atol(e) : 0;
        return (int64_t)(v > 0 ? v : 16);
    }();
    p.L = cdiv(mult * p.P1, 256) * 256;
    p.G = p.T > 0 ? cdiv(p.T, p.L) : 0;
    return p;
}

hipError_t launch_scan_prefix(const int64_t *lens, const int32_t *order, int64_t F,
                              int64_t *prefix, hipStream_t s) {
    hipLaunchKernelGGL(k_scan_prefix, dim3(1), dim3(1024), 0, s, lens, order, F, prefix);
    return hipGetLastError();
}

hipError_t launch_partition(const Geometry &g, const RankDesc *ranks, int32_t rank_lo,
                            int32_t nr, const int64_t *prefix, int64_t F, int64_t *seg_off,
                            int32_t *seg_file, int64_t *seg_lo, int64_t *seg_hi,
                            int64_t seg_cap, int32_t *err, hipStream_t s) {
    if (nr <= 0) return hipSuccess;
    const int blocks = (int)cdiv(nr, 256);
    hipLaunchKernelGGL(k_part_count, dim3(blocks), dim3(256), 0, s, g, ranks, rank_lo, nr, prefix, F, seg_off);
    hipLaunchKernelGGL(k_excl_scan_inplace, dim3(1), dim3(1024), 0, s, seg_off, (int64_t)nr);
    if (seg_cap > 0)
        hipLaunchKernelGGL(k_part_emit, dim3(blocks), dim3(256), 0, s, g, ranks, rank_lo, nr, prefix, F,
                           (const int64_t *)seg_off, seg_file, seg_lo, seg_hi, seg_cap, err);
    return hipGetLastError();
}

static inline int grid_for(int64_t n, int bs) {
    int64_t b = cdiv(n, bs);
    if (b > 8192) b = 8192;
    if (b < 1) b = 1;
    return (int)b;
}

hipError_t launch_map(const int64_t *prefix, int64_t F, const int64_t *ids, int64_t n,
                      int32_t *fpos, int64_t *off, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_map, dim3(grid_for(n, 256)), dim3(256), 0, s, prefix, F, ids, n, fpos, off);
    return hipGetLastError();
}

hipError_t launch_digest(const int64_t *ids, int64_t n, uint64_t *acc, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_digest, dim3(grid_for(n, 256)), dim3(256), 0, s, ids, n, acc);
    return hipGetLastError();
}

hipError_t launch_digest_range(int64_t lo, int64_t hi, uint64_t *acc, hipStream_t s) {
    if (hi <= lo) return hipSuccess;
    hipLaunchKernelGGL(k_digest_range, dim3(grid_for(hi - lo, 256)), dim3(256), 0, s, lo, hi, acc);
    return hipGetLastError();
}

hipError_t launch_debug_wave_scan(const uint64_t *in, uint64_t *out, int64_t n, hipStream_t s) {
    hipLaunchKernelGGL(k_debug_wave_scan, dim3(cdiv(n, 256)), dim3(256), 0, s, in, out, n);
    return hipGetLastError();
}

template <int EPT>
static void launch_v1_ept(const Geometry &g, const RankDesc *ranks, int32_t rank_lo, int32_t nr,
                          int64_t w_lo, int64_t nw, int64_t pos_lo, int64_t count, int64_t *out,
                          hipStream_t s) {
    hipLaunchKernelGGL(k_v1_lds<EPT>, dim3((uint32_t)(nr * nw)), dim3(256), sort_lds_bytes<EPT>(), s,
                       g, ranks, rank_lo, w_lo, nw, pos_lo, count, out);
}

size_t v1_workspace_bytes(const Geometry &, int32_t, int64_t, int64_t) { return 0; }

hipError_t launch_v1(const Geometry &g, const RankDesc *ranks, int32_t rank_lo, int32_t nr,
                     int64_t pos_lo, int64_t count, int64_t *out, uint32_t *, int32_t *,
                     hipStream_t s, const Marker &mk) {
    int64_t pos_hi = pos_lo + count < g.ns ? pos_lo + count : g.ns;
    if (nr <= 0 || pos_hi <= pos_lo) return hipSuccess;
    const int64_t w_lo = pos_lo / g.B, w_hi = (pos_hi - 1) / g.B;
    const int64_t nw = w_hi - w_lo + 1;
    const int64_t nmax = g.B < g.ns ? g.B : g.ns;
    if (nmax > kLdsSortMax) return hipErrorNotSupported;   // HBM multi-pass: see launch_v1_big
    mk(K_V1, s);
    if (nmax <= 1024) launch_v1_ept<4>(g, ranks, rank_lo, nr, w_lo, nw, pos_lo, count, out, s);
    else if (nmax <= 4096) launch_v1_ept<16>(g, ranks, rank_lo, nr, w_lo, nw, pos_lo, count, out, s);
    else if (nmax <= 8192) launch_v1_ept<32>(g, ranks, rank_lo, nr, w_lo, nw, pos_lo, count, out, s);
    else launch_v1_ept<64>(g, ranks, rank_lo, nr, w_lo, nw, pos_lo, count, out, s);
    mk(-1, s);
    return hipGetLastError();
}

size_t v2_val_bytes(const Geometry &g, int32_t nr) {
    const V2Plan p = v2_plan(g);
    return (size_t)nr * (size_t)p.G * (size_t)p.P1 * sizeof(uint32_t);
}
size_t v2_buf_bytes(const Geometry &, int32_t) { return 0; }
size_t v2_sort_bytes(const Geometry &, int32_t) { return 0; }

template <int EPT>
static void launch_tail_ept(const Geometry &g, const V2Plan &pl, const RankDesc *ranks,
                            int32_t rank_lo, int32_t nr, const uint32_t *VAL, int64_t pos_lo,
                            int64_t count, int64_t *out, hipStream_t s) {
    hipLaunchKernelGGL(k_v2_tail<EPT>, dim3((uint32_t)nr), dim3(256), sort_lds_bytes<EPT>(), s,
                       g, pl, ranks, rank_lo, VAL, pos_lo, count, out);
}

hipError_t launch_v2(const Geometry &g, const RankDesc *ranks, int32_t rank_lo, int32_t nr,
                     int64_t pos_lo, int64_t count, int64_t *out, uint32_t *VAL, uint32_t *,
                     uint32_t *, int32_t *, hipStream_t s, const Marker &mk) {
    const V2Plan pl = v2_plan(g);
    int64_t pos_hi = pos_lo + count < g.ns ? pos_lo + count : g.ns;
    if (nr <= 0 || pos_hi <= pos_lo) return hipSuccess;
    if (pl.P1 > kLdsSlotMax || pl.P1 > kLdsSortMax) return hipErrorNotSupported;
    const int64_t nwin_max = pl.L / g.B + 2;
    const size_t lds_slot = (size_t)(pl.P1 + 4 * nwin_max) * sizeof(uint32_t) +
                            (size_t)((pl.P1 + 15) / 16 * 16);   // + collision-probe bytes
    const bool need_tail = pos_hi > pl.T;
    // tiles needed: pass A over [0, g_need), pass B over the tiles overlapping the range
    if (pl.G > 0) {
        const int64_t last_emit = pos_lo < pl.T ? ((pos_hi < pl.T ? pos_hi : pl.T) - 1) / pl.L : -1;
        const int64_t g_need = need_tail ? pl.G : last_emit + 1;
        if (g_need > 0) {
            mk(K_V2_LASTOCC, s);
            hipLaunchKernelGGL(k_v2_lastocc, dim3((uint32_t)(nr * g_need)), dim3(256), lds_slot, s,
                               g, pl, rank_lo, g_need, VAL);
        }
        // k_v2_lastocc indexes VAL by (rl*G + tile) with tile < g_need: consistent layout
        if (last_emit >= 0) {
            const int64_t g_lo = pos_lo / pl.L;
            const int64_t ng = last_emit - g_lo + 1;
            mk(K_V2_EMIT, s);
            hipLaunchKernelGGL(k_v2_emit, dim3((uint32_t)(nr * ng)), dim3(64), lds_slot, s,
                               g, pl, ranks, rank_lo, g_lo, ng, (const uint32_t *)VAL, pos_lo, count, out);
        }
    }
    if (need_tail) {
        mk(K_V2_TAIL, s);
        const int64_t P1 = pl.P1;
        if (P1 <= 1024) launch_tail_ept<4>(g, pl, ranks, rank_lo, nr, VAL, pos_lo, count, out, s);
        else if (P1 <= 4096) launch_tail_ept<16>(g, pl, ranks, rank_lo, nr, VAL, pos_lo, count, out, s);
        else if (P1 <= 8192) launch_tail_ept<32>(g, pl, ranks, rank_lo, nr, VAL, pos_lo, count, out, s);
        else launch_tail_ept<64>(g, pl, ranks, rank_lo, nr, VAL, pos_lo, count, out, s);
    }
    mk(-1, s);
    return hipGetLastError();
}

hipError_t init_kernel_attributes() {
    const int big = 160 * 1024;
    hipError_t e = hipSuccess;
#define PSS_ATTR(fn) { hipError_t x = hipFuncSetAttribute((const void *)(fn), hipFuncAttributeMaxDynamicSharedMemorySize, big); if (x != hipSuccess) e = x; }
    PSS_ATTR(k_v1_lds<32>);
    PSS_ATTR(k_v1_lds<64>);
    PSS_ATTR(k_v2_tail<32>);
    PSS_ATTR(k_v2_tail<64>);
    PSS_ATTR(k_v2_lastocc);
    PSS_ATTR(k_v2_emit);
#undef PSS_ATTR
    return e;
}

}  // namespace pss
