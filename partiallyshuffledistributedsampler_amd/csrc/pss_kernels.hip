// pss_kernels.hip -- gfx950 (MI355X / CDNA4) kernels of the partial-shuffle sampler:
// prologue (scan + partition), V1 generation, id -> (file, offset) map, coverage digest.
// V2 lives in pss_v2.hip (pools beyond LDS: pss_v2grp.hip), primitives in pss_device.h.
//
// The hot path of the reference (index generation, V1:157-172 / V2:96-116, and the id ->
// (file, offset) scan, V1:181-221) is restated as integer, HBM-write-bound kernels:
//
//   k_scan_partial/_final  exclusive scan of files_len over the shuffled file order (wave64 DPP)
//   k_part_*           balanced file -> rank partition (segments of each rank's id block)
//   k_v1_feistel       V1: each window's permutation is a keyed Feistel bijection, evaluated
//                      per position (random access, no sort; k_v1_keys: per-window round keys)
//   k_map, k_digest    id -> (file position, offset); coverage digest for the RCCL check
//
// Schedule definitions: DESIGN.md §3, restated on the CPU in oracle/pss_oracle.c
// (orc_v1_philox_stream / orc_v2_philox_stream); both must agree bit for bit.  No MFMA
// anywhere -- this is integer, memory/latency-bound work.
#include <cstdlib>

#include <type_traits>

#include "pss_device.h"
#include "pss_map.h"

namespace pss {

// ------------------------------------------------------------------------------------------
// scan + partition (V1:27-53,181-190 / V2:27-49,184-193)
// ------------------------------------------------------------------------------------------
// Two passes over chunks of 4096 files (256 threads x 16, coalesced order reads):
// k_scan_partial sums each chunk; k_scan_final adds the sums of the chunks before its own and
// scans its chunk with 16 workgroup DPP scans.  One chunk (F <= 4096) skips the first pass.
constexpr int kScanChunk = 4096;

__device__ __forceinline__ uint64_t block_sum256(uint64_t x, uint64_t *tot) {
    uint64_t total;
    (void)block_excl_scan<256>(x, tot, total);
    return total;
}

__global__ __launch_bounds__(256) void k_scan_partial(const int64_t *__restrict__ lens,
                                                      const int32_t *__restrict__ order,
                                                      int64_t F, uint64_t *__restrict__ part) {
    __shared__ uint64_t tot[4];
    const int64_t base = (int64_t)blockIdx.x * kScanChunk;
    uint64_t s = 0;
#pragma unroll
    for (int j = 0; j < kScanChunk / 256; j++) {
        const int64_t f = base + j * 256 + threadIdx.x;
        if (f < F) s += (uint64_t)lens[order[f]];
    }
    const uint64_t total = block_sum256(s, tot);
    if (threadIdx.x == 0) part[blockIdx.x] = total;
}

__global__ __launch_bounds__(256) void k_scan_final(const int64_t *__restrict__ lens,
                                                    const int32_t *__restrict__ order, int64_t F,
                                                    const uint64_t *__restrict__ part,
                                                    int64_t *__restrict__ prefix) {
    __shared__ uint64_t tot[4];
    const int64_t c = blockIdx.x;
    const int64_t base = c * kScanChunk;
    uint64_t x[kScanChunk / 256];
#pragma unroll
    for (int j = 0; j < kScanChunk / 256; j++) {       // all 16 gathers in flight
        const int64_t f = base + j * 256 + threadIdx.x;
        x[j] = f < F ? (uint64_t)lens[order[f]] : 0;
    }
    uint64_t cs = 0;
    for (int64_t i = threadIdx.x; i < c; i += 256) cs += part[i];
    uint64_t carry = block_sum256(cs, tot);
#pragma unroll
    for (int j = 0; j < kScanChunk / 256; j++) {
        const int64_t f = base + j * 256 + threadIdx.x;
        uint64_t total;
        const uint64_t ex = block_excl_scan<256>(x[j], tot, total);
        if (f < F) prefix[f] = (int64_t)(carry + ex);
        carry += total;
    }
    if (c == gridDim.x - 1 && threadIdx.x == 0) prefix[F] = (int64_t)carry;
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
__global__ void k_bucket_index(const int64_t *__restrict__ prefix, int64_t F, int32_t kb, int64_t nb,
                               int32_t *__restrict__ BT) {
    for (int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; b < nb;
         b += (int64_t)gridDim.x * blockDim.x)
        BT[b] = (int32_t)file_of(prefix, F, b << kb);
}

constexpr int kMapIlp = 4;

template <typename OFF>
__global__ __launch_bounds__(256) void k_map(const int64_t *__restrict__ prefix, int64_t F,
                                             const int32_t *__restrict__ BT, int32_t kb, int64_t nb,
                                             const int64_t *__restrict__ ids, int64_t n,
                                             int32_t *__restrict__ fpos, OFF *__restrict__ off) {
    // each id is a chain of dependent L2 reads (bucket bounds, then the prefix): a thread runs
    // kMapIlp ids a grid-stride apart, coalesced and with their chains interleaved
    const int64_t T = prefix[F];
    const int64_t S = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i0 < n; i0 += kMapIlp * S) {
        int64_t id[kMapIlp];
#pragma unroll
        for (int k = 0; k < kMapIlp; k++) id[k] = i0 + k * S < n ? ids[i0 + k * S] : 0;
        int32_t f[kMapIlp];
        int64_t o[kMapIlp];
#pragma unroll
        for (int k = 0; k < kMapIlp; k++) map_one_bucketed_t(prefix, F, T, BT, kb, nb, id[k], f[k], o[k]);
#pragma unroll
        for (int k = 0; k < kMapIlp; k++)
            if (i0 + k * S < n) { fpos[i0 + k * S] = f[k]; off[i0 + k * S] = (OFF)o[k]; }
    }
}

// Rows of device-resident files: out[i] = data[base[order[f_i]] + off_i] (row_bytes each), the
// on-GPU form of the reference's per-file fancy-index gather (V1:243-248).  `base` gives each
// file's first row in the data tensor, files in dataset order; reflected ids (f < 0) read
// file -1 - f.  One 16-, 4- or 1-byte word per thread.
template <typename W>
__global__ void k_gather(const W *__restrict__ data, int64_t row_words, const int64_t *__restrict__ base,
                         const int32_t *__restrict__ order, const int32_t *__restrict__ fpos,
                         const int32_t *__restrict__ off, int64_t n, W *__restrict__ out) {
    const int64_t total = n * row_words;
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < total;
         k += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = k / row_words, w = k - i * row_words;
        const int32_t f = fpos[i] < 0 ? -1 - fpos[i] : fpos[i];
        const int64_t row = base[order[f]] + off[i];
        out[k] = data[row * row_words + w];
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
// V1 (V1:157-172): window w of rank r -> ids start + w*B + perm_w[p], wrap at N, where perm_w
// is the keyed Feistel bijection of [0, len_w) under round_keys8(w, rank, DOM_V1_WIN).  Random
// access, no sort: every position is computed independently, so the kernel is a pure
// compute + coalesced-store stream (the sort-based kernel it replaces spent its time in Philox
// sort keys and LDS bucket passes).
// ------------------------------------------------------------------------------------------
// mc != nullptr (the mapped one-shot kernel): also each (rank, window)'s map segments
// (window_map_segments) as kV1MapWords words -- f0, f1, f2, d0, -s1, -s2, s1, s2; f0 = -1: the
// window has none (it wraps at N, reaches past the scanned total or crosses three boundaries)
constexpr int kV1MapWords = 8;
__global__ __launch_bounds__(256) void k_v1_keys(Geometry g, int32_t rank_lo, int64_t w_lo,
                                                 int64_t nw, uint32_t *__restrict__ kt,
                                                 uint32_t *__restrict__ mc, MapArgs ma,
                                                 const RankDesc *__restrict__ ranks, RankArgs ra, int use_ra) {
    const int32_t rl = (int32_t)blockIdx.y;
    const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (j >= nw) return;
    uint32_t k[kRoundKeyWords];
    round_keys8(g.key0, g.key1, (uint32_t)(w_lo + j), (uint32_t)(rank_lo + rl), DOM_V1_WIN, k);
    uint32_t *b = kt + ((int64_t)rl * nw + j) * kRoundKeyWords;
#pragma unroll
    for (int i = 0; i < kRoundKeyWords; i++) b[i] = k[i];
    if (!mc) return;
    uint32_t c[kV1MapWords] = {kNone, 0u, 0u, 0u, 0u, 0u, kNone, kNone};
    const int64_t wB = (w_lo + j) * g.B;
    const int64_t len = g.ns - wB < g.B ? g.ns - wB : g.B;
    int64_t a = (use_ra ? ra.r[rl].new_start : ranks[rank_lo + rl].new_start) + wB;
    if (a >= g.N) a -= g.N;
    int32_t f[3];
    uint32_t d0, sg[2];
    if (a + len <= g.N && window_map_segments(ma, a, len, f, d0, sg)) {
        c[0] = (uint32_t)f[0]; c[1] = (uint32_t)f[1]; c[2] = (uint32_t)f[2];
        c[3] = d0; c[4] = 0u - sg[0]; c[5] = 0u - sg[1]; c[6] = sg[0]; c[7] = sg[1];
    }
    uint32_t *m = mc + ((int64_t)rl * nw + j) * kV1MapWords;
#pragma unroll
    for (int i = 0; i < kV1MapWords; i++) m[i] = c[i];
}

struct V1Plan {
    int64_t sb_lo, nsb;        // 256-position super-blocks [sb_lo, sb_lo + nsb) of each rank
    int64_t per_wave;          // super-blocks per wave
    int64_t w_lo, nw;          // windows of the key table
    uint32_t B, hB, walk_full, fast_ok;
    uint32_t pairs;            // fast super-blocks in the 16-B pair layout (on; 8-B stores measured slower)
};

// One wave per (rank, run of per_wave super-blocks).  Lane l computes positions p0 + 64 j + l,
// j < 4, of each 256-position super-block p0.  MAPPED: instead of the int64 id, the id's
// (int32 file position, int32 offset) through the epoch's bucket index (MapArgs) -- the fused
// form of pss_map, same 8 bytes per position.
template <bool PACKED, bool MAPPED>
__global__ __launch_bounds__(64) void k_v1_feistel(Geometry g, V1Plan vp, const RankDesc *__restrict__ ranks,
                                                   int32_t rank_lo, const uint32_t *__restrict__ kt,
                                                   int64_t pos_lo, int64_t count,
                                                   int64_t *__restrict__ out, MapArgs ma) {
    extern __shared__ uint32_t v1_pad[];   // occupancy limiter only (8 waves per CU)
    if (vp.nsb < 0) v1_pad[threadIdx.x] = 0;
    const int lane = threadIdx.x;
    const int64_t waves_per_rank = (vp.nsb + vp.per_wave - 1) / vp.per_wave;
    const int32_t rl = (int32_t)(blockIdx.x / waves_per_rank);
    const int64_t sb0 = vp.sb_lo + (int64_t)(blockIdx.x % waves_per_rank) * vp.per_wave;
    const int64_t sb1 = sb0 + vp.per_wave < vp.sb_lo + vp.nsb ? sb0 + vp.per_wave : vp.sb_lo + vp.nsb;
    const int64_t start = ranks[rank_lo + rl].new_start;
    const int64_t pos_hi = pos_lo + count < g.ns ? pos_lo + count : g.ns;
    int64_t *o = out + (int64_t)rl * count - pos_lo;
    int32_t *ofp = ma.fpos + (int64_t)rl * count - pos_lo;
    int32_t *ooff = ma.off + (int64_t)rl * count - pos_lo;
    auto put = [&](int64_t p, int64_t id) __attribute__((always_inline)) {
        if constexpr (MAPPED) {
            int32_t f, of;
            map_id_fast(ma, id, f, of);
            ofp[p] = f;
            ooff[p] = of;
        } else {
            o[p] = id;
        }
    };
    const uint32_t *ktr = kt + (int64_t)rl * vp.nw * kRoundKeyWords;
    const int64_t B = vp.B;
    // one super-block through the general path (range edges, short or cycle-walking windows)
    auto slow_sb = [&](int64_t sb) __attribute__((always_inline)) {
        const int64_t p0 = sb * 256;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int64_t p = p0 + 64 * j + lane;
            if (p < pos_lo || p >= pos_hi) continue;
            int64_t y = p;
            if (g.shuffle) {
                const int64_t wp = p / B;
                const int64_t len = g.ns - wp * B < B ? g.ns - wp * B : B;
                const uint32_t *kw = ktr + (wp - vp.w_lo) * kRoundKeyWords;
                uint32_t kk[kFeistelRounds];
#pragma unroll
                for (int i = 0; i < kFeistelRounds; i++) kk[i] = kw[i];
                y = wp * B + feistel((uint32_t)(p - wp * B), (uint32_t)len,
                                     feistel_half_bits((uint32_t)len), kk);
            }
            put(p, wrap_id(start + y, g.N));
        }
    };
    // wave-uniform layout choices: the 16-B pair stores need the rank's output 16-B aligned
    // (super-blocks start at multiples of 2 KB), the 32-bit ids N + ns < 2^32
    const bool pair = __builtin_amdgcn_readfirstlane(
        vp.pairs && (MAPPED ? (((uintptr_t)(ofp + sb0 * 256) | (uintptr_t)(ooff + sb0 * 256)) & 7u) == 0
                            : ((uintptr_t)(o + sb0 * 256) & 15u) == 0));
    const bool narrow = g.N + g.ns < (int64_t)UINT32_MAX;
    int64_t sb = sb0;
    while (sb < sb1) {
        if (!vp.fast_ok) { slow_sb(sb++); continue; }
        // the wave's super-blocks inside window w (B % 256 == 0: super-blocks never straddle
        // windows): one division and one key load per window, not per super-block
        const int64_t w = (sb * 256) / B;
        const int64_t wB = w * B;
        const int64_t sb_w_end = (wB + B) / 256 < sb1 ? (wB + B) / 256 : sb1;
        if (wB + B > g.ns) {   // the short last window: cycle walking
            for (; sb < sb_w_end; sb++) slow_sb(sb);
            continue;
        }
        if (sb * 256 < pos_lo || sb * 256 + 256 > pos_hi) { slow_sb(sb++); continue; }   // range edges
        // whole super-blocks of the range from here to the window's end
        const int64_t sb_full_end = pos_hi / 256 < sb_w_end ? pos_hi / 256 : sb_w_end;
        const uint32_t *kw = ktr + (w - vp.w_lo) * kRoundKeyWords;
        const int64_t base = start + wB;
        uint32_t kp[kFeistelRounds];
#pragma unroll
        for (int i = 0; i < kFeistelRounds; i++) {
            const uint32_t k = __builtin_amdgcn_readfirstlane(kw[i]);
            kp[i] = PACKED ? (k & 0xFFFFu) * 0x10001u : k;
        }
        // the window's whole super-blocks; PAIR / NARROW are fixed per wave, so each combination
        // is its own loop (no per-super-block branches, nothing hoisted across them)
        auto run = [&](auto pair_c, auto narrow_c) __attribute__((always_inline)) {
            constexpr bool PAIR = decltype(pair_c)::value, NARROW = decltype(narrow_c)::value;
            // narrow: every id start + p < N + ns < 2^32 wraps with one 32-bit subtract and an
            // unsigned min (id - N underflows exactly when id < N)
            auto wrap = [&](uint32_t y) -> int64_t {
                if constexpr (NARROW) {
                    const uint32_t id = (uint32_t)base + y;
                    return (int64_t)__builtin_elementwise_min(id, id - (uint32_t)g.N);
                } else {
                    return wrap_id(base + y, g.N);
                }
            };
            const uint32_t l2 = 2u * (uint32_t)lane;
            for (; sb < sb_full_end; sb++) {
                const int64_t p0 = sb * 256;
                // whole super-block inside one full window of 4^hB elements: no cycle walking.
                // Pair layout (16-B aligned output): lane l owns positions p0 + 2l, 2l + 1 and
                // p0 + 128 + 2l, 2l + 1, written by two 16-byte stores (8-byte pairs when
                // mapped) instead of four 8-byte ones.
                const uint32_t x0 = (uint32_t)(p0 - wB);
                uint32_t x[4], y[4];
                if constexpr (PAIR) { x[0] = x0 + l2; x[1] = x0 + l2 + 1u; x[2] = x0 + 128u + l2; x[3] = x0 + 129u + l2; }
                else { x[0] = x0 + lane; x[1] = x0 + 64u + lane; x[2] = x0 + 128u + lane; x[3] = x0 + 192u + lane; }
                if constexpr (PACKED) {
                    feistel4_pk16(x, vp.hB, kp, y);
                } else {
#pragma unroll
                    for (int j = 0; j < 4; j++) y[j] = feistel_once(x[j], vp.hB, kp);
                }
                if constexpr (PAIR) {
#pragma unroll
                    for (int h = 0; h < 2; h++) {
                        const int64_t p = p0 + 128 * h + l2;
                        const int64_t ia = wrap(y[2 * h]), ib = wrap(y[2 * h + 1]);
                        if constexpr (MAPPED) {
                            int32_t fa, fb, oa, ob;
                            map_id_fast(ma, ia, fa, oa);
                            map_id_fast(ma, ib, fb, ob);
                            *(int2 *)(ofp + p) = make_int2(fa, fb);
                            *(int2 *)(ooff + p) = make_int2(oa, ob);
                        } else {
                            longlong2 v;
                            v.x = ia;
                            v.y = ib;
                            *(longlong2 *)(o + p) = v;
                        }
                    }
                } else {
#pragma unroll
                    for (int j = 0; j < 4; j++) put(p0 + 64 * j + lane, wrap(y[j]));
                }
            }
        };
        if (pair && narrow) run(std::true_type{}, std::true_type{});
        else if (pair) run(std::true_type{}, std::false_type{});
        else if (narrow) run(std::false_type{}, std::true_type{});
        else run(std::false_type{}, std::false_type{});
    }
}

// One-shot V1 (unmapped ids): a grid of short-lived 256-thread workgroups, each 1024
// consecutive positions of one rank -- 4 per lane, written as two 16-byte stores (the store
// pattern of torch's fill_, which MI355X writes at 6.2-6.9 TB/s against 5.2-5.3 TB/s for waves
// that loop over their own runs, tools/ubench_store2.hip).  Fast workgroups (inside one full
// window that needs no cycle walking, inside the position range, 16-B aligned output) take the
// packed Feistel on the window's SGPR keys; the others the per-position general path.  C2 V1:
// 168 -> 150 us per epoch against the persistent k_v1_feistel, which now serves the mapped
// hand-off only (same box, profiles/r04/ab_v1_oneshot/).
#ifndef PSS_V1OS_PER
#define PSS_V1OS_PER 4
#endif
#ifndef PSS_V1OS_ITERS
#define PSS_V1OS_ITERS 2
#endif
constexpr int kV1OsPer = PSS_V1OS_PER;             // positions per lane (2, 4 or 8) per iteration
static_assert(kV1OsPer == 2 || kV1OsPer == 4 || kV1OsPer == 8, "one or more 16-byte pair stores per lane");
constexpr int kV1OsIters = PSS_V1OS_ITERS;         // iterations per workgroup (one prologue):
                                                   // 2 against 1: C2 V1 639-656 vs 637-641 G idx/s,
                                                   // 4: 601-612 (profiles/r04/ab_v1os_iters/)
constexpr int64_t kV1OsPos = 256 * kV1OsPer;       // positions per iteration
constexpr int64_t kV1OsSpan = kV1OsPos * kV1OsIters;   // positions per workgroup
struct V1OsPlan {
    int64_t blk_lo;            // first 1024-position block of each rank
    uint32_t bpr;              // blocks per rank
    uint32_t b_log;            // B = 2^b_log when b_pow2
    int64_t w_lo, nw;          // windows of the key table
    uint32_t B, hB, fast_ok, b_pow2;
};

// MAPPED (pss_generate_mapped): (int32 file position, int32 offset) into ma.fpos / ma.off --
// on fast workgroups from the window's map segments (mc, k_v1_keys: two compares and selects
// per position, 16-byte stores of 4 file positions and 4 offsets), elsewhere through the global
// bucketed map
template <bool PACKED, bool NARROW, bool MAPPED = false>
__global__ __launch_bounds__(256) void k_v1_os(Geometry g, V1OsPlan vp, const RankDesc *__restrict__ ranks,
                                               int32_t rank_lo, const uint32_t *__restrict__ kt,
                                               int64_t pos_lo, int64_t count, int64_t *__restrict__ out,
                                               RankArgs ra, int use_ra, MapArgs ma,
                                               const uint32_t *__restrict__ mc) {
    const uint32_t rl = blockIdx.x / vp.bpr;
    const int64_t p0 = (vp.blk_lo + (int64_t)(blockIdx.x - rl * vp.bpr)) * kV1OsSpan;
    const int64_t pos_hi = pos_lo + count < g.ns ? pos_lo + count : g.ns;
    // (use_ra: the rank's descriptor from the kernel arguments, no upload kernel ahead)
    const int64_t start = use_ra ? ra.r[rl].new_start : ranks[rank_lo + (int32_t)rl].new_start;
    int64_t *o = out + (int64_t)rl * count - pos_lo;
    int32_t *ofp = ma.fpos + (int64_t)rl * count - pos_lo;
    int32_t *ooff = ma.off + (int64_t)rl * count - pos_lo;
    const uint32_t *ktr = kt + (int64_t)rl * vp.nw * kRoundKeyWords;
    const int64_t B = vp.B;
    const int64_t w = vp.b_pow2 ? (p0 >> vp.b_log) : p0 / B;
    const int64_t wB = w * B;
    uint32_t mcw[kV1MapWords];   // MAPPED: the window's map segments (wave-uniform)
    bool aligned;
    if constexpr (MAPPED) {
        static_assert(!MAPPED || kV1OsPer % 4 == 0, "mapped stores: 4 positions per 16-byte store");
        const bool inw = vp.fast_ok && w >= vp.w_lo && w < vp.w_lo + vp.nw;
        const uint32_t *m = mc + ((int64_t)rl * vp.nw + (inw ? w - vp.w_lo : 0)) * kV1MapWords;
#pragma unroll
        for (int i = 0; i < kV1MapWords; i++) mcw[i] = kNone;
        if (inw) {
#pragma unroll
            for (int i = 0; i < kV1MapWords; i++) mcw[i] = __builtin_amdgcn_readfirstlane(m[i]);
        }
        aligned = mcw[0] != kNone && ((((uintptr_t)(ofp + p0)) | ((uintptr_t)(ooff + p0))) & 15u) == 0;
    } else {
        aligned = (((uintptr_t)(o + p0)) & 15u) == 0;
    }
    const bool fast = vp.fast_ok && wB + B <= g.ns && p0 + kV1OsSpan <= wB + B && p0 >= pos_lo &&
                      p0 + kV1OsSpan <= pos_hi && aligned;
    const uint32_t l4 = (uint32_t)kV1OsPer * threadIdx.x;
    if (fast) {
        uint32_t kp[kFeistelRounds];
#ifdef PSS_V1OS_INKEYS   // the window's keys computed here (wave-uniform) instead of the key table
        uint32_t kr[8];
        round_keys8(g.key0, g.key1, (uint32_t)w, (uint32_t)(rank_lo + (int32_t)rl), DOM_V1_WIN, kr);
#pragma unroll
        for (int i = 0; i < kFeistelRounds; i++) {
            const uint32_t k = __builtin_amdgcn_readfirstlane(kr[i]);
            kp[i] = PACKED ? (k & 0xFFFFu) * 0x10001u : k;
        }
#else
        const uint32_t *kw = ktr + (w - vp.w_lo) * kRoundKeyWords;
#pragma unroll
        for (int i = 0; i < kFeistelRounds; i++) {
            const uint32_t k = __builtin_amdgcn_readfirstlane(kw[i]);
            kp[i] = PACKED ? (k & 0xFFFFu) * 0x10001u : k;
        }
#endif
        const int64_t base = start + wB;
#pragma unroll
        for (int it = 0; it < kV1OsIters; it++) {
        const uint32_t x0 = (uint32_t)(p0 - wB) + (uint32_t)(it * kV1OsPos) + l4;
        uint32_t x[kV1OsPer], y[kV1OsPer];
#pragma unroll
        for (int j = 0; j < kV1OsPer; j++) x[j] = x0 + (uint32_t)j;
        if constexpr (PACKED && kV1OsPer == 2) {
            feistel2_pk16(x[0], x[1], vp.hB, kp, y[0], y[1]);
        } else if constexpr (PACKED) {
#pragma unroll
            for (int j = 0; j < kV1OsPer; j += 4) feistel4_pk16(x + j, vp.hB, kp, y + j);
        } else {
#pragma unroll
            for (int j = 0; j < kV1OsPer; j++) y[j] = feistel_once(x[j], vp.hB, kp);
        }
        if constexpr (MAPPED) {
            // y -> (f_k, y + d_k) on segment k of the window's ids (window_map_segments)
            uint32_t fv[kV1OsPer], ov[kV1OsPer];
#pragma unroll
            for (int j = 0; j < kV1OsPer; j++) {
                const bool a1 = y[j] >= mcw[6], a2 = y[j] >= mcw[7];
                fv[j] = a2 ? mcw[2] : (a1 ? mcw[1] : mcw[0]);
                ov[j] = y[j] + (a2 ? mcw[5] : (a1 ? mcw[4] : mcw[3]));
            }
            const int64_t e = p0 + it * kV1OsPos + l4;
#pragma unroll
            for (int j = 0; j < kV1OsPer; j += 4) {
                *(uint4 *)(ofp + e + j) = make_uint4(fv[j], fv[j + 1], fv[j + 2], fv[j + 3]);
                *(uint4 *)(ooff + e + j) = make_uint4(ov[j], ov[j + 1], ov[j + 2], ov[j + 3]);
            }
            continue;
        }
        int64_t id[kV1OsPer];
#pragma unroll
        for (int j = 0; j < kV1OsPer; j++) {
            if constexpr (NARROW) {
                const uint32_t v = (uint32_t)base + y[j];
                id[j] = (int64_t)__builtin_elementwise_min(v, v - (uint32_t)g.N);
            } else {
                id[j] = wrap_id(base + y[j], g.N);
            }
        }
#pragma unroll
        for (int j = 0; j < kV1OsPer; j += 2) {
            longlong2 a;
            a.x = id[j]; a.y = id[j + 1];
            *(longlong2 *)(o + p0 + it * kV1OsPos + l4 + j) = a;
        }
        }
        return;
    }
#pragma unroll
    for (int q = 0; q < kV1OsPer * kV1OsIters; q++) {
        const int j = q % kV1OsPer;
        const int64_t p = p0 + (q / kV1OsPer) * kV1OsPos + l4 + j;
        if (p < pos_lo || p >= pos_hi) continue;
        int64_t y = p;
        if (g.shuffle) {
            const int64_t wp = p / B;
            const int64_t len = g.ns - wp * B < B ? g.ns - wp * B : B;
            uint32_t kk[8];
#ifdef PSS_V1OS_INKEYS
            round_keys8(g.key0, g.key1, (uint32_t)wp, (uint32_t)(rank_lo + (int32_t)rl), DOM_V1_WIN, kk);
#else
            const uint32_t *kw = ktr + (wp - vp.w_lo) * kRoundKeyWords;
#pragma unroll
            for (int i = 0; i < kFeistelRounds; i++) kk[i] = kw[i];
#endif
            y = wp * B + feistel((uint32_t)(p - wp * B), (uint32_t)len, feistel_half_bits((uint32_t)len), kk);
        }
        if constexpr (MAPPED) {
            int32_t f, of;
            map_id_fast(ma, wrap_id(start + y, g.N), f, of);
            ofp[p] = f;
            ooff[p] = of;
        } else {
            o[p] = wrap_id(start + y, g.N);
        }
    }
}

// ------------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------------
static inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

__global__ __launch_bounds__(kArgRanks) void k_put_ranks(RankArgs a, int32_t n, RankDesc *dst) {
    if ((int32_t)threadIdx.x < n) dst[threadIdx.x] = a.r[threadIdx.x];
}

// Host -> device upload by a kernel reading pinned host memory (mapped into the device's address
// space), in place of hipMemcpyAsync: on the epoch path the runtime's async copy of the 40 KB file
// order once blocked the calling thread for 7-8 ms (the 8th upload of a process, every run; the
// other uploads 2 us, HIP API trace in profiles/r06/).  16-byte loads when both ends allow.
__global__ __launch_bounds__(256) void k_upload(const uint32_t *__restrict__ src, uint32_t *__restrict__ dst,
                                                int64_t nwords) {
    const int64_t stride = (int64_t)gridDim.x * 256;
    int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if ((((uintptr_t)src | (uintptr_t)dst) & 15u) == 0) {
        const int64_t n4 = nwords / 4;
        for (int64_t q = i; q < n4; q += stride) ((uint4 *)dst)[q] = ((const uint4 *)src)[q];
        for (int64_t k = n4 * 4 + i; k < nwords; k += stride) dst[k] = src[k];
    } else {
        for (int64_t k = i; k < nwords; k += stride) dst[k] = src[k];
    }
}

hipError_t launch_upload(const void *host_pinned, void *dst, size_t bytes, hipStream_t s) {
    if (bytes == 0) return hipSuccess;
    if (bytes % 4) return hipErrorInvalidValue;
    void *src = nullptr;
    hipError_t e = hipHostGetDevicePointer(&src, const_cast<void *>(host_pinned), 0);
    if (e != hipSuccess) return e;
    const int64_t nwords = (int64_t)(bytes / 4);
    const int64_t blocks = (nwords / 4 + 255) / 256;
    hipLaunchKernelGGL(k_upload, dim3((uint32_t)(blocks < 1 ? 1 : (blocks > 1024 ? 1024 : blocks))), dim3(256), 0, s,
                       (const uint32_t *)src, (uint32_t *)dst, nwords);
    return hipGetLastError();
}

hipError_t launch_put_ranks(const RankDesc *host, int32_t R, RankDesc *dst, hipStream_t s) {
    for (int32_t r0 = 0; r0 < R; r0 += kArgRanks) {
        RankArgs a;
        const int32_t n = R - r0 < kArgRanks ? R - r0 : kArgRanks;
        for (int32_t i = 0; i < n; i++) a.r[i] = host[r0 + i];
        hipLaunchKernelGGL(k_put_ranks, dim3(1), dim3(kArgRanks), 0, s, a, n, dst + r0);
    }
    return hipGetLastError();
}

size_t scan_scratch_words(int64_t F) { return (size_t)cdiv(F > 0 ? F : 1, kScanChunk); }

hipError_t launch_scan_prefix(const int64_t *lens, const int32_t *order, int64_t F,
                              int64_t *prefix, uint64_t *scratch, hipStream_t s) {
    const int64_t nc = cdiv(F > 0 ? F : 1, kScanChunk);
    if (nc > 1)
        hipLaunchKernelGGL(k_scan_partial, dim3((uint32_t)nc), dim3(256), 0, s, lens, order, F, scratch);
    hipLaunchKernelGGL(k_scan_final, dim3((uint32_t)nc), dim3(256), 0, s, lens, order, F,
                       (const uint64_t *)scratch, prefix);
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

hipError_t launch_bucket_index(const int64_t *prefix, int64_t F, int32_t kb, int64_t nb, int32_t *BT,
                               hipStream_t s) {
    hipLaunchKernelGGL(k_bucket_index, dim3(grid_for(nb, 256)), dim3(256), 0, s, prefix, F, kb, nb, BT);
    return hipGetLastError();
}

hipError_t launch_map(const int64_t *prefix, int64_t F, const int32_t *BT, int32_t kb, int64_t nb,
                      const int64_t *ids, int64_t n, int32_t *fpos, int64_t *off, int32_t *off32,
                      hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const dim3 grid(grid_for(cdiv(n, kMapIlp), 256));
    if (off32)
        hipLaunchKernelGGL(k_map<int32_t>, grid, dim3(256), 0, s, prefix, F, BT, kb, nb, ids, n, fpos, off32);
    else
        hipLaunchKernelGGL(k_map<int64_t>, grid, dim3(256), 0, s, prefix, F, BT, kb, nb, ids, n, fpos, off);
    return hipGetLastError();
}

hipError_t launch_gather(const void *data, int64_t row_bytes, const int64_t *base, const int32_t *order,
                         const int32_t *fpos, const int32_t *off, int64_t n, void *out, hipStream_t s) {
    if (n <= 0 || row_bytes <= 0) return hipSuccess;
    const bool a16 = row_bytes % 16 == 0 && ((uintptr_t)data % 16) == 0 && ((uintptr_t)out % 16) == 0;
    const bool a4 = row_bytes % 4 == 0 && ((uintptr_t)data % 4) == 0 && ((uintptr_t)out % 4) == 0;
    if (a16)
        hipLaunchKernelGGL(k_gather<uint4>, dim3(grid_for(n * (row_bytes / 16), 256)), dim3(256), 0, s,
                           (const uint4 *)data, row_bytes / 16, base, order, fpos, off, n, (uint4 *)out);
    else if (a4)
        hipLaunchKernelGGL(k_gather<uint32_t>, dim3(grid_for(n * (row_bytes / 4), 256)), dim3(256), 0, s,
                           (const uint32_t *)data, row_bytes / 4, base, order, fpos, off, n, (uint32_t *)out);
    else
        hipLaunchKernelGGL(k_gather<uint8_t>, dim3(grid_for(n * row_bytes, 256)), dim3(256), 0, s,
                           (const uint8_t *)data, row_bytes, base, order, fpos, off, n, (uint8_t *)out);
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

static int64_t gcus_v1() {
    static const int64_t n = [] {
        int dev = 0, c = 0;
        if (hipGetDevice(&dev) != hipSuccess) dev = 0;
        if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c <= 0) c = 256;
        return (int64_t)c;
    }();
    return n;
}

static bool v1_window_range(const Geometry &g, int64_t pos_lo, int64_t count, int64_t &w_lo,
                            int64_t &nw) {
    const int64_t pos_hi = pos_lo + count < g.ns ? pos_lo + count : g.ns;
    if (pos_hi <= pos_lo) return false;
    w_lo = pos_lo / g.B;
    nw = (pos_hi - 1) / g.B - w_lo + 1;
    return true;
}

// key table: kRoundKeyWords words per (local rank, window of the position range)
size_t v1_workspace_bytes(const Geometry &g, int32_t nr, int64_t pos_lo, int64_t count) {
    int64_t w_lo, nw;
    if (!g.shuffle || nr <= 0 || !v1_window_range(g, pos_lo, count, w_lo, nw)) return 0;
    // the round keys, then (a mapped launch) the windows' map segments
    return (size_t)nr * (size_t)nw * (kRoundKeyWords + kV1MapWords) * sizeof(uint32_t);
}

hipError_t launch_v1(const Geometry &g, const RankDesc *ranks, int32_t rank_lo, int32_t nr,
                     int64_t pos_lo, int64_t count, int64_t *out, uint32_t *key_ws,
                     hipStream_t s, const Marker &mk, const MapArgs *mapped, const RankArgs *rank_args) {
    int64_t w_lo, nw;
    if (nr <= 0 || !v1_window_range(g, pos_lo, count, w_lo, nw)) return hipSuccess;
    if (rank_args && nr > kArgRanks) return hipErrorInvalidValue;
    const int64_t pos_hi = pos_lo + count < g.ns ? pos_lo + count : g.ns;
    mk(K_V1, s);
    const MapArgs ma = mapped ? *mapped : MapArgs{};
    RankArgs ra;
    if (rank_args) ra = *rank_args;
    const int use_ra = rank_args ? 1 : 0;
    uint32_t *mc = mapped && key_ws ? key_ws + (size_t)nr * (size_t)nw * kRoundKeyWords : nullptr;
#ifdef PSS_V1OS_INKEYS
    if (g.shuffle && (mapped || (uint64_t)((pos_hi - 1) / kV1OsSpan - pos_lo / kV1OsSpan + 1) * (uint64_t)nr >= ((uint64_t)1 << 31)))
#else
    if (g.shuffle)
#endif
        hipLaunchKernelGGL(k_v1_keys, dim3((uint32_t)cdiv(nw, 256), (uint32_t)nr), dim3(256), 0, s,
                           g, rank_lo, w_lo, nw, key_ws, mc, ma, ranks, ra, use_ra);
    {
        V1OsPlan op{};
        op.blk_lo = pos_lo / kV1OsSpan;
        const int64_t bpr = (pos_hi - 1) / kV1OsSpan - op.blk_lo + 1;
        op.bpr = (uint32_t)bpr;
        op.w_lo = w_lo;
        op.nw = nw;
        op.B = (uint32_t)g.B;
        op.hB = feistel_half_bits(op.B);
        op.b_pow2 = (g.B & (g.B - 1)) == 0 ? 1u : 0u;
        op.b_log = (uint32_t)ceil_log2_u64((uint64_t)g.B);
        op.fast_ok = g.shuffle && op.B == (1u << (2 * op.hB)) && (g.B % kV1OsSpan) == 0;
        const bool narrow = g.N + g.ns < (int64_t)UINT32_MAX;
        const uint64_t blocks = (uint64_t)bpr * (uint64_t)nr;
        if (blocks < ((uint64_t)1 << 31)) {
            const dim3 grid((uint32_t)blocks);
#define PSS_V1OS(PK, NA) do { if (mapped) hipLaunchKernelGGL((k_v1_os<PK, NA, true>), grid, dim3(256), 0, s, g, op, ranks, \
                                                             rank_lo, (const uint32_t *)key_ws, pos_lo, count, out, ra, \
                                                             use_ra, ma, (const uint32_t *)mc); \
                              else hipLaunchKernelGGL((k_v1_os<PK, NA>), grid, dim3(256), 0, s, g, op, ranks, rank_lo, \
                                                      (const uint32_t *)key_ws, pos_lo, count, out, ra, use_ra, ma, \
                                                      (const uint32_t *)nullptr); } while (0)
            const bool pk = feistel_packed_ok(op.hB);
            if (pk && narrow) PSS_V1OS(true, true);
            else if (pk) PSS_V1OS(true, false);
            else if (narrow) PSS_V1OS(false, true);
            else PSS_V1OS(false, false);
#undef PSS_V1OS
            mk(-1, s);
            return hipGetLastError();
        }
    }
    if (rank_args) {   // the kernels below read the device table
        const hipError_t e = launch_put_ranks(rank_args->r, nr, const_cast<RankDesc *>(ranks) + rank_lo, s);
        if (e != hipSuccess) return e;
    }
    V1Plan vp{};
    vp.sb_lo = pos_lo / 256;
    vp.nsb = (pos_hi - 1) / 256 - vp.sb_lo + 1;
    vp.w_lo = w_lo;
    vp.nw = nw;
    vp.B = (uint32_t)g.B;
    vp.hB = feistel_half_bits(vp.B);
    vp.walk_full = vp.B != (1u << (2 * vp.hB));
    // fast super-blocks: inside one full window that needs no cycle walking
    vp.fast_ok = g.shuffle && !vp.walk_full && (g.B % 256) == 0;
    vp.pairs = 1;   // 16-byte pair stores on fast super-blocks
    // One round of waves: the stream is cut into exactly as many waves as the chip holds at 8
    // resident waves per CU (two per SIMD, an LDS claim caps it), each a run of consecutive
    // super-blocks.  A round-1/2 shape of 16 super-blocks per wave at full occupancy (3 rounds
    // of 8 waves per SIMD) stored at 4.3-4.6 TB/s (C2 V1: 184 us), one round of 2 per SIMD at
    // 4.6 (175 us): fewer stores in flight, no tail round.
    constexpr int64_t wpc = 8;
    // the mapped form reads the bucket index and the prefix for every id (dependent global
    // loads): it wants latency hiding, i.e. the full 32 waves per CU, where the plain form stores
    // best at one round of 8 (C2 V1 mapped: 0.55-0.63 ms at 8 per CU, round 2's 0.32-0.36 at
    // full occupancy)
    const int64_t wpc_run = mapped ? 32 : wpc;
    const int64_t slots_per_rank = wpc_run * gcus_v1() / nr;
    // (mapped: round 2's shape, runs of 16 super-blocks at full occupancy, several rounds)
    int64_t per = mapped ? 16 : cdiv(vp.nsb, slots_per_rank > 1 ? slots_per_rank : 1);
    if (per < 1) per = 1;
    vp.per_wave = per;
    const int64_t waves = (int64_t)nr * cdiv(vp.nsb, per);
    const size_t v1_lds = (size_t)(160 * 1024 / wpc_run - 64);   // caps the resident waves per CU
#define PSS_V1(PK, MP) hipLaunchKernelGGL((k_v1_feistel<PK, MP>), dim3((uint32_t)waves), dim3(64), v1_lds, s, g, vp, \
                                          ranks, rank_lo, (const uint32_t *)key_ws, pos_lo, count, out, ma)
    if (feistel_packed_ok(vp.hB) && mapped) PSS_V1(true, true);
    else if (feistel_packed_ok(vp.hB)) PSS_V1(true, false);
    else if (mapped) PSS_V1(false, true);
    else PSS_V1(false, false);
#undef PSS_V1
    mk(-1, s);
    return hipGetLastError();
}

hipError_t init_kernel_attributes() {
    hipError_t e = init_kernel_attributes_v2();
#define PSS_ATTR1(fn) { hipError_t x = hipFuncSetAttribute((const void *)(fn), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024); if (x != hipSuccess) e = x; }
    PSS_ATTR1((k_v1_feistel<true, true>));
    PSS_ATTR1((k_v1_feistel<true, false>));
    PSS_ATTR1((k_v1_feistel<false, true>));
    PSS_ATTR1((k_v1_feistel<false, false>));
#undef PSS_ATTR1
    return e;
}

}  // namespace pss
