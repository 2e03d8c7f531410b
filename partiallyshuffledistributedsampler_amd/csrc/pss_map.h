// pss_map.h -- id -> (file, offset) and rank -> file segment arithmetic (V1:181-221), shared
// by the gfx950 kernels (pss_kernels.hip) and the CPU mode (pss_cpu.cpp).
#pragma once
#include "pss_common.h"
#include "pss_kernels.h"

namespace pss {

// largest f in [0, F) with prefix[f] <= id  (the file holding id; empty files are skipped
// because an empty file shares its prefix with the next one)
PSS_HD int64_t file_of(const int64_t *prefix, int64_t F, int64_t id) {
    int64_t lo = 0, hi = F;
    while (hi - lo > 1) {
        const int64_t mid = (lo + hi) >> 1;
        if (prefix[mid] <= id) lo = mid; else hi = mid;
    }
    return lo;
}

// The id ranges a rank reads in one epoch, in stream order, wrapped at N and clipped to the
// scanned total T = prefix[F] (ids >= T are reflected, V1:191-196).
struct Ranges { int64_t lo[4], hi[4]; int n; };

PSS_HD void rank_ranges(const Geometry &g, const RankDesc &rd, int64_t T, Ranges &r) {
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
            const int64_t l = lo;
            if (h > T) h = T;
            if (l < h) { r.lo[r.n] = l; r.hi[r.n] = h; r.n++; }
            len -= take;
            lo = 0;
        }
    }
}

// one id -> (file position, offset); ids at or past the scanned total T = prefix[F] are
// reflected as V1:191-196 does and flagged by fpos = -1 - f
PSS_HD void map_one(const int64_t *prefix, int64_t F, int64_t id0, int32_t &fpos, int64_t &off) {
    const int64_t T = prefix[F];
    int64_t id = id0;
    bool refl = false;
    if (id >= T) {
        id = 2 * T - id;
        if (id == T) id = T - 1;
        refl = true;
    }
    if (id < 0) { fpos = INT32_MIN; off = id0; return; }
    const int64_t f = file_of(prefix, F, id);
    fpos = refl ? (int32_t)(-1 - f) : (int32_t)f;
    off = id - prefix[f];
}

// Bucket index of the epoch's prefix (pss_kernels.hip k_bucket_index): BT[b] = file_of(b << kb),
// one bucket per ~average file length, so an id's file is found between BT[b] and BT[b + 1]
// -- usually one or two probes instead of a binary search over all F files.
PSS_HD int32_t bucket_shift(int64_t total, int64_t F) {
    int64_t avg = F > 0 ? total / F : 1;
    int32_t kb = 0;
    while (((int64_t)2 << kb) <= avg && kb < 40) kb++;
    return kb;
}
PSS_HD int64_t bucket_count(int64_t total, int32_t kb) { return (total >> kb) + 2; }

// T = prefix[F] (the scanned total), hoisted by callers that map many ids
PSS_HD void map_one_bucketed_t(const int64_t *prefix, int64_t F, int64_t T, const int32_t *BT,
                               int32_t kb, int64_t nb, int64_t id0, int32_t &fpos, int64_t &off) {
    int64_t id = id0;
    bool refl = false;
    if (id >= T) {
        id = 2 * T - id;
        if (id == T) id = T - 1;
        refl = true;
    }
    if (id < 0) { fpos = INT32_MIN; off = id0; return; }
    const int64_t b = id >> kb;
    int64_t lo = BT[b];
    int64_t hi = b + 1 < nb ? (int64_t)BT[b + 1] : F - 1;   // answer in [lo, hi]
    while (hi > lo) {                                        // largest f with prefix[f] <= id
        const int64_t mid = (lo + hi + 1) >> 1;
        if (prefix[mid] <= id) lo = mid; else hi = mid - 1;
    }
    fpos = refl ? (int32_t)(-1 - lo) : (int32_t)lo;
    off = id - prefix[lo];
}

PSS_HD void map_one_bucketed(const int64_t *prefix, int64_t F, const int32_t *BT, int32_t kb,
                             int64_t nb, int64_t id0, int32_t &fpos, int64_t &off) {
    map_one_bucketed_t(prefix, F, prefix[F], BT, kb, nb, id0, fpos, off);
}

}  // namespace pss
