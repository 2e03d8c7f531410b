// pss_cpu.cpp -- the product's CPU mode (pss.h PSS_DEVICE_CPU).
//
// The counter schedule is evaluated from the very definitions the gfx950 kernels use
// (pss_common.h: Philox keys, slot hash, grouped draws, Feistel bijections; pss_map.h: id ->
// (file, offset)), one host thread per (rank) or (rank, group) stream, so CPU mode == GPU bit
// for bit by construction; tests check both against the independent oracle twin.  The exact
// order replays the reference's own CPython-MT draws: V1 windows (V1:102,114-115,165-171) and
// V2 get_index (V2:96-116) with order-statistic trees in place of list.remove.
#include <hip/hip_runtime.h>
#include <sched.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <thread>
#include <vector>

#include "pss_common.h"
#include "pss_cpu.h"
#include "pss_host_mt.h"
#include "pss_map.h"

namespace pss {
namespace cpu {

int threads() {
    static const int n = [] {
        const char *e = getenv("PSS_CPU_THREADS");
        if (e && atoi(e) > 0) return atoi(e);
        cpu_set_t set;
        CPU_ZERO(&set);
        int c = 0;
        if (sched_getaffinity(0, sizeof(set), &set) == 0) c = CPU_COUNT(&set);
        if (c <= 0) c = (int)std::thread::hardware_concurrency();
        return c > 0 ? c : 1;
    }();
    return n;
}

template <class Fn>
static void parallel_for(int64_t n, Fn fn) {
    const int64_t nt = std::min<int64_t>(threads(), n);
    if (nt <= 1) {
        for (int64_t i = 0; i < n; i++) fn(i);
        return;
    }
    std::atomic<int64_t> next(0);
    std::vector<std::thread> pool;
    pool.reserve((size_t)nt);
    for (int64_t w = 0; w < nt; w++)
        pool.emplace_back([&] {
            for (int64_t i = next++; i < n; i = next++) fn(i);
        });
    for (auto &t : pool) t.join();
}

static inline int64_t wrap(int64_t id, int64_t N) { return id >= N ? id - N : id; }

// one rank's output row: positions [lo, hi) of its stream
struct Row {
    int64_t *o;
    int64_t lo, hi;
    void put(int64_t pos, int64_t id) const {
        if (pos >= lo && pos < hi) o[pos - lo] = id;
    }
};

// ---- V1 -------------------------------------------------------------------------------------
static void v1_counter(const Geometry &g, uint32_t rank, int64_t start, const Row &row) {
    for (int64_t w = row.lo / g.B; w * g.B < row.hi; w++) {
        const int64_t wB = w * g.B;
        const int64_t len = std::min<int64_t>(g.B, g.ns - wB);
        uint32_t k[8];
        if (g.shuffle) round_keys8(g.key0, g.key1, (uint32_t)w, rank, DOM_V1_WIN, k);
        const uint32_t h = feistel_half_bits((uint32_t)len);
        const int64_t p0 = std::max(row.lo, wB), p1 = std::min(row.hi, wB + len);
        for (int64_t p = p0; p < p1; p++) {
            const int64_t y = g.shuffle ? feistel((uint32_t)(p - wB), (uint32_t)len, h, k) : p - wB;
            row.put(p, wrap(start + wB + y, g.N));
        }
    }
}

// V1:102,114-115 (window 0: seed(epoch)) and V1:165-171 (window b: seed(epoch + b * 10000)),
// each a CPython shuffle of range(len)
static void v1_exact(const Geometry &g, int64_t epoch, int64_t start, const Row &row) {
    std::vector<int64_t> perm;
    for (int64_t w = row.lo / g.B; w * g.B < row.hi; w++) {
        const int64_t wB = w * g.B;
        const int64_t len = std::min<int64_t>(g.B, g.ns - wB);
        perm.resize((size_t)len);
        for (int64_t i = 0; i < len; i++) perm[i] = i;
        if (g.shuffle) {
            CPythonMT mt;
            mt.seed(w == 0 ? epoch : epoch + w * 10000);
            mt.shuffle(perm.data(), len);
        }
        const int64_t p0 = std::max(row.lo, wB), p1 = std::min(row.hi, wB + len);
        for (int64_t p = p0; p < p1; p++) row.put(p, wrap(start + wB + perm[p - wB], g.N));
    }
}

// ---- V2 counter schedule ----------------------------------------------------------------------
static inline int64_t v2_id(uint32_t v, const RankDesc &rd, const Geometry &g) {
    return wrap(((int64_t)v < 2 * g.B ? rd.old_start : rd.new_start) + (int64_t)v, g.N);
}

// value inserted at step t (pool2 window w = 1 + t / B in the order of its Feistel bijection),
// with the current window's round keys cached
struct Inserter {
    const Geometry &g;
    uint32_t rank;
    int64_t cur = -1;
    uint32_t k[8];
    uint32_t len = 0, h = 0;
    uint32_t operator()(int64_t t) {
        const int64_t w = 1 + t / g.B;
        if (w != cur) {
            round_keys8(g.key0, g.key1, (uint32_t)w, rank, DOM_V2_INS, k);
            len = (uint32_t)std::min<int64_t>(g.B, g.ns - w * g.B);
            h = feistel_half_bits(len);
            cur = w;
        }
        return (uint32_t)(w * g.B) + feistel((uint32_t)(t - (w - 1) * g.B), len, h, k);
    }
};

static void slot_key_of(const Geometry &g, uint32_t rank, uint32_t &s0, uint32_t &s1) {
    uint32_t c0 = 0, c1 = 0, c2 = rank, c3 = DOM_V2_SLOT;
    philox4x32_10_rolled(c0, c1, c2, c3, g.key0, g.key1);
    s0 = c0; s1 = c1;
}

// pools up to kLdsSlotMax: one slot machine per rank
static void v2_small(const Geometry &g, uint32_t rank, const RankDesc &rd, const Row &row) {
    const int64_t P1 = std::min(g.B, g.ns), T = g.ns - P1;
    std::vector<uint32_t> buf((size_t)P1);
    for (int64_t s = 0; s < P1; s++) buf[s] = (uint32_t)s;
    uint32_t s0, s1;
    slot_key_of(g, rank, s0, s1);
    Inserter ins{g, rank};
    const int64_t tend = std::min(T, row.hi);
    for (int64_t t = 0; t < tend; t++) {
        const uint32_t k = slot_draw((uint32_t)t, s0, s1, (uint32_t)P1);
        if (t >= row.lo) row.o[t - row.lo] = v2_id(buf[k], rd, g);
        buf[k] = ins(t);
    }
    if (row.hi > T) {
        uint32_t tk[8];
        round_keys8(g.key0, g.key1, 0, rank, DOM_V2_TAIL, tk);
        const uint32_t hT = feistel_half_bits((uint32_t)P1);
        for (int64_t j = std::max<int64_t>(0, row.lo - T); j < P1 && T + j < row.hi; j++)
            row.put(T + j, v2_id(buf[feistel((uint32_t)j, (uint32_t)P1, hT, tk)], rd, g));
    }
}

// pools beyond kLdsSlotMax: group g of a rank is its own slot machine over its slots of the
// rank's table (pss_v2grp.hip), then drains its final slots into its tail positions
static void v2_group(const Geometry &g, uint32_t rank, const RankDesc &rd, const Groups &gr,
                     uint32_t grp, uint32_t *buf, const Row &row) {
    const int64_t P1 = std::min(g.B, g.ns), T = g.ns - P1;
    const uint32_t S = group_size(gr, grp), base = group_base(gr, grp);
    uint32_t s0, s1;
    slot_key_of(g, rank, s0, s1);
    Inserter ins{g, rank};
    const uint64_t Tg = group_steps(gr, grp, (uint64_t)T);
    for (uint64_t u = 0; u < Tg; u++) {
        const int64_t t = (int64_t)group_step(gr, grp, u);
        if (t >= row.hi) break;
        const uint32_t k = base + group_slot(gr, grp, S, u, (uint32_t)t, s0, s1);
        if (t >= row.lo) row.o[t - row.lo] = v2_id(buf[k], rd, g);
        buf[k] = ins(t);
    }
    if (row.hi > T) {
        uint32_t tk[8];
        round_keys8(g.key0, g.key1, grp, rank, DOM_V2_TAIL, tk);
        const uint32_t hS = feistel_half_bits(S);
        for (uint32_t e = 0; e < S; e++)
            row.put(T + group_tail_pos(gr, grp, e), v2_id(buf[base + feistel(e, S, hS, tk)], rd, g));
    }
}

// ---- V2 exact order ---------------------------------------------------------------------------
// Order-statistic tree over slot positions: k-th alive in O(log n) (list.remove in the reference)
struct Fenwick {
    std::vector<int32_t> t;
    int64_t n = 0;
    int64_t top = 1;
    void build(int64_t size, int64_t alive) {   // positions [0, alive) alive
        n = size;
        t.assign((size_t)n + 1, 0);
        for (int64_t i = 1; i <= alive; i++) t[i] += 1;
        for (int64_t i = 1; i <= n; i++) {
            const int64_t j = i + (i & -i);
            if (j <= n) t[j] += t[i];
        }
        top = 1;
        while (top * 2 <= n) top *= 2;
    }
    void add(int64_t i, int32_t d) {
        for (i++; i <= n; i += i & -i) t[i] += d;
    }
    int64_t kth(int64_t k) const {   // position of the k-th (0-based) alive entry
        int64_t pos = 0;
        for (int64_t b = top; b; b >>= 1)
            if (pos + b <= n && t[pos + b] <= k) { pos += b; k -= t[pos]; }
        return pos;
    }
};

// V2:96-116 with its seeding (V2:135-148): pools 0/1 from the OLD start, seed(epoch + 2), then
// choice / remove / append, reseeding seed(epoch + buffers * 10000) whenever pool2 empties
// (every step of the tail).  Same semantics as oracle/pss_oracle.c's v2_exact.
static void v2_exact(const Geometry &g, int64_t epoch, const RankDesc &rd, const Row &row) {
    const int64_t B = g.B, ns = g.ns;
    const int64_t P1 = std::min(B, ns);
    std::vector<int64_t> v1((size_t)(P1 + ns));
    Fenwick f1, f2;
    f1.build(P1 + ns, P1);
    for (int64_t i = 0; i < P1; i++) v1[i] = rd.old_start + i;
    int64_t end1 = P1, n1 = P1;
    int64_t lo2 = rd.old_start + B;
    int64_t hi2 = std::min(rd.old_start + 2 * B, rd.old_start + ns);
    int64_t n2 = std::max<int64_t>(0, hi2 - lo2);
    f2.build(std::max<int64_t>(B, 1), n2);
    CPythonMT mt;
    mt.seed(epoch + 2);
    int64_t buffers = 0, drawn = 0;
    while ((n1 > 0 || n2 > 0) && drawn < row.hi) {
        const int64_t k = mt.randbelow((uint32_t)n1);
        if (n1 == 0) break;
        const int64_t p = f1.kth(k);
        const int64_t index = v1[p];
        f1.add(p, -1);
        n1--;
        if (n2 != 0) {
            const int64_t k2 = mt.randbelow((uint32_t)n2);
            const int64_t q = f2.kth(k2);
            f2.add(q, -1);
            n2--;
            v1[end1] = lo2 + q;
            f1.add(end1, +1);
            end1++;
            n1++;
        }
        if (n2 == 0) {
            mt.seed(epoch + buffers * 10000);
            buffers++;
            const int64_t lo = rd.new_start + (buffers + 1) * B;
            const int64_t hi = std::min(rd.new_start + (buffers + 2) * B, rd.new_start + ns);
            if (lo < hi) {
                lo2 = lo;
                n2 = hi - lo;
                f2.build(std::max<int64_t>(B, 1), n2);
            }
        }
        row.put(drawn, wrap(index, g.N));
        drawn++;
    }
}

// ---- entry points ----------------------------------------------------------------------------
void generate(const Geometry &g, const RankDesc *ranks, int32_t rank_lo, int32_t nr, int64_t pos_lo,
              int64_t count, int64_t epoch, bool exact, int64_t *out) {
    const int64_t pos_hi = std::min(pos_lo + count, g.ns);
    if (nr <= 0 || pos_hi <= pos_lo) return;
    auto row = [&](int32_t rl) { return Row{out + (int64_t)rl * count, pos_lo, pos_hi}; };
    const int64_t P1 = std::min(g.B, g.ns);
    if (g.version == 2 && !exact && P1 > (int64_t)kLdsSlotMax) {
        const Groups gr = v2_groups((uint32_t)P1);
        // per-rank tables (window 0 in its init Feistel order), then (rank, group) streams
        std::vector<std::vector<uint32_t>> bufs((size_t)nr);
        parallel_for(nr, [&](int64_t rl) {
            const uint32_t rank = (uint32_t)(rank_lo + rl);
            uint32_t ik[8];
            round_keys8(g.key0, g.key1, 0, rank, DOM_V2_INIT, ik);
            const uint32_t hP = feistel_half_bits((uint32_t)P1);
            auto &b = bufs[(size_t)rl];
            b.resize((size_t)P1);
            for (int64_t s = 0; s < P1; s++) b[s] = feistel((uint32_t)s, (uint32_t)P1, hP, ik);
        });
        parallel_for((int64_t)nr * gr.G, [&](int64_t i) {
            const int32_t rl = (int32_t)(i / gr.G);
            const uint32_t grp = (uint32_t)(i % gr.G);
            const uint32_t rank = (uint32_t)(rank_lo + rl);
            v2_group(g, rank, ranks[rank], gr, grp, bufs[(size_t)rl].data(), row(rl));
        });
        return;
    }
    parallel_for(nr, [&](int64_t rl) {
        const uint32_t rank = (uint32_t)(rank_lo + rl);
        const RankDesc &rd = ranks[rank];
        if (g.version == 1) {
            if (exact) v1_exact(g, epoch, rd.new_start, row((int32_t)rl));
            else v1_counter(g, rank, rd.new_start, row((int32_t)rl));
        } else {
            if (exact) v2_exact(g, epoch, rd, row((int32_t)rl));
            else v2_small(g, rank, rd, row((int32_t)rl));
        }
    });
}

void scan_prefix(const int64_t *lens, const int32_t *order, int64_t F, int64_t *prefix) {
    int64_t acc = 0;
    for (int64_t f = 0; f < F; f++) {
        prefix[f] = acc;
        acc += lens[order[f]];
    }
    prefix[F] = acc;
}

void map(const int64_t *prefix, int64_t F, const int64_t *ids, int64_t n, int32_t *fpos,
         int64_t *off) {
    const int64_t chunk = 1 << 16;
    parallel_for((n + chunk - 1) / chunk, [&](int64_t c) {
        const int64_t e = std::min(n, (c + 1) * chunk);
        for (int64_t i = c * chunk; i < e; i++) map_one(prefix, F, ids[i], fpos[i], off[i]);
    });
}

bool partition(const Geometry &g, const RankDesc *ranks, int32_t rank_lo, int32_t nr,
               const int64_t *prefix, int64_t F, int64_t *seg_off, int32_t *seg_file,
               int64_t *seg_lo, int64_t *seg_hi, int64_t seg_cap) {
    const int64_t T = prefix[F];
    seg_off[0] = 0;
    for (int32_t i = 0; i < nr; i++) {
        Ranges rr;
        rank_ranges(g, ranks[rank_lo + i], T, rr);
        int64_t c = 0;
        for (int k = 0; k < rr.n; k++) {
            const int64_t f0 = file_of(prefix, F, rr.lo[k]), f1 = file_of(prefix, F, rr.hi[k] - 1);
            for (int64_t f = f0; f <= f1; f++) c += prefix[f + 1] > prefix[f];
        }
        seg_off[i + 1] = seg_off[i] + c;
    }
    if (seg_cap <= 0) return true;
    if (seg_off[nr] > seg_cap) return false;
    for (int32_t i = 0; i < nr; i++) {
        Ranges rr;
        rank_ranges(g, ranks[rank_lo + i], T, rr);
        int64_t o = seg_off[i];
        for (int k = 0; k < rr.n; k++) {
            const int64_t f0 = file_of(prefix, F, rr.lo[k]), f1 = file_of(prefix, F, rr.hi[k] - 1);
            for (int64_t f = f0; f <= f1; f++) {
                if (prefix[f + 1] <= prefix[f]) continue;
                seg_file[o] = (int32_t)f;
                seg_lo[o] = std::max(rr.lo[k], prefix[f]) - prefix[f];
                seg_hi[o] = std::min(rr.hi[k], prefix[f + 1]) - prefix[f];
                o++;
            }
        }
    }
    return true;
}

uint64_t digest(const int64_t *ids, int64_t n) {
    uint64_t d = 0;
    for (int64_t i = 0; i < n; i++) d += mix64((uint64_t)ids[i]);
    return d;
}

uint64_t digest_range(int64_t lo, int64_t hi) {
    uint64_t d = 0;
    for (int64_t i = lo; i < hi; i++) d += mix64((uint64_t)i);
    return d;
}

}  // namespace cpu
}  // namespace pss
