// pss_cpu_driver.cpp -- host-side workout of libpss's C ABI in CPU mode, built with sanitizers
// (tools/sanitize/Makefile: ASan + UBSan, TSan).  Exercises everything the host runtime does
// without a GPU: the constructor math, the init_iter history with the file-permutation prefetch
// threads (PermPrefetcher: worker threads, recycled buffers, epoch jumps that miss the prefetch),
// the CPU mode's per-rank / per-group host threads (counter order V1 / V2 with small and grouped
// pools, exact order with CPython MT windows and the Fenwick-tree V2), partial position and rank
// ranges, the map, the fused hand-off, the partition, the digests, the lookahead knobs, and several
// handles driven from concurrent threads (handles share no state -- SURVEY.md §5's reference hazard
// is the process-global `random`).  Exit code 0 and a clean sanitizer log are the result.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

#include "../../include/pss.h"

static int g_fail = 0;
#define CHECK(x)                                                                           \
    do {                                                                                   \
        int rc_ = (x);                                                                     \
        if (rc_ != PSS_OK) {                                                               \
            std::fprintf(stderr, "%s:%d %s -> %d (%s)\n", __FILE__, __LINE__, #x, rc_,     \
                         pss_last_error());                                                \
            g_fail = 1;                                                                    \
        }                                                                                  \
    } while (0)
#define EXPECT(c)                                                                          \
    do {                                                                                   \
        if (!(c)) {                                                                        \
            std::fprintf(stderr, "%s:%d expectation failed: %s\n", __FILE__, __LINE__, #c); \
            g_fail = 1;                                                                    \
        }                                                                                  \
    } while (0)

struct Shape {
    int64_t F, lo, hi, extra;
    int32_t R;
    int64_t B;
    int32_t version, shuffle, order;
};

// one handle through several epochs: every call the host runtime serves in CPU mode
static void workout(const Shape &sh, uint64_t seed) {
    std::mt19937_64 rng(seed);
    std::vector<int64_t> lens(sh.F);
    int64_t N = 0;
    for (auto &l : lens) {
        l = sh.lo + (int64_t)(rng() % (uint64_t)(sh.hi - sh.lo + 1));
        N += l;
    }
    N += sh.extra;
    pss_sampler *h = nullptr;
    CHECK(pss_create(lens.data(), sh.F, N, sh.R, sh.B, sh.version, sh.shuffle, seed, PSS_DEVICE_CPU, &h));
    if (!h) return;
    CHECK(pss_set_order_mode(h, sh.order));
    CHECK(pss_set_lookahead(h, -1, (int64_t)1 << 20, -1));   // no effect in CPU mode
    int64_t ns = 0;
    CHECK(pss_num_samples(h, &ns));
    std::vector<int64_t> ids((size_t)sh.R * ns), off((size_t)sh.R * ns);
    std::vector<int32_t> fpos((size_t)sh.R * ns), fpos2((size_t)sh.R * ns), off32((size_t)sh.R * ns);
    std::vector<int32_t> order(sh.F), blocks(sh.R);
    std::vector<int64_t> olds(sh.R), news(sh.R);
    // consecutive epochs (the prefetch hits), a jump (a miss), a repeat (the cumulative history)
    const int64_t epochs[] = {0, 1, 2, 7, 8, 8, 3};
    for (int64_t e : epochs) {
        CHECK(pss_init_iter(h, e));
        CHECK(pss_file_order(h, order.data()));
        CHECK(pss_blocks(h, blocks.data()));
        CHECK(pss_rank_starts(h, olds.data(), news.data()));
        CHECK(pss_prepare(h, nullptr));
        CHECK(pss_generate(h, 0, sh.R, 0, ns, ids.data(), nullptr));
        // coverage: every id of [0, N) once, plus the padding ns * R - N from the front
        uint64_t acc = 0, want = 0;
        CHECK(pss_digest_host(ids.data(), (int64_t)ids.size(), &acc));
        CHECK(pss_digest_range_host(0, N, &want));
        CHECK(pss_digest_range_host(0, ns * sh.R - N, &want));
        EXPECT(acc == want);
        CHECK(pss_map(h, ids.data(), (int64_t)ids.size(), fpos.data(), off.data(), nullptr));
        CHECK(pss_generate_mapped(h, 0, sh.R, 0, ns, fpos2.data(), off32.data(), nullptr));
        for (size_t i = 0; i < ids.size(); i++) EXPECT(fpos[i] == fpos2[i] && off[i] == off32[i]);
        // partial ranges: a rank range, a position window, the tail
        const int64_t p0 = ns / 3, cnt = std::min<int64_t>(ns - p0, sh.B + 17);
        std::vector<int64_t> part((size_t)sh.R * cnt);
        CHECK(pss_generate(h, sh.R > 1 ? 1 : 0, sh.R, p0, cnt, part.data(), nullptr));
        const int32_t r0 = sh.R > 1 ? 1 : 0;
        for (int32_t r = r0; r < sh.R; r++)
            for (int64_t i = 0; i < cnt; i++) EXPECT(part[(size_t)(r - r0) * cnt + i] == ids[(size_t)r * ns + p0 + i]);
        std::vector<int64_t> seg_off(sh.R + 1);
        CHECK(pss_partition(h, 0, sh.R, seg_off.data(), nullptr, nullptr, nullptr, 0, nullptr));
        const int64_t nseg = seg_off[sh.R];
        std::vector<int32_t> sf(nseg > 0 ? nseg : 1);
        std::vector<int64_t> sl(sf.size()), shi(sf.size());
        CHECK(pss_partition(h, 0, sh.R, seg_off.data(), sf.data(), sl.data(), shi.data(), (int64_t)sf.size(), nullptr));
    }
    double ms[8];
    int64_t n[8];
    CHECK(pss_profile(h, 1));
    CHECK(pss_generate(h, 0, sh.R, 0, ns, ids.data(), nullptr));
    CHECK(pss_profile_read(h, ms, n, 8));
    int64_t bytes = -1, stats[4];
    CHECK(pss_workspace_bytes(h, &bytes));
    EXPECT(bytes == 0);
    CHECK(pss_lookahead_stats(h, stats));
    CHECK(pss_destroy(h));
}

int main() {
    const Shape shapes[] = {
        // F, lo, hi, extra, R, B, version, shuffle, order
        {64, 800, 1200, 0, 2, 256, 1, 1, PSS_ORDER_COUNTER},        // C1-like, small
        {40, 300, 900, 77, 3, 128, 2, 1, PSS_ORDER_COUNTER},        // reflected ids past the files
        {30, 0, 400, 0, 4, 100, 2, 1, PSS_ORDER_COUNTER},           // empty files, odd pool
        {20, 2000, 3000, 0, 2, 20000, 2, 1, PSS_ORDER_COUNTER},     // grouped pools (P1 > 16384)
        {50, 100, 300, 0, 3, 64, 1, 0, PSS_ORDER_COUNTER},          // V1 shuffle=False
        {40, 200, 600, 5, 3, 256, 1, 1, PSS_ORDER_EXACT},           // exact V1 windows
        {40, 200, 600, 5, 3, 256, 2, 1, PSS_ORDER_EXACT},           // exact V2 (Fenwick)
        {12, 3000, 5000, 0, 2, 5000, 2, 1, PSS_ORDER_EXACT},        // exact V2, one long window
    };
    for (int i = 0; i < (int)(sizeof(shapes) / sizeof(shapes[0])); i++) workout(shapes[i], 1000 + i);
    // several handles from concurrent threads (each handle is single-threaded by contract)
    std::vector<std::thread> ts;
    for (int t = 0; t < 4; t++)
        ts.emplace_back([t, &shapes] { workout(shapes[t % 8], 77 + t); workout(shapes[(t + 5) % 8], 99 + t); });
    for (auto &t : ts) t.join();
    // argument errors come back as codes, never as crashes
    pss_sampler *h = nullptr;
    EXPECT(pss_create(nullptr, 5, 10, 1, 4, 1, 1, 0, PSS_DEVICE_CPU, &h) == PSS_EINVAL);
    int64_t one = 10;
    EXPECT(pss_create(&one, 1, 10, 0, 4, 1, 1, 0, PSS_DEVICE_CPU, &h) == PSS_EINVAL);
    CHECK(pss_create(&one, 1, 10, 2, 4, 2, 1, 0, PSS_DEVICE_CPU, &h));
    int64_t x[10];
    EXPECT(pss_generate(h, 0, 2, 0, 5, x, nullptr) == PSS_ESTATE);
    EXPECT(pss_generate(h, 0, 3, 0, 5, x, nullptr) == PSS_EINVAL);
    EXPECT(pss_set_lookahead(h, 9, 0, 0) == PSS_EINVAL);
    CHECK(pss_destroy(h));
    std::printf(g_fail ? "pss_cpu_driver: FAILED\n" : "pss_cpu_driver: ok\n");
    return g_fail;
}
