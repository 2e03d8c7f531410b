// stamp_v2x.hip -- diagnostic: the V2 exchange replay k_v2_emit_x built with -DPSS_STAMPS
// -DPSS_STAMPS_EMIT_ONLY on the C2 shape (8 ranks x 12.5M ids, B = 4096); prints per-wave phase
// times (start, setup done, replay end, end) by tile role (first / middle / last of a rank) and
// the end times per XCD.
//   stamp_v2x pass    each replay beside the next epoch's last-occurrence pass on a second
//                     stream (the bench's steady state)
//   stamp_v2x alone   the replays only
//   stamp_v2x alone <shift>   ... into the output buffer shifted by <shift> ids (address effects)
// (-DPSS_DIAG_TILE_SWAP: block b replays tile b ^ 1, so that tile parity and XCD trade places)
// Build (from the repo root; -DPSS_V2_SRC='"<path>"' stamps another copy of pss_v2.hip):
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DPSS_STAMPS -DPSS_STAMPS_EMIT_ONLY \
//     -Ipartiallyshuffledistributedsampler_amd/csrc -o build/stamp_v2x tools/stamp_v2x.hip \
//     partiallyshuffledistributedsampler_amd/csrc/pss_v2grp.hip
#ifndef PSS_V2_SRC
#define PSS_V2_SRC "../partiallyshuffledistributedsampler_amd/csrc/pss_v2.hip"
#endif
#include PSS_V2_SRC
#include <cstdio>
#include <vector>
#include <algorithm>
#include <map>
#include <string>

static void pct(const char *what, std::vector<double> v) {
    if (v.empty()) return;
    std::sort(v.begin(), v.end());
    printf("  %-14s p0 %7.1f p10 %7.1f p50 %7.1f p90 %7.1f max %7.1f us\n", what, v[0],
           v[v.size() / 10], v[v.size() / 2], v[v.size() * 9 / 10], v.back());
}

int main(int argc, char **argv) {
    using namespace pss;
    const bool pass = argc < 2 || std::string(argv[1]) == "pass";
    const int64_t shift = argc > 2 ? atoll(argv[2]) : 0;
    Geometry g{};
    g.N = 100000000; g.R = 8; g.ns = 12500000; g.B = 4096; g.version = 2; g.shuffle = 1;
    g.key0 = 0x12345678u; g.key1 = 0x9abcdef0u;
    std::vector<RankDesc> rd(8);
    for (int r = 0; r < 8; r++) { rd[r].old_start = (int64_t)r * g.ns; rd[r].new_start = (int64_t)((r + 3) % 8) * g.ns; }
    RankDesc *d_rd; hipMalloc(&d_rd, sizeof(RankDesc) * 8);
    hipMemcpy(d_rd, rd.data(), sizeof(RankDesc) * 8, hipMemcpyHostToDevice);
    init_kernel_attributes_v2();
    int64_t *out0; hipMalloc(&out0, sizeof(int64_t) * (8 * g.ns + shift));
    int64_t *out = out0 + shift;
    uint32_t *val[2]; hipMalloc(&val[0], v2_val_bytes(g, 8)); hipMalloc(&val[1], v2_val_bytes(g, 8));
    hipStream_t s1, s2; hipStreamCreate(&s1); hipStreamCreate(&s2);
    const V2Plan pl = v2_plan(g, 8);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    launch_v2(g, d_rd, 0, 8, 0, g.ns, out, val[0], nullptr, nullptr, nullptr, s1, Marker(),
              EMIT_XCHG, V2_STAGE_PRE);
    launch_v2(g, d_rd, 0, 8, 0, g.ns, out, val[1], nullptr, nullptr, nullptr, s1, Marker(),
              EMIT_XCHG, V2_STAGE_PRE);
    hipDeviceSynchronize();
    for (int it = 0; it < 6; it++) {
        hipEventRecord(e0, s1);
        launch_v2(g, d_rd, 0, 8, 0, g.ns, out, val[it & 1], nullptr, nullptr, nullptr, s1,
                  Marker(), EMIT_XCHG, V2_STAGE_EMIT);
        if (pass)
            launch_v2(g, d_rd, 0, 8, 0, g.ns, out, val[(it + 1) & 1], nullptr, nullptr, nullptr, s2,
                      Marker(), EMIT_XCHG, V2_STAGE_PRE);
        hipEventRecord(e1, s1);
        hipDeviceSynchronize();
        float ms = 0; hipEventElapsedTime(&ms, e0, e1);
        printf("launch %d: %.1f us (G=%lld L=%lld)\n", it, ms * 1e3, (long long)pl.G, (long long)pl.L);
    }
    const int nwg = (int)(8 * pl.G);
    std::vector<uint64_t> st((size_t)65536 * 8);
    hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(pss_stamps), st.size() * 8);
    uint64_t r0 = ~0ull;
    for (int b = 0; b < nwg; b++) r0 = std::min(r0, st[(size_t)b * 8 + 2]);
    const char *role[3] = {"first tile", "middle tiles", "last tile"};
    for (int k = 0; k < 3; k++) {
        std::vector<double> s0, s1v, rend, end;
        for (int b = 0; b < nwg; b++) {
            const int tile = (int)(b % pl.G);
            const int kind = tile == 0 ? 0 : tile == pl.G - 1 ? 2 : 1;
            if (kind != k) continue;
            const uint64_t *s = &st[(size_t)b * 8];
            s0.push_back((s[2] - r0) / 100.0);
            s1v.push_back((s[3] - r0) / 100.0);
            rend.push_back((s[4] - r0) / 100.0);
            end.push_back((s[5] - r0) / 100.0);
        }
        printf("%s (%zu waves)\n", role[k], s0.size());
        pct("start", s0); pct("setup done", s1v); pct("replay end", rend); pct("end", end);
    }
    std::map<uint32_t, std::vector<double>> byx;
    for (int b = 0; b < nwg; b++) {
        const uint64_t *s = &st[(size_t)b * 8];
        byx[(uint32_t)s[7] & 0xFu].push_back((s[5] - r0) / 100.0);
    }
    for (auto &kv : byx) { char nm[32]; snprintf(nm, sizeof nm, "end, XCC %u", kv.first); pct(nm, kv.second); }
    printf("block -> XCC:");
    for (int b = 0; b < 16; b++) printf(" %u", (uint32_t)st[(size_t)b * 8 + 7] & 0xFu);
    printf("\n");
    // by tile parity (the tile's output region) within each XCC parity
    for (int xp = 0; xp < 2; xp++)
        for (int tp = 0; tp < 2; tp++) {
            std::vector<double> v;
            for (int b = 0; b < nwg; b++) {
                const uint64_t *s = &st[(size_t)b * 8];
#ifdef PSS_DIAG_TILE_SWAP
                const int tile = (int)((b % pl.G) ^ 1);
#else
                const int tile = (int)(b % pl.G);
#endif
                if ((int)(((uint32_t)s[7] & 0xFu) & 1u) == xp && (tile & 1) == tp) v.push_back((s[5] - r0) / 100.0);
            }
            char nm[40]; snprintf(nm, sizeof nm, "XCC%%2=%d tile%%2=%d", xp, tp); pct(nm, v);
        }
    return 0;
}

// (the rank upload of the non-fused tail lives in pss_kernels.hip; never reached here)
namespace pss {
hipError_t launch_put_ranks(const RankDesc *, int, RankDesc *, hipStream_t) { return hipErrorNotSupported; }
}
