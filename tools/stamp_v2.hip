// stamp_v2.hip -- diagnostic: the V2 kernels built with -DPSS_STAMPS in one TU, launched on a
// synthetic C2 shape (8 ranks x 12.5M ids, B = 4096); prints per-phase clock statistics of
// the last-occurrence pass.  Build (from the repo root):
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DPSS_STAMPS -Ipartiallyshuffledistributedsampler_amd/csrc \
//     -o build/stamp_v2 tools/stamp_v2.hip partiallyshuffledistributedsampler_amd/csrc/pss_v2grp.hip
#include "../partiallyshuffledistributedsampler_amd/csrc/pss_v2.hip"
#include <cstdio>
#include <vector>
#include <algorithm>
#include <map>

int main() {
    using namespace pss;
    Geometry g{};
    g.N = 100000000; g.R = 8; g.ns = 12500000; g.B = 4096; g.version = 2; g.shuffle = 1;
    g.key0 = 0x12345678u; g.key1 = 0x9abcdef0u;
    std::vector<RankDesc> rd(8);
    for (int r = 0; r < 8; r++) { rd[r].old_start = (int64_t)r * g.ns; rd[r].new_start = (int64_t)((r + 3) % 8) * g.ns; }
    RankDesc *d_rd; hipMalloc(&d_rd, sizeof(RankDesc) * 8);
    hipMemcpy(d_rd, rd.data(), sizeof(RankDesc) * 8, hipMemcpyHostToDevice);
    init_kernel_attributes_v2();
    int64_t *out; hipMalloc(&out, sizeof(int64_t) * 8 * g.ns);
    uint32_t *val; hipMalloc(&val, v2_val_bytes(g, 8));
    // full replays, then the last-occurrence pass alone (the emit kernel writes the same stamp
    // slots), back to back
    for (int it = 0; it < 3; it++)
        launch_v2(g, d_rd, 0, 8, 0, g.ns, out, val, nullptr, nullptr, nullptr, 0, Marker(), EMIT_XCHG);
    for (int it = 0; it < 5; it++)
        launch_v2(g, d_rd, 0, 8, 0, g.ns, out, val, nullptr, nullptr, nullptr, 0, Marker(), EMIT_XCHG, V2_STAGE_PRE);
    hipDeviceSynchronize();
    const V2Plan pl = v2_plan(g, 8);
    const int nwg = (int)(8 * pl.G);
    std::vector<uint64_t> st((size_t)65536 * 8);
    hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(pss_stamps), st.size() * 8);
    uint64_t r0 = ~0ull, r1 = 0;
    for (int b = 0; b < nwg; b++) { uint64_t *s = &st[(size_t)b * 8]; r0 = std::min(r0, s[4]); r1 = std::max(r1, s[5]); }
    std::vector<double> rs, re, life;
    std::map<uint32_t, int> percu;
    double ph[3] = {0, 0, 0};
    for (int b = 0; b < nwg; b++) {
        uint64_t *s = &st[(size_t)b * 8];
        rs.push_back((s[4] - r0) / 100.0); re.push_back((s[5] - r0) / 100.0); life.push_back((s[5] - s[4]) / 100.0);
        for (int i = 0; i < 3; i++) ph[i] += (double)(s[i + 1] - s[i]);
        const uint32_t hw = (uint32_t)s[6];
        percu[((uint32_t)s[7] << 16) | (hw & 0xFF00)]++;
    }
    std::sort(rs.begin(), rs.end()); std::sort(re.begin(), re.end()); std::sort(life.begin(), life.end());
    int mn = 1 << 30, mx = 0;
    for (auto &kv : percu) { mn = std::min(mn, kv.second); mx = std::max(mx, kv.second); }
    printf("lastocc: %d WGs G=%lld L=%lld: span %.1f us; start(us) p50 %.1f p90 %.1f max %.1f; end p10 %.1f p50 %.1f max %.1f; life p50 %.1f max %.1f\n",
           nwg, (long long)pl.G, (long long)pl.L, (r1 - r0) / 100.0, rs[nwg / 2], rs[nwg * 9 / 10], rs[nwg - 1],
           re[nwg / 10], re[nwg / 2], re[nwg - 1], life[nwg / 2], life[nwg - 1]);
    {   // by XCC: mean end and life of the workgroups; and by tile position in the rank
        double en[8] = {0}, lf[8] = {0}; int nx[8] = {0};
        double enl = 0, enf = 0; int nl = 0, nf = 0;
        for (int b = 0; b < nwg; b++) {
            const uint64_t *x = &st[(size_t)b * 8];
            const int xc = (int)(x[7] & 7);
            en[xc] += (x[5] - r0) / 100.0; lf[xc] += (x[5] - x[4]) / 100.0; nx[xc]++;
            if (b % pl.G == pl.G - 1) { enl += (x[5] - r0) / 100.0; nl++; } else { enf += (x[5] - r0) / 100.0; nf++; }
        }
        printf("by XCC (WGs, mean end us, mean life us):");
        for (int k = 0; k < 8; k++) if (nx[k]) printf(" [%d: %d %.0f %.0f]", k, nx[k], en[k] / nx[k], lf[k] / nx[k]);
        printf("\nlast tiles mean end %.1f us (%d), others %.1f us (%d)\n", enl / nl, nl, enf / nf, nf);
    }
    printf("mean phase clk: prologue %.0f loop %.0f epilogue %.0f; CUs %zu, WGs per CU %d..%d\n",
           ph[0] / nwg, ph[1] / nwg, ph[2] / nwg, percu.size(), mn, mx);
    return 0;
}
