// clock_v2.hip -- diagnostic (-DPSS_STAMPS build): in-kernel shader clock of the V2 replay,
// back to back vs with idle gaps: clock = d(s_memtime) / d(s_memrealtime) * 100 MHz per wave.
#include "../partiallyshuffledistributedsampler_amd/csrc/pss_v2.hip"
#include <cstdio>
#include <vector>
#include <unistd.h>
#include <algorithm>
#include <map>
#include <cmath>

int main() {
    using namespace pss;
    Geometry g{};
    g.N = 100000000; g.R = 8; g.ns = 12500000; g.B = 4096; g.version = 2; g.shuffle = 1;
    g.key0 = 0x1234u; g.key1 = 0x9abcu;
    std::vector<RankDesc> rd(8);
    for (int r = 0; r < 8; r++) { rd[r].old_start = (int64_t)r * g.ns; rd[r].new_start = (int64_t)((r + 3) % 8) * g.ns; }
    RankDesc *d_rd; (void)hipMalloc(&d_rd, sizeof(RankDesc) * 8);
    (void)hipMemcpy(d_rd, rd.data(), sizeof(RankDesc) * 8, hipMemcpyHostToDevice);
    (void)init_kernel_attributes_v2();
    int64_t *out; (void)hipMalloc(&out, sizeof(int64_t) * 8 * g.ns);
    uint32_t *val; (void)hipMalloc(&val, v2_val_bytes(g, 8));
    launch_v2(g, d_rd, 0, 8, 0, g.ns, out, val, nullptr, nullptr, nullptr, 0, Marker(), EMIT_XCHG, V2_STAGE_PRE);
    (void)hipDeviceSynchronize();
    std::vector<uint64_t> st((size_t)65536 * 8);
    for (int mode = 0; mode < 2; mode++) {
        for (int e = 0; e < 30; e++) {
            launch_v2(g, d_rd, 0, 8, 0, g.ns, out, val, nullptr, nullptr, nullptr, 0, Marker(), EMIT_XCHG, V2_STAGE_EMIT);
            if (mode == 1) { (void)hipDeviceSynchronize(); usleep(300); }
        }
        (void)hipDeviceSynchronize();
        (void)hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(pss_stamps), st.size() * 8);
        double clk = 0, rt = 0;
        std::vector<double> life;
        for (int b = 0; b < 2048; b++) {
            clk += (double)st[(size_t)b * 8]; rt += (double)st[(size_t)b * 8 + 1];
            life.push_back(st[(size_t)b * 8 + 1] / 100.0);
        }
        std::sort(life.begin(), life.end());
        uint64_t t0 = ~0ull, t1 = 0;
        double pro = 0, epi = 0;
        for (int b = 0; b < 2048; b++) {
            const uint64_t *x = &st[(size_t)b * 8];
            t0 = std::min(t0, x[2]); t1 = std::max(t1, x[5]);
            pro += (double)(x[3] - x[2]); epi += (double)(x[5] - x[4]);
        }
        // waves per SIMD and the mean life of waves by their SIMD's wave count
        std::map<uint64_t, int> per;
        for (int b = 0; b < 2048; b++) {
            const uint64_t *x = &st[(size_t)b * 8];
            const uint64_t hw = x[6], key = (x[7] << 32) | (hw & 0xFF30);   // xcc | se,sh,cu | simd
            per[key]++;
        }
        std::map<int, std::pair<double, int>> bycount;
        for (int b = 0; b < 2048; b++) {
            const uint64_t *x = &st[(size_t)b * 8];
            const uint64_t key = (x[7] << 32) | (x[6] & 0xFF30);
            auto &e = bycount[per[key]];
            e.first += x[1] / 100.0; e.second++;
        }
        // pairs of waves sharing a SIMD: loop-start and loop-end skew
        std::map<uint64_t, std::vector<const uint64_t *>> simd;
        for (int b = 0; b < 2048; b++) {
            const uint64_t *x = &st[(size_t)b * 8];
            simd[(x[7] << 32) | (x[6] & 0xFF30)].push_back(x);
        }
        double dstart = 0, dend = 0, pspan = 0; int np = 0;
        for (auto &kv : simd) if (kv.second.size() == 2) {
            const uint64_t *a = kv.second[0], *c = kv.second[1];
            dstart += std::fabs((double)a[3] - (double)c[3]);
            dend += std::fabs((double)a[4] - (double)c[4]);
            pspan += (double)(std::max(a[4], c[4]) - std::min(a[3], c[3]));
            np++;
        }
        if (np) printf("  SIMD pairs %d: |start skew| %.1f us, |end skew| %.1f us, pair span %.1f us\n", np, dstart / np / 100.0, dend / np / 100.0, pspan / np / 100.0);
        {   // timeline quantiles (us from the first wave's entry): entry, loop start, loop end, exit
            std::vector<double> q[4];
            for (int b = 0; b < 2048; b++) {
                const uint64_t *x = &st[(size_t)b * 8];
                for (int k = 0; k < 4; k++) q[k].push_back((double)(x[2 + k] - t0) / 100.0);
            }
            const char *nm[4] = {"entry", "loop start", "loop end", "exit"};
            for (int k = 0; k < 4; k++) {
                std::sort(q[k].begin(), q[k].end());
                printf("  %-10s min %.1f p10 %.1f p50 %.1f p90 %.1f max %.1f\n", nm[k], q[k][0], q[k][204], q[k][1024], q[k][1843], q[k][2047]);
            }
            // by XCC: mean loop and mean loop end
            double ml[8] = {0}, me[8] = {0}; int nx[8] = {0};
            for (int b = 0; b < 2048; b++) {
                const uint64_t *x = &st[(size_t)b * 8];
                int xc = (int)(x[7] & 7);
                ml[xc] += (double)(x[4] - x[3]) / 100.0; me[xc] += (double)(x[4] - t0) / 100.0; nx[xc]++;
            }
            printf("  by XCC (waves, loop us, loop end us):");
            for (int k = 0; k < 8; k++) if (nx[k]) printf(" [%d: %d %.0f %.0f]", k, nx[k], ml[k] / nx[k], me[k] / nx[k]);
            printf("\n");
        }
        for (auto &kv : bycount) printf("  SIMDs with %d waves: %d waves, mean loop %.1f us\n", kv.first, kv.second.second, kv.second.first / kv.second.second);
        printf("  span %.1f us; mean prologue %.1f us, epilogue (tail) %.1f us\n", (t1 - t0) / 100.0, pro / 2048 / 100.0, epi / 2048 / 100.0);
        printf("%s: wave us mean %.1f p10 %.1f p50 %.1f p90 %.1f max %.1f, shader clock %.2f GHz\n",
               mode ? "300us gaps" : "back-to-back", rt / 2048 / 100.0, life[204], life[1024], life[1843],
               life[2047], clk / rt * 0.1);
    }
    return 0;
}
