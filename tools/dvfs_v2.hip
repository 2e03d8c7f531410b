// dvfs_v2.hip -- experiment: is the V2 replay clock/power limited?  Times k_v2_emit_x launches
// (C2 shape) back to back, and the same launches separated by idle gaps, with HIP events per
// launch; also the last-occurrence pass alone.
#include "pss_kernels.h"
#include <cstdio>
#include <vector>
#include <unistd.h>

using namespace pss;

int main() {
    Geometry g{};
    g.N = 100000000; g.R = 8; g.ns = 12500000; g.B = 4096; g.version = 2; g.shuffle = 1;
    g.key0 = 0x1234u; g.key1 = 0x9abcu;
    std::vector<RankDesc> rd(8);
    for (int r = 0; r < 8; r++) { rd[r].old_start = (int64_t)r * g.ns; rd[r].new_start = (int64_t)((r + 3) % 8) * g.ns; }
    RankDesc *d_rd; (void)hipMalloc(&d_rd, sizeof(RankDesc) * 8);
    (void)hipMemcpy(d_rd, rd.data(), sizeof(RankDesc) * 8, hipMemcpyHostToDevice);
    (void)init_kernel_attributes();
    int64_t *out; (void)hipMalloc(&out, sizeof(int64_t) * 8 * g.ns);
    uint32_t *val; (void)hipMalloc(&val, v2_val_bytes(g, 8));
    launch_v2(g, d_rd, 0, 8, 0, g.ns, out, val, nullptr, nullptr, nullptr, 0, Marker(), EMIT_XCHG, V2_STAGE_PRE);
    (void)hipDeviceSynchronize();
    const int E = 30;
    std::vector<hipEvent_t> ev(2 * E);
    for (auto &e : ev) (void)hipEventCreate(&e);
    for (int mode = 0; mode < 4; mode++) {
        for (int e = 0; e < E; e++) {
            (void)hipEventRecord(ev[2 * e], 0);
            const int stage = (mode == 2) ? V2_STAGE_PRE : V2_STAGE_EMIT;
            launch_v2(g, d_rd, 0, 8, 0, g.ns, out, val, nullptr, nullptr, nullptr, 0, Marker(), EMIT_XCHG, stage);
            (void)hipEventRecord(ev[2 * e + 1], 0);
            if (mode == 1 || mode == 3) { (void)hipDeviceSynchronize(); usleep(mode == 1 ? 300 : 2000); }
        }
        (void)hipDeviceSynchronize();
        double sum = 0, mn = 1e9, mx = 0;
        for (int e = 5; e < E; e++) {
            float ms = 0;
            (void)hipEventElapsedTime(&ms, ev[2 * e], ev[2 * e + 1]);
            sum += ms; mn = ms < mn ? ms : mn; mx = ms > mx ? ms : mx;
        }
        const char *names[] = {"emit back-to-back", "emit, 300us idle gaps", "lastocc back-to-back", "emit, 2ms idle gaps"};
        printf("%-24s mean %.1f us  min %.1f  max %.1f\n", names[mode], sum / (E - 5) * 1e3, mn * 1e3, mx * 1e3);
    }
    return 0;
}
