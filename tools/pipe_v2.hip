// pipe_v2.hip -- experiment: does the V2 last-occurrence pass of epoch e+1 hide under the replay
// of epoch e when they run on two streams (replay on a high-priority stream, VAL double
// buffered)?  C2 shape (8 ranks x 12.5M ids, B = 4096), 20 epochs each way.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -Ipartiallyshuffledistributedsampler_amd/csrc \
//   -o build/pipe_v2 tools/pipe_v2.hip build/obj/pss_{kernels,v2,v2big,bigsort}.hip.o
#include "pss_kernels.h"
#include <cstdio>
#include <vector>

using namespace pss;

int main() {
    Geometry g{};
    g.N = 100000000; g.R = 8; g.ns = 12500000; g.B = 4096; g.version = 2; g.shuffle = 1;
    std::vector<RankDesc> rd(8);
    for (int r = 0; r < 8; r++) { rd[r].old_start = (int64_t)r * g.ns; rd[r].new_start = (int64_t)((r + 3) % 8) * g.ns; }
    RankDesc *d_rd; (void)hipMalloc(&d_rd, sizeof(RankDesc) * 8);
    (void)hipMemcpy(d_rd, rd.data(), sizeof(RankDesc) * 8, hipMemcpyHostToDevice);
    (void)init_kernel_attributes();
    int64_t *out; (void)hipMalloc(&out, sizeof(int64_t) * 8 * g.ns);
    uint32_t *val[4];
    for (int i = 0; i < 4; i++) (void)hipMalloc(&val[i], v2_val_bytes(g, 8));
    hipEvent_t evG[4];
    for (int i = 0; i < 4; i++) (void)hipEventCreateWithFlags(&evG[i], hipEventDisableTiming);
    int lo = 0, hi = 0;
    (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
    hipStream_t sA, sB;
    (void)hipStreamCreateWithPriority(&sA, hipStreamNonBlocking, lo);
    (void)hipStreamCreateWithPriority(&sB, hipStreamNonBlocking, hi);
    hipEvent_t evA[2], evB[2], t0, t1;
    for (int i = 0; i < 2; i++) { (void)hipEventCreateWithFlags(&evA[i], hipEventDisableTiming); (void)hipEventCreateWithFlags(&evB[i], hipEventDisableTiming); }
    (void)hipEventCreate(&t0); (void)hipEventCreate(&t1);
    const int E = 20;
    for (int mode = 0; mode < 6; mode++) {
        for (int rep = 0; rep < 2; rep++) {
            (void)hipDeviceSynchronize();
            (void)hipEventRecord(t0, sB);
            (void)hipStreamWaitEvent(sA, t0, 0);
            for (int e = 0; e < E; e++) {
                g.key0 = 0x1234u + e; g.key1 = 0x9abcu ^ e;
                const int p = e & 1;
                if (mode >= 3) {
                    // within one epoch: rank groups, group k+1's last-occurrence pass beside group
                    // k's replay; the next epoch starts after this one's last replay
                    const int ng = mode == 3 ? 2 : (mode == 4 ? 4 : 1), per = 8 / ng;
                    if (e > 0) (void)hipStreamWaitEvent(sA, evB[0], 0);
                    for (int k = 0; k < ng; k++) {
                        launch_v2(g, d_rd, k * per, per, 0, g.ns, out + (int64_t)k * per * g.ns, val[k], nullptr, nullptr, nullptr, sA, Marker(), EMIT_XCHG, V2_STAGE_PRE);
                        (void)hipEventRecord(evG[k], sA);
                    }
                    for (int k = 0; k < ng; k++) {
                        (void)hipStreamWaitEvent(sB, evG[k], 0);
                        launch_v2(g, d_rd, k * per, per, 0, g.ns, out + (int64_t)k * per * g.ns, val[k], nullptr, nullptr, nullptr, sB, Marker(), EMIT_XCHG, V2_STAGE_EMIT);
                    }
                    (void)hipEventRecord(evB[0], sB);
                } else if (mode == 0) {
                    launch_v2(g, d_rd, 0, 8, 0, g.ns, out, val[p], nullptr, nullptr, nullptr, sB, Marker(), EMIT_XCHG, V2_STAGE_ALL);
                } else {
                    hipStream_t spre = mode == 1 ? sA : sB;
                    if (e >= 2 && mode == 1) (void)hipStreamWaitEvent(sA, evB[p], 0);
                    launch_v2(g, d_rd, 0, 8, 0, g.ns, out, val[p], nullptr, nullptr, nullptr, spre, Marker(), EMIT_XCHG, V2_STAGE_PRE);
                    (void)hipEventRecord(evA[p], spre);
                    (void)hipStreamWaitEvent(sB, evA[p], 0);
                    launch_v2(g, d_rd, 0, 8, 0, g.ns, out, val[p], nullptr, nullptr, nullptr, sB, Marker(), EMIT_XCHG, V2_STAGE_EMIT);
                    (void)hipEventRecord(evB[p], sB);
                }
            }
            (void)hipEventRecord(t1, sB);
            (void)hipEventSynchronize(t1);
            float ms = 0;
            (void)hipEventElapsedTime(&ms, t0, t1);
            printf("%s: %.1f us per epoch\n", mode == 0 ? "serial (ALL)" : mode == 1 ? "pipelined 2 streams (across epochs)" : mode == 2 ? "split, 1 stream" : mode == 3 ? "2 rank groups, 2 streams" : mode == 4 ? "4 rank groups, 2 streams" : "1 group, 2 streams", ms * 1e3 / E);
        }
    }
    return 0;
}
