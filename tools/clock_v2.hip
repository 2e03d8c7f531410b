// clock_v2.hip -- diagnostic (-DPSS_STAMPS build): in-kernel shader clock of the V2 replay,
// back to back vs with idle gaps: clock = d(s_memtime) / d(s_memrealtime) * 100 MHz per wave.
#include "../partiallyshuffledistributedsampler_amd/csrc/pss_v2.hip"
#include <cstdio>
#include <vector>
#include <unistd.h>

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
        for (int b = 0; b < 2048; b++) { clk += (double)st[(size_t)b * 8]; rt += (double)st[(size_t)b * 8 + 1]; }
        printf("%s: mean wave %.1f us, shader clock %.2f GHz\n", mode ? "300us gaps" : "back-to-back", rt / 2048 / 100.0,
               clk / rt * 0.1);
    }
    return 0;
}
