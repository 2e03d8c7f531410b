// Device check: feistel4_uniform (keyed-carry / packed forms) == feistel_once, all half widths.
#include <cstdio>
#include <vector>
#include "../partiallyshuffledistributedsampler_amd/csrc/pss_device.h"
#include "../partiallyshuffledistributedsampler_amd/csrc/pss_v2grp.hip"
using namespace pss;
__global__ void k_check(uint32_t h, uint32_t seed, uint32_t *bad) {
    uint32_t K[6];
    for (int i = 0; i < 6; i++) K[i] = slot_hash(seed * 7 + i, 0x1234567u, 0x89ABCDEFu);
    const uint32_t n = 1u << (2 * h);
    const uint32_t base = (blockIdx.x * 64u + threadIdx.x) * 4u;
    uint32_t x[4], y[4];
    for (int c = 0; c < 4; c++) x[c] = (base + c) & (n - 1u);
    if (h <= 8) feistel4_uniform<true>(x, h, K, y); else feistel4_uniform<false>(x, h, K, y);
    for (int c = 0; c < 4; c++) {
        const uint32_t z = feistel_once(x[c], h, K);
        if (y[c] != z) {
            const uint32_t i = atomicAdd(bad, 1u);
            if (i < 4) { bad[1 + 3 * i] = x[c]; bad[2 + 3 * i] = y[c]; bad[3 + 3 * i] = z; }
        }
    }
}
int main() {
    uint32_t *d; (void)hipMalloc(&d, 64);
    for (uint32_t h = 1; h <= 15; h++) {
        (void)hipMemset(d, 0, 64);
        hipLaunchKernelGGL(k_check, dim3(4096), dim3(64), 0, 0, h, h, d);
        uint32_t b[16] = {0}; (void)hipMemcpy(b, d, 64, hipMemcpyDeviceToHost);
        uint32_t K[6];
        for (int i = 0; i < 6; i++) K[i] = slot_hash(h * 7 + i, 0x1234567u, 0x89ABCDEFu);
        printf("h=%u bad=%u", h, b[0]);
        for (int i = 0; i < 2 && i < (int)b[0]; i++)
            printf("  [x=%u uni=%u once=%u host_once=%u]", b[1 + 3 * i], b[2 + 3 * i], b[3 + 3 * i], feistel_once(b[1 + 3 * i], h, K));
        printf("\n");
    }
    return 0;
}
