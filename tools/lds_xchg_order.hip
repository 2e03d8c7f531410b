// lds_xchg_order.hip -- does one ds_wrxchg_rtn_b32 whose lanes hit the same LDS word behave like
// the lanes exchanging one after another in ascending lane order (lane l gets what the highest
// lower lane on that word wrote, the lowest gets the old word, the word ends with the highest
// lane's value)?  Random slot patterns over several table sizes; counts mismatches against that
// sequential model.  Build: hipcc --offload-arch=gfx950 -O3 -o build/lds_xchg_order tools/lds_xchg_order.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ uint32_t h32(uint32_t x) {
    x ^= x >> 16; x *= 0x21F0AAADu; x ^= x >> 15; x *= 0x735A2D97u; x ^= x >> 15; return x;
}

template <int P>
__global__ __launch_bounds__(64) void k(int iters, unsigned long long *bad, unsigned long long *coll) {
    __shared__ uint32_t buf[P];
    __shared__ uint32_t model[P];
    const int lane = threadIdx.x;
    for (int s = lane; s < P; s += 64) { buf[s] = 0xF0000000u | s; model[s] = 0xF0000000u | s; }
    __syncthreads();
    unsigned long long nbad = 0, ncoll = 0;
    for (int it = 0; it < iters; it++) {
        const uint32_t u = h32((blockIdx.x * 977u + it) * 64u + lane);
        const uint32_t kslot = (uint32_t)(((uint64_t)u * P) >> 32);
        const uint32_t ins = (blockIdx.x << 20) ^ (it << 6) ^ lane;
        const uint32_t got = atomicExch(&buf[kslot], ins);
        __syncthreads();
        // sequential model by lane 0
        uint32_t expect = 0;
        for (int l = 0; l < 64; l++) {
            const uint32_t kl = __shfl(kslot, l);
            const uint32_t il = __shfl(ins, l);
            uint32_t old = 0;
            if (lane == 0) { old = model[kl]; model[kl] = il; }
            old = __shfl(old, 0);
            if (lane == l) expect = old;
        }
        __syncthreads();
        nbad += got != expect;
        // collisions in this batch (lanes sharing a slot with a lower lane)
        int c = 0;
        for (int l = 0; l < lane; l++) c |= __shfl(kslot, l) == kslot;
        ncoll += c;
    }
    atomicAdd(bad, nbad);
    atomicAdd(coll, ncoll);
}

template <int P>
void run(int blocks, int iters) {
    unsigned long long *d, h[2];
    hipMalloc(&d, 16); hipMemset(d, 0, 16);
    hipLaunchKernelGGL(k<P>, dim3(blocks), dim3(64), 0, 0, iters, d, d + 1);
    hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
    printf("P=%5d lane-steps=%llu colliding-lanes=%llu mismatches=%llu\n", P,
           (unsigned long long)blocks * iters * 64, h[1], h[0]);
    hipFree(d);
}

int main() {
    run<64>(512, 400);
    run<256>(512, 400);
    run<4096>(512, 400);
    return 0;
}
