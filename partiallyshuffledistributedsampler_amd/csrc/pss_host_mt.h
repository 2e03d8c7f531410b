// pss_host_mt.h -- CPython 3.10's `random` (MT19937) on the host: the file-order / block
// permutations of init_iter (pss_runtime.cpp) and the CPU mode's exact-order streams
// (pss_cpu.cpp) need the reference's own draws bit for bit.
#pragma once
#include <stdint.h>

namespace pss {

// ------------------------------------------------------------------------------------------
// CPython 3.10 `random` (MT19937): seed(int) = init_by_array over the 32-bit words of
// abs(seed); shuffle = Fisher-Yates with _randbelow_with_getrandbits (random.py:239-249,
// 380-396).  The file-order and block permutations pin the file->rank assignment, so they
// must match the reference exactly.
// ------------------------------------------------------------------------------------------
class CPythonMT {
  public:
    void seed(int64_t a) {
        uint64_t m = a < 0 ? (uint64_t)(-(a + 1)) + 1u : (uint64_t)a;
        uint32_t key[2] = {(uint32_t)m, (uint32_t)(m >> 32)};
        init_by_array(key, key[1] ? 2 : 1);
    }
    uint32_t next() {
        if (__builtin_expect(mti_ >= kN, 0)) twist();
        return out_[mti_++];
    }
    // random.py:239-249 (_randbelow_with_getrandbits): k = n.bit_length(), draw getrandbits(k)
    // (the top k bits of one 32-bit output) until below n
    uint32_t randbelow(uint32_t n) {  // n < 2^32
        if (n == 0) return 0;
        const int sh = __builtin_clz(n);                 // 32 - k
        uint32_t r;
        do { r = next() >> sh; } while (r >= n);
        return r;
    }
    template <typename T>
    void shuffle(T *x, int64_t n) {   // random.py:380-396
        for (int64_t i = n - 1; i >= 1; i--) {
            const int64_t j = randbelow((uint32_t)(i + 1));
            const T t = x[i]; x[i] = x[j]; x[j] = t;
        }
    }

  private:
    static constexpr int kN = 624, kM = 397;
    uint32_t mt_[kN];
    uint32_t out_[kN];   // tempered outputs of the current block
    int mti_ = kN + 1;

    void init_genrand(uint32_t s) {
        mt_[0] = s;
        for (int i = 1; i < kN; i++) mt_[i] = 1812433253u * (mt_[i - 1] ^ (mt_[i - 1] >> 30)) + (uint32_t)i;
        mti_ = kN;
    }
    void init_by_array(const uint32_t *key, int klen) {
        init_genrand(19650218u);
        int i = 1, j = 0;
        for (int k = kN > klen ? kN : klen; k; k--) {
            mt_[i] = (mt_[i] ^ ((mt_[i - 1] ^ (mt_[i - 1] >> 30)) * 1664525u)) + key[j] + (uint32_t)j;
            i++; j++;
            if (i >= kN) { mt_[0] = mt_[kN - 1]; i = 1; }
            if (j >= klen) j = 0;
        }
        for (int k = kN - 1; k; k--) {
            mt_[i] = (mt_[i] ^ ((mt_[i - 1] ^ (mt_[i - 1] >> 30)) * 1566083941u)) - (uint32_t)i;
            i++;
            if (i >= kN) { mt_[0] = mt_[kN - 1]; i = 1; }
        }
        mt_[0] = 0x80000000u;
        mti_ = kN;
    }
    void twist() {
        static const uint32_t mag01[2] = {0u, 0x9908b0dfu};
        int kk = 0;
        uint32_t y;
        for (; kk < kN - kM; kk++) {
            y = (mt_[kk] & 0x80000000u) | (mt_[kk + 1] & 0x7fffffffu);
            mt_[kk] = mt_[kk + kM] ^ (y >> 1) ^ mag01[y & 1u];
        }
        for (; kk < kN - 1; kk++) {
            y = (mt_[kk] & 0x80000000u) | (mt_[kk + 1] & 0x7fffffffu);
            mt_[kk] = mt_[kk + (kM - kN)] ^ (y >> 1) ^ mag01[y & 1u];
        }
        y = (mt_[kN - 1] & 0x80000000u) | (mt_[0] & 0x7fffffffu);
        mt_[kN - 1] = mt_[kM - 1] ^ (y >> 1) ^ mag01[y & 1u];
        for (int i = 0; i < kN; i++) {   // temper the whole block at once (vectorises)
            uint32_t t = mt_[i];
            t ^= t >> 11;
            t ^= (t << 7) & 0x9d2c5680u;
            t ^= (t << 15) & 0xefc60000u;
            t ^= t >> 18;
            out_[i] = t;
        }
        mti_ = 0;
    }
};

}  // namespace pss
