/*
 * pss_oracle.c -- TEST INFRASTRUCTURE ONLY.  CPU restatement of the reference sampler's
 * index-generation path, used as the *checker* by tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py.  Nothing in the product links, loads or calls this file.
 *
 * Two families live here:
 *
 *  (1) "exact": a plain-C restatement of the reference algorithm, bit-for-bit, including the
 *      CPython 3.10 `random` module (MT19937) it depends on.  The MT code follows the
 *      published CPython 3.10.12 `_randommodule.c` algorithm (init_genrand, init_by_array,
 *      genrand_uint32, random_seed) and `/usr/lib/python3.10/random.py:239-249`
 *      (_randbelow_with_getrandbits), `:375-378` (choice), `:380-396` (shuffle).
 *      Pinned by tests/golden/mt_kats.json and the v1_xxx / v2_xxx fixtures, which were generated
 *      by running the reference itself (tools/gen_golden.py).
 *
 *  (2) "philox": the C twin of the counter-based schedule the HIP kernels implement
 *      (DESIGN.md §3).  The GPU must match it bit-for-bit; it shares the reference's
 *      multiset/assignment semantics (checked against (1)) but not its within-pool order.
 *
 * Build: see oracle/Makefile (gcc -O2 -shared -fPIC).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>

/* ------------------------------------------------------------------------------------ */
/* (1a) CPython MT19937                                                                  */
/* ------------------------------------------------------------------------------------ */
#define MT_N 624
#define MT_M 397

typedef struct { uint32_t mt[MT_N]; int mti; } orc_mt;

static void mt_init_genrand(orc_mt *s, uint32_t seed) {
    s->mt[0] = seed;
    for (int i = 1; i < MT_N; i++)
        s->mt[i] = 1812433253U * (s->mt[i - 1] ^ (s->mt[i - 1] >> 30)) + (uint32_t)i;
    s->mti = MT_N;
}

static void mt_init_by_array(orc_mt *s, const uint32_t *key, size_t klen) {
    mt_init_genrand(s, 19650218U);
    size_t i = 1, j = 0;
    size_t k = (MT_N > klen ? MT_N : klen);
    for (; k; k--) {
        s->mt[i] = (s->mt[i] ^ ((s->mt[i - 1] ^ (s->mt[i - 1] >> 30)) * 1664525U)) + key[j] +
                   (uint32_t)j;
        i++; j++;
        if (i >= MT_N) { s->mt[0] = s->mt[MT_N - 1]; i = 1; }
        if (j >= klen) j = 0;
    }
    for (k = MT_N - 1; k; k--) {
        s->mt[i] = (s->mt[i] ^ ((s->mt[i - 1] ^ (s->mt[i - 1] >> 30)) * 1566083941U)) -
                   (uint32_t)i;
        i++;
        if (i >= MT_N) { s->mt[0] = s->mt[MT_N - 1]; i = 1; }
    }
    s->mt[0] = 0x80000000U;
    s->mti = MT_N;
}

uint32_t orc_mt_u32(orc_mt *s) {
    static const uint32_t mag01[2] = {0x0U, 0x9908b0dfU};
    uint32_t y;
    if (s->mti >= MT_N) {
        int kk;
        for (kk = 0; kk < MT_N - MT_M; kk++) {
            y = (s->mt[kk] & 0x80000000U) | (s->mt[kk + 1] & 0x7fffffffU);
            s->mt[kk] = s->mt[kk + MT_M] ^ (y >> 1) ^ mag01[y & 0x1U];
        }
        for (; kk < MT_N - 1; kk++) {
            y = (s->mt[kk] & 0x80000000U) | (s->mt[kk + 1] & 0x7fffffffU);
            s->mt[kk] = s->mt[kk + (MT_M - MT_N)] ^ (y >> 1) ^ mag01[y & 0x1U];
        }
        y = (s->mt[MT_N - 1] & 0x80000000U) | (s->mt[0] & 0x7fffffffU);
        s->mt[MT_N - 1] = s->mt[MT_M - 1] ^ (y >> 1) ^ mag01[y & 0x1U];
        s->mti = 0;
    }
    y = s->mt[s->mti++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680U;
    y ^= (y << 15) & 0xefc60000U;
    y ^= (y >> 18);
    return y;
}

/* random.seed(a) for an int a: key = 32-bit little-endian words of abs(a) (CPython
 * random_seed; keyused = max(1, ceil(bits/32))).  Words are passed in by the caller so
 * arbitrarily large Python ints work; orc_mt_seed_i64 covers the int64 seeds the
 * reference actually produces (epoch + k, epoch + buffers*10000). */
void orc_mt_seed_words(orc_mt *s, const uint32_t *words, int64_t nwords) {
    uint32_t zero = 0;
    while (nwords > 1 && words[nwords - 1] == 0) nwords--;
    if (nwords <= 0) { words = &zero; nwords = 1; }
    mt_init_by_array(s, words, (size_t)nwords);
}

void orc_mt_seed_i64(orc_mt *s, int64_t a) {
    uint64_t m = a < 0 ? (uint64_t)(-(a + 1)) + 1u : (uint64_t)a;
    uint32_t w[2] = {(uint32_t)m, (uint32_t)(m >> 32)};
    orc_mt_seed_words(s, w, w[1] ? 2 : 1);
}

static int bit_length_u64(uint64_t n) { int k = 0; while (n) { k++; n >>= 1; } return k; }

/* random.py:239-249, restricted to n < 2**32 (every list the reference shuffles). */
uint64_t orc_mt_randbelow(orc_mt *s, uint64_t n) {
    if (!n) return 0;
    int k = bit_length_u64(n);
    uint64_t r;
    if (k <= 32) {
        do { r = orc_mt_u32(s) >> (32 - k); } while (r >= n);
    } else { /* getrandbits(k>32): words little-endian, top word masked (CPython) */
        do {
            uint64_t lo = orc_mt_u32(s);
            uint64_t hi = orc_mt_u32(s) >> (64 - k);
            r = lo | (hi << 32);
        } while (r >= n);
    }
    return r;
}

/* random.py:380-396 */
void orc_mt_shuffle_i64(orc_mt *s, int64_t *x, int64_t n) {
    for (int64_t i = n - 1; i >= 1; i--) {
        int64_t j = (int64_t)orc_mt_randbelow(s, (uint64_t)(i + 1));
        int64_t t = x[i]; x[i] = x[j]; x[j] = t;
    }
}
void orc_mt_shuffle_i32(orc_mt *s, int32_t *x, int64_t n) {
    for (int64_t i = n - 1; i >= 1; i--) {
        int64_t j = (int64_t)orc_mt_randbelow(s, (uint64_t)(i + 1));
        int32_t t = x[i]; x[i] = x[j]; x[j] = t;
    }
}

orc_mt *orc_mt_new(void) { orc_mt *s = (orc_mt *)calloc(1, sizeof(orc_mt)); orc_mt_seed_i64(s, 0); return s; }
void orc_mt_free(orc_mt *s) { free(s); }

/* seed(a); shuffle(x) -- the idiom of V1:114-119 and V2:143-146 */
void orc_seeded_shuffle_i32(int64_t seed, int32_t *x, int64_t n) {
    orc_mt s; orc_mt_seed_i64(&s, seed); orc_mt_shuffle_i32(&s, x, n);
}

/* ------------------------------------------------------------------------------------ */
/* (1b) partition math -- V1:42 `int(math.ceil(N * 1.0 / R))` evaluated in IEEE doubles   */
/* ------------------------------------------------------------------------------------ */
int64_t orc_num_samples(int64_t N, int64_t R) {
    double q = (double)N / (double)R;
    return (int64_t)ceil(q);
}

/* ------------------------------------------------------------------------------------ */
/* (1c) exact reference streams                                                          */
/* ------------------------------------------------------------------------------------ */
static inline int64_t wrap_id(int64_t id, int64_t N) { return id >= N ? id - N : id; }

/* V1 stream of one rank: V1:102,114-115 (window 0, seed(epoch)) and V1:157-172 (windows
 * b>=1, seed(epoch + b*10000)).  `resume_pos` >= 0 reproduces find_ckpt_position
 * (V1:134-140): the window holding resume_pos is left UNshuffled (the reference's lossy
 * resume) and generation starts at resume_pos.  Returns the number of ids written, or -1
 * where the reference itself would raise IndexError. */
int64_t orc_v1_exact_stream(int64_t epoch, int64_t start, int64_t ns, int64_t B, int64_t N,
                            int shuffle, int64_t resume_pos, int64_t *out) {
    orc_mt s;
    int64_t *ids = (int64_t *)malloc(sizeof(int64_t) * (size_t)(B > 0 ? B : 1));
    int64_t buffers = 0, pos = 0, len, n_out = 0;
    if (resume_pos < 0) {
        len = B < ns ? B : ns;
        for (int64_t i = 0; i < len; i++) ids[i] = i;
        if (shuffle) { orc_mt_seed_i64(&s, epoch); orc_mt_shuffle_i64(&s, ids, len); }
    } else {
        buffers = resume_pos / B;
        len = ns - buffers * B; if (len > B) len = B; if (len < 0) len = 0;
        for (int64_t i = 0; i < len; i++) ids[i] = i;
        pos = resume_pos - buffers * B;
        if (len > 0 && pos >= len) { free(ids); return -1; }
    }
    while (len > 0) {
        out[n_out++] = wrap_id(ids[pos] + B * buffers + start, N);
        pos++;
        if (pos >= len) {
            buffers++;
            len = ns - buffers * B; if (len > B) len = B; if (len < 0) len = 0;
            for (int64_t i = 0; i < len; i++) ids[i] = i;
            if (shuffle) { orc_mt_seed_i64(&s, epoch + buffers * 10000); orc_mt_shuffle_i64(&s, ids, len); }
            pos = 0;
        }
    }
    free(ids);
    return n_out;
}

/* V2 stream of one rank: pools seeded from the OLD start (V2:135-138), MT reseeded with
 * seed(epoch+2) at the end of init_iter (V2:147), then get_index (V2:96-116): choice +
 * list.remove from pool1, choice + remove from pool2 appended to pool1, reseed
 * seed(epoch + buffers*10000) and refill pool2 from the NEW start whenever it empties.
 * `skip` ids are drawn and discarded first (find_ckpt_position replay, V2:118-122). */
static int64_t v2_exact(int64_t epoch, int64_t old_start, int64_t new_start, int64_t ns,
                        int64_t B, int64_t N, int64_t skip, int64_t limit, int64_t *out) {
    orc_mt s;
    int64_t cap = B > 0 ? B : 1;
    int64_t *p1 = (int64_t *)malloc(sizeof(int64_t) * (size_t)(cap + 1));
    int64_t *p2 = (int64_t *)malloc(sizeof(int64_t) * (size_t)cap);
    int64_t n1 = 0, n2 = 0, buffers = 0, n_out = 0, drawn = 0;
    int64_t e1 = old_start + (B < ns ? B : ns);
    for (int64_t v = old_start; v < e1; v++) p1[n1++] = v;
    int64_t e2 = old_start + 2 * B; if (e2 > old_start + ns) e2 = old_start + ns;
    for (int64_t v = old_start + B; v < e2; v++) p2[n2++] = v;
    orc_mt_seed_i64(&s, epoch + 2);
    while (n1 > 0 || n2 > 0) {
        int64_t k = (int64_t)orc_mt_randbelow(&s, (uint64_t)n1);
        if (n1 == 0) break; /* choice([]) raises IndexError in the reference */
        int64_t index = p1[k];
        memmove(p1 + k, p1 + k + 1, sizeof(int64_t) * (size_t)(n1 - k - 1));
        n1--;
        if (n2 != 0) {
            int64_t k2 = (int64_t)orc_mt_randbelow(&s, (uint64_t)n2);
            int64_t index2 = p2[k2];
            memmove(p2 + k2, p2 + k2 + 1, sizeof(int64_t) * (size_t)(n2 - k2 - 1));
            n2--;
            p1[n1++] = index2;
        }
        if (n2 == 0) {
            orc_mt_seed_i64(&s, epoch + buffers * 10000);
            buffers++;
            int64_t lo = new_start + (buffers + 1) * B;
            int64_t hi = new_start + (buffers + 2) * B;
            if (hi > new_start + ns) hi = new_start + ns;
            for (int64_t v = lo; v < hi; v++) p2[n2++] = v;
        }
        if (drawn++ >= skip) out[n_out++] = wrap_id(index, N);
        if (limit >= 0 && n_out >= limit) break;
    }
    free(p1); free(p2);
    return n_out;
}

int64_t orc_v2_exact_stream(int64_t epoch, int64_t old_start, int64_t new_start, int64_t ns,
                            int64_t B, int64_t N, int64_t skip, int64_t *out) {
    return v2_exact(epoch, old_start, new_start, ns, B, N, skip, -1, out);
}

/* the first `limit` ids only (bench.py's bounded cpu_baseline sample) */
int64_t orc_v2_exact_prefix(int64_t epoch, int64_t old_start, int64_t new_start, int64_t ns,
                            int64_t B, int64_t N, int64_t limit, int64_t *out) {
    return v2_exact(epoch, old_start, new_start, ns, B, N, 0, limit, out);
}

/* ------------------------------------------------------------------------------------ */
/* (1d) the same V2 stream for big pools: rank-select bitmaps instead of list.remove      */
/* ------------------------------------------------------------------------------------ */
/* A Python list that only ever loses elements by position and gains them at its end is a
 * bitmap over its insertion slots: element k of the list is the k-th set bit.  The bitmap
 * keeps a 64-ary tree of set-bit counts above its words (node i of level l covers words
 * [i*64^(l+1), (i+1)*64^(l+1))), so select / clear / append cost O(64 log_64 n) instead of
 * list.remove's O(n) shift.  This is the whole of the speed-up: orc_v2_exact_stream_rs
 * performs exactly the draws, reseeds and refills of v2_exact above (V2:96-116), and
 * tests/test_oracle_golden.py checks the two against each other and against the goldens. */
typedef struct {
    int64_t nwords;
    uint64_t *w;
    int nlev;
    int64_t len[8];
    uint32_t *cnt[8];
} orc_rsb;

static void rsb_init(orc_rsb *b, int64_t nbits) {
    memset(b, 0, sizeof(*b));
    b->nwords = (nbits + 63) / 64;
    if (b->nwords < 1) b->nwords = 1;
    b->w = (uint64_t *)calloc((size_t)b->nwords, sizeof(uint64_t));
    int64_t n = b->nwords;
    do {
        n = (n + 63) / 64;
        b->len[b->nlev] = n;
        b->cnt[b->nlev] = (uint32_t *)calloc((size_t)n, sizeof(uint32_t));
        b->nlev++;
    } while (n > 1);
}

static void rsb_free(orc_rsb *b) {
    free(b->w);
    for (int l = 0; l < b->nlev; l++) free(b->cnt[l]);
}

/* bits [0, n) set, the rest clear (a fresh list(range(lo, lo + n))) */
static void rsb_fill(orc_rsb *b, int64_t n) {
    memset(b->w, 0, sizeof(uint64_t) * (size_t)b->nwords);
    for (int l = 0; l < b->nlev; l++) memset(b->cnt[l], 0, sizeof(uint32_t) * (size_t)b->len[l]);
    for (int64_t i = 0; i < n / 64; i++) b->w[i] = ~0ull;
    if (n % 64) b->w[n / 64] = (1ull << (n % 64)) - 1ull;
    for (int64_t i = 0; i < b->nwords; i++) b->cnt[0][i / 64] += (uint32_t)__builtin_popcountll(b->w[i]);
    for (int l = 1; l < b->nlev; l++)
        for (int64_t i = 0; i < b->len[l - 1]; i++) b->cnt[l][i / 64] += b->cnt[l - 1][i];
}

static void rsb_add(orc_rsb *b, int64_t pos, int delta) {
    int64_t node = pos / 64;
    for (int l = 0; l < b->nlev; l++) {
        node /= 64;
        b->cnt[l][node] = (uint32_t)((int64_t)b->cnt[l][node] + delta);
    }
}

static void rsb_set(orc_rsb *b, int64_t pos) {
    b->w[pos / 64] |= 1ull << (pos % 64);
    rsb_add(b, pos, 1);
}

static void rsb_clear(orc_rsb *b, int64_t pos) {
    b->w[pos / 64] &= ~(1ull << (pos % 64));
    rsb_add(b, pos, -1);
}

/* position of the k-th set bit (k counted from 0; k < number of set bits) */
static int64_t rsb_select(const orc_rsb *b, int64_t k) {
    int64_t node = 0;                       /* the root: the single node of the top level */
    for (int l = b->nlev - 2; l >= 0; l--) {
        int64_t c = node * 64, e = c + 64 < b->len[l] ? c + 64 : b->len[l];
        while (c < e - 1 && (int64_t)b->cnt[l][c] <= k) { k -= b->cnt[l][c]; c++; }
        node = c;
    }
    int64_t wi = node * 64, we = wi + 64 < b->nwords ? wi + 64 : b->nwords;
    for (;;) {
        const int64_t pc = __builtin_popcountll(b->w[wi]);
        if (k < pc || wi == we - 1) break;
        k -= pc;
        wi++;
    }
    uint64_t x = b->w[wi];
    for (; k > 0; k--) x &= x - 1ull;
    return wi * 64 + __builtin_ctzll(x);
}

static int64_t v2_exact_rs(int64_t epoch, int64_t old_start, int64_t new_start, int64_t ns,
                           int64_t B, int64_t N, int64_t skip, int64_t limit, int64_t *out) {
    orc_mt s;
    /* pool1: insertion slots [0, P) hold old_start + slot (V2:135-136); every append takes the
     * next slot, at most one per step */
    const int64_t P = B < ns ? B : ns;
    const int64_t cap1 = ns + 1;
    int64_t *val1 = (int64_t *)malloc(sizeof(int64_t) * (size_t)cap1);
    orc_rsb p1, p2;
    rsb_init(&p1, cap1);
    rsb_init(&p2, B > 0 ? B : 1);
    for (int64_t v = 0; v < P; v++) val1[v] = old_start + v;
    rsb_fill(&p1, P);
    int64_t n1 = P, next1 = P;
    /* pool2: the window list(range(lo2, hi2)) (V2:137-138, then V2:110-112) */
    int64_t lo2 = old_start + B, hi2 = old_start + 2 * B;
    if (hi2 > old_start + ns) hi2 = old_start + ns;
    int64_t n2 = hi2 > lo2 ? hi2 - lo2 : 0;
    rsb_fill(&p2, n2);
    int64_t buffers = 0, n_out = 0, drawn = 0;
    orc_mt_seed_i64(&s, epoch + 2);                              /* V2:147 */
    while (n1 > 0 || n2 > 0) {
        const int64_t k = (int64_t)orc_mt_randbelow(&s, (uint64_t)n1);   /* V2:101 */
        if (n1 == 0) break;
        const int64_t slot = rsb_select(&p1, k);
        const int64_t index = val1[slot];
        rsb_clear(&p1, slot);                                    /* V2:102 */
        n1--;
        if (n2 != 0) {                                           /* V2:103-106 */
            const int64_t k2 = (int64_t)orc_mt_randbelow(&s, (uint64_t)n2);
            const int64_t j = rsb_select(&p2, k2);
            rsb_clear(&p2, j);
            n2--;
            val1[next1] = lo2 + j;
            rsb_set(&p1, next1);
            next1++;
            n1++;
        }
        if (n2 == 0) {                                           /* V2:107-112 */
            orc_mt_seed_i64(&s, epoch + buffers * 10000);
            buffers++;
            lo2 = new_start + (buffers + 1) * B;
            hi2 = new_start + (buffers + 2) * B;
            if (hi2 > new_start + ns) hi2 = new_start + ns;
            n2 = hi2 > lo2 ? hi2 - lo2 : 0;
            if (n2) rsb_fill(&p2, n2);
        }
        if (drawn++ >= skip) out[n_out++] = wrap_id(index, N);   /* V2:113-115 */
        if (limit >= 0 && n_out >= limit) break;
    }
    free(val1);
    rsb_free(&p1);
    rsb_free(&p2);
    return n_out;
}

int64_t orc_v2_exact_stream_rs(int64_t epoch, int64_t old_start, int64_t new_start, int64_t ns,
                               int64_t B, int64_t N, int64_t skip, int64_t *out) {
    return v2_exact_rs(epoch, old_start, new_start, ns, B, N, skip, -1, out);
}

/* ------------------------------------------------------------------------------------ */
/* (2) Philox schedule -- C twin of the HIP kernels                        */
/* ------------------------------------------------------------------------------------ */
#define PHILOX_M0 0xD2511F53U
#define PHILOX_M1 0xCD9E8D57U
#define PHILOX_W0 0x9E3779B9U
#define PHILOX_W1 0xBB67AE85U
enum { DOM_V1_WIN = 1, DOM_V2_SLOT = 2, DOM_V2_INS = 3, DOM_V2_TAIL = 4, DOM_V2_INIT = 5 };

void orc_philox4x32(const uint32_t ctr_in[4], uint64_t key64, uint32_t out[4]) {
    uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
    uint32_t k0 = (uint32_t)key64, k1 = (uint32_t)(key64 >> 32);
    for (int r = 0; r < 10; r++) {
        uint64_t p0 = (uint64_t)PHILOX_M0 * c0;
        uint64_t p1 = (uint64_t)PHILOX_M1 * c2;
        uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
        uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        c0 = n0; c1 = (uint32_t)p1; c2 = n2; c3 = (uint32_t)p0;
        k0 += PHILOX_W0; k1 += PHILOX_W1;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

uint64_t orc_mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

uint64_t orc_epoch_key(uint64_t seed, int64_t epoch) {
    return orc_mix64(orc_mix64(seed) ^ (uint64_t)epoch);
}

/* keyed bijection of [0,n): balanced Feistel on 2h bits + cycle walking.  Halves of h <= 5
 * bits (n <= 1024): 8 rounds of f = top h bits of murmur3 fmix32(R ^ k_i), k_i = rk[i % 6] +
 * i * 0x9E3779B9.  Wider halves, 6 rounds: h <= 10 -> top h bits of the low 16 bits of
 * (R ^ k) * 0x9E37; h > 10 -> bits [24 - h, 24) of ((R ^ k) mod 2^24) * 0x9E3779. */
static uint32_t orc_fmix32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x85EBCA6BU;
    x ^= x >> 13;
    x *= 0xC2B2AE35U;
    x ^= x >> 16;
    return x;
}

uint32_t orc_feistel(uint32_t x, uint32_t n, const uint32_t rk[6]) {
    if (n <= 1) return 0;
    int bits = 0; while ((1ull << bits) < (uint64_t)n) bits++;
    int h = (bits + 1) >> 1;
    uint32_t mask = (1u << h) - 1u;
    do {
        uint32_t L = x >> h, R = x & mask;
        if (h <= 5) {
            for (int i = 0; i < 8; i++) {
                uint32_t f = orc_fmix32(R ^ (rk[i % 6] + (uint32_t)i * 0x9E3779B9U)) >> (32 - h);
                uint32_t t = L ^ f;
                L = R; R = t;
            }
        } else {
            for (int i = 0; i < 6; i++) {
                uint32_t f = h <= 10 ? ((((R ^ rk[i]) * 0x9E37u) & 0xFFFFu) >> (16 - h))
                                    : (((((R ^ rk[i]) & 0xFFFFFFu) * 0x9E3779u) >> (24 - h)) & mask);
                uint32_t t = L ^ f;
                L = R; R = t;
            }
        }
        x = (L << h) | R;
    } while (x >= n);
    return x;
}

/* 8 key words: Philox blocks (c0, 0, c2, dom) and (c0, 1, c2, dom) under key64 */
static void orc_keys8(uint64_t key64, uint32_t c0, uint32_t c2, uint32_t dom, uint32_t k[8]) {
    uint32_t a[4] = {c0, 0, c2, dom}, b[4] = {c0, 1, c2, dom};
    orc_philox4x32(a, key64, k);
    orc_philox4x32(b, key64, k + 4);
}

/* V1 under the counter schedule: window w of the rank block is ordered by the keyed Feistel
 * bijection of [0, len_w) with round keys orc_keys8(w, rank, DOM_V1_WIN); id = start + w*B +
 * feistel_w(p) (wrap at N, V1:161-163).  Same multiset as orc_v1_exact_stream.  Positions
 * [pos_lo, pos_lo+count). */
int64_t orc_v1_philox_stream(uint64_t key64, uint32_t rank, int64_t start, int64_t ns,
                             int64_t B, int64_t N, int shuffle, int64_t pos_lo, int64_t count,
                             int64_t *out) {
    int64_t pos_hi = pos_lo + count; if (pos_hi > ns) pos_hi = ns;
    if (pos_lo >= pos_hi) return 0;
    int64_t n_out = 0;
    for (int64_t w = pos_lo / B; w * B < pos_hi; w++) {
        int64_t len = ns - w * B; if (len > B) len = B;
        uint32_t rk[8];
        if (shuffle) orc_keys8(key64, (uint32_t)w, rank, DOM_V1_WIN, rk);
        int64_t p0 = pos_lo > w * B ? pos_lo - w * B : 0;
        int64_t p1 = pos_hi - w * B < len ? pos_hi - w * B : len;
        for (int64_t p = p0; p < p1; p++) {
            int64_t y = shuffle ? (int64_t)orc_feistel((uint32_t)p, (uint32_t)len, rk) : p;
            out[n_out++] = wrap_id(start + w * B + y, N);
        }
    }
    return n_out;
}

/* V2 slot draw of step t (pss_common.h slot_hash): keyed 2-round multiply-xorshift mixer on
 * 24-bit operands, key = the first two words of Philox block (0, 0, rank, DOM_V2_SLOT). */
static inline uint32_t orc_slot_hash(uint32_t t, uint32_t s0, uint32_t s1) {
    uint32_t x = t ^ s0;
    x ^= x >> 16;
    x = (x & 0xFFFFFFu) * 0xA2F0ADu;
    x ^= x >> 15;
    x ^= s1;
    x = (x & 0xFFFFFFu) * 0x5A2D97u;
    x ^= x >> 15;
    return x;
}

/* P1 = 2^b, b <= 16: steps t and t + 64 of each 128-step block share the hash of index
 * (t >> 7) * 64 + (t & 63); step t takes the top b bits of the high half-word, t + 64 those of
 * the low half-word.  Other P1: one hash per step, multiply-shift scaled. */
static inline uint32_t v2_slot(const uint32_t sk[4], int64_t t, uint32_t P1) {
    if (P1 <= 65536u && (P1 & (P1 - 1u)) == 0u) {
        if (P1 == 1u) return 0u;
        int b = 0;
        while ((1u << b) < P1) b++;
        uint32_t tt = (uint32_t)t;
        uint32_t u = orc_slot_hash(((tt >> 7) << 6) | (tt & 63u), sk[0], sk[1]);
        if (tt & 64u) u <<= 16;
        return u >> (32 - b);
    }
    uint32_t u = orc_slot_hash((uint32_t)t, sk[0], sk[1]);
    return (uint32_t)(((uint64_t)u * P1) >> 32);
}

/* virtual index v in [0,ns) of one rank -> global id: the first two windows come from the
 * OLD start (V2:135-138), the rest from the NEW one (V2:110-112). */
static inline int64_t v2_vid_to_id(int64_t v, int64_t old_start, int64_t new_start, int64_t B,
                                   int64_t N) {
    return wrap_id((v < 2 * B ? old_start : new_start) + v, N);
}

/* Pools beyond LDS (P1 > 16384): grouped draws.  G = ceil(P1 / 4096) groups of consecutive
 * slots, q = P1 / G each plus one for the first P1 mod G; step t belongs to burst t / 32 and
 * that burst to group (t / 32) mod G (bursts of 16 up to schedule 3); u = the step's index inside its group's own stream.
 * The step draws uniformly inside its group: power-of-two groups pair sub-steps u and u + 64
 * (u mod 128 < 64) on one hash of the lower one's step (high / low half-word), other sizes
 * hash every step. */
#define ORC_LDS_SLOT_MAX 16384
#define ORC_BURST 32u
typedef struct { uint32_t G, q, r; } orc_groups;
static orc_groups orc_groups_of(uint32_t P1) {
    orc_groups gr; gr.G = (P1 + 4095u) / 4096u; gr.q = P1 / gr.G; gr.r = P1 % gr.G; return gr;
}
static uint32_t orc_gbase(orc_groups gr, uint32_t g) { return g * gr.q + (g < gr.r ? g : gr.r); }
static uint32_t orc_gsize(orc_groups gr, uint32_t g) { return gr.q + (g < gr.r ? 1u : 0u); }
static uint64_t orc_gstep(orc_groups gr, uint32_t g, uint64_t u) {
    return ((u / ORC_BURST) * gr.G + g) * ORC_BURST + u % ORC_BURST;
}
static inline uint32_t v2_slot_grouped(const uint32_t sk[4], int64_t t, uint32_t P1) {
    orc_groups gr = orc_groups_of(P1);
    uint32_t g = (uint32_t)(((uint64_t)t / ORC_BURST) % gr.G);
    uint32_t size = orc_gsize(gr, g);
    uint64_t u = ((uint64_t)t / ORC_BURST / gr.G) * ORC_BURST + (uint64_t)t % ORC_BURST;
    uint32_t local;
    if ((size & (size - 1u)) == 0u) {
        int b = 0; while ((1u << b) < size) b++;
        if (b == 0) local = 0;
        else if (u & 64u)
            local = (orc_slot_hash((uint32_t)orc_gstep(gr, g, u - 64u), sk[0], sk[1]) << 16) >> (32 - b);
        else
            local = orc_slot_hash((uint32_t)t, sk[0], sk[1]) >> (32 - b);
    } else {
        local = (uint32_t)(((uint64_t)orc_slot_hash((uint32_t)t, sk[0], sk[1]) * size) >> 32);
    }
    return orc_gbase(gr, g) + local;
}

/* Grouped tail: rounds in which every group emits its next (up to) ORC_BURST elements, groups in
 * order; group g's e-th element is slot orc_feistel(e, S_g, keys8(g, rank, DOM_V2_TAIL)) of
 * the group. */
static uint32_t orc_gtail_pos(orc_groups gr, uint32_t g, uint32_t e) {
    uint32_t full = gr.q / ORC_BURST;
    if (e < full * ORC_BURST) return (e / ORC_BURST) * ORC_BURST * gr.G + g * ORC_BURST + e % ORC_BURST;
    uint32_t c = gr.q % ORC_BURST;
    return full * ORC_BURST * gr.G + g * c + (g < gr.r ? g : gr.r) + (e - full * ORC_BURST);
}

/* V2 under the counter schedule (slot-replacement form of V2:96-116):
 *   P1 = min(B, ns) slots initialised with window 0 -- slot s holds s, or for grouped pools
 *   (P1 > 16384) the Feistel image of s keyed by orc_keys8(0, rank, DOM_V2_INIT); T = ns - P1
 *   steps; step t draws slot k_t (slot hash keyed by Philox DOM_V2_SLOT, grouped for big
 *   pools), emits buf[k_t] and stores the t-th inserted element there: window w = 1 + t/B,
 *   inserted in the order of the Feistel bijection keyed by orc_keys8(w, rank, DOM_V2_INS);
 *   then the final buffer is emitted in the order of the Feistel bijection of [0, P1) keyed by
 *   orc_keys8(0, rank, DOM_V2_TAIL) (grouped pools: the round-robin group drain above).
 * Writes all ns ids (rank order) to out; returns ns. */
int64_t orc_v2_philox_stream(uint64_t key64, uint32_t rank, int64_t old_start,
                             int64_t new_start, int64_t ns, int64_t B, int64_t N, int64_t *out) {
    int64_t P1 = B < ns ? B : ns;
    int64_t T = ns - P1;
    int grouped = P1 > ORC_LDS_SLOT_MAX;
    uint32_t *buf = (uint32_t *)malloc(sizeof(uint32_t) * (size_t)P1);
    if (grouped) {
        uint32_t ik[8];
        orc_keys8(key64, 0, rank, DOM_V2_INIT, ik);
        for (int64_t s = 0; s < P1; s++) buf[s] = orc_feistel((uint32_t)s, (uint32_t)P1, ik);
    } else {
        for (int64_t s = 0; s < P1; s++) buf[s] = (uint32_t)s;
    }
    int64_t cur_w = -1;
    uint32_t rk[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint32_t sk[4], skc[4] = {0, 0, rank, DOM_V2_SLOT};
    orc_philox4x32(skc, key64, sk);
    for (int64_t t = 0; t < T; t++) {
        uint32_t k = grouped ? v2_slot_grouped(sk, t, (uint32_t)P1) : v2_slot(sk, t, (uint32_t)P1);
        out[t] = v2_vid_to_id(buf[k], old_start, new_start, B, N);
        int64_t w = 1 + t / B, p = t % B;
        if (w != cur_w) {
            orc_keys8(key64, (uint32_t)w, rank, DOM_V2_INS, rk);
            cur_w = w;
        }
        int64_t len = ns - w * B; if (len > B) len = B;
        buf[k] = (uint32_t)(w * B + orc_feistel((uint32_t)p, (uint32_t)len, rk));
    }
    uint32_t tk[8];
    if (grouped) {
        orc_groups gr = orc_groups_of((uint32_t)P1);
        for (uint32_t g = 0; g < gr.G; g++) {
            uint32_t S = orc_gsize(gr, g), base = orc_gbase(gr, g);
            orc_keys8(key64, g, rank, DOM_V2_TAIL, tk);
            for (uint32_t e = 0; e < S; e++)
                out[T + orc_gtail_pos(gr, g, e)] =
                    v2_vid_to_id(buf[base + orc_feistel(e, S, tk)], old_start, new_start, B, N);
        }
    } else {
        orc_keys8(key64, 0, rank, DOM_V2_TAIL, tk);
        for (int64_t j = 0; j < P1; j++)
            out[T + j] = v2_vid_to_id(buf[orc_feistel((uint32_t)j, (uint32_t)P1, tk)], old_start,
                                      new_start, B, N);
    }
    free(buf);
    return ns;
}

/* the slot drawn at each step t < T of one rank's V2 stream (schedule-quality tests) */
void orc_v2_slots(uint64_t key64, uint32_t rank, int64_t P1, int64_t T, uint32_t *out) {
    uint32_t sk[4], skc[4] = {0, 0, rank, DOM_V2_SLOT};
    orc_philox4x32(skc, key64, sk);
    int grouped = P1 > ORC_LDS_SLOT_MAX;
    for (int64_t t = 0; t < T; t++)
        out[t] = grouped ? v2_slot_grouped(sk, t, (uint32_t)P1) : v2_slot(sk, t, (uint32_t)P1);
}

/* ------------------------------------------------------------------------------------ */
/* id -> (file position, offset) over an exclusive prefix of the shuffled file order      */
/* (V1:181-221 for ids below the scanned total; reflection is host-side semantics).       */
/* ------------------------------------------------------------------------------------ */
void orc_map(const int64_t *prefix, int64_t F, const int64_t *ids, int64_t n, int32_t *fpos,
             int64_t *off) {
    for (int64_t i = 0; i < n; i++) {
        int64_t lo = 0, hi = F; /* largest f with prefix[f] <= id, skipping empty files */
        int64_t id = ids[i];
        while (hi - lo > 1) {
            int64_t mid = (lo + hi) >> 1;
            if (prefix[mid] <= id) lo = mid; else hi = mid;
        }
        fpos[i] = (int32_t)lo;
        off[i] = id - prefix[lo];
    }
}

uint64_t orc_digest(const int64_t *ids, int64_t n) {
    uint64_t d = 0;
    for (int64_t i = 0; i < n; i++) d += orc_mix64((uint64_t)ids[i]);
    return d;
}

uint64_t orc_digest_range(int64_t lo, int64_t hi) {
    uint64_t d = 0;
    for (int64_t i = lo; i < hi; i++) d += orc_mix64((uint64_t)i);
    return d;
}
