// pss_v2split.h -- the draws of V2's long pool2 windows spread over the chip (order mode
// PSS_ORDER_EXACT; included by pss_v2exact.hip, which defines V2xGeo and v2x_tail_block).
//
// A window's draws (V2:101-106: k1 = _randbelow(P) and k2 = _randbelow(W - j) alternating) come
// from ONE freshly seeded MT19937 stream, and which word serves which draw depends on every
// rejection before it.  mt_draws_pair_wg (pss_mt.h) resolves a window on one CU: ~9.6 ms per
// 2^20-step window (C5), of which the word generation is a small part and the per-block work of
// the summaries / combine / emission the rest.  Here the generation stays serial (a workgroup per
// window, raw words to HBM, in chunks on a side stream) and the rest is split:
//
//   plan     (host, per window length) the window's words cut into SEGMENTS in PHASES, each
//            segment's length keeping the expected number of verdicts that differ over its
//            interval at about PSS_SPLIT_TARGET; the interval (sp_interval, on the device) is
//            the expected k2 index at the segment's word offset +- K standard deviations of the
//            renewal count, counted from the phase's ANCHOR (the exact state the previous phase's
//            walk ended in).  A phase ends where its intervals grow too wide, and ahead of every
//            power-of-two crossing of the bound W - j.
//   level 1  (one wave per segment and start role, the whole chip) the segment's transfer as a
//            function of its start index j over the interval: evaluated exactly at the low end of
//            a piece (pair_eval), it holds unchanged up to the largest shift of j under which no
//            k2 verdict changes (an accepted k2 word r at bound n stays accepted while n - d > r,
//            and no bound crosses a power of two) -- the rest of the piece is evaluated again.  So
//            a segment's transfer is a short list of pieces [a_p, a_{p+1}) -> (role, j + c_p).
//   walk     (one wave per window and phase) the segments in order from the exact anchor, 64 at
//            a time by guess and verify (a DPP scan of the pieces' transfers at guessed starts,
//            settled up to the first lane whose start lies in another piece); a segment whose
//            start falls outside its interval or whose pieces overflowed is run exactly.  The
//            walk's end anchors the next phase.  After the last phase the walk runs the rest of the
//            window exactly, emitting -- past the generated words from the stream's saved state.
//   emit     (one wave per segment) every segment again from its now known start, emitting draws.
// Each phase waits only for the generator chunk holding its last word.
// The pieces are exact, so the draws are the reference's whatever the intervals: a bad estimate
// only costs an exact run in the walk.
// V1's long windows (kV1: pss_v1exact.hip's Fisher-Yates draws j = _randbelow(n - d), V1:165-171)
// are the single-role case of the same machinery: every word serves a draw of bound n - d, the
// stream ends after n - 1 draws, the emission writes J[n - 1 - d], and k_v1x_sp_count counts the
// draws' buckets afterwards.
#pragma once
// (included inside namespace pss)

namespace {
constexpr int kSpPh = 10;       // phases (re-anchored intervals) before the exact remainder
constexpr int kSpPieces = 14;   // pieces kept per (segment, start role)
constexpr int kSpRec = 32;      // uint2 per segment record: pieces of role 0 | role 1, (lo, hi),
                                // (count role 0, count role 1), (q, L)
constexpr int kSpRecLoHi = 28, kSpRecCnt = 29, kSpRecQL = 30;
constexpr uint32_t kSpOver = 0xFFFFFFFFu;
constexpr double kSpCrossMargin = 300.0;   // a phase ends ahead of a crossing its intervals are wider than
#ifndef PSS_SPLIT_K
#define PSS_SPLIT_K 6.0      // interval margin in standard deviations (V2)
#endif
#ifndef PSS_SPLIT_K_V1
#define PSS_SPLIT_K_V1 4.0   // (V1; same-box sweeps, profiles/r06/exact_split/sweep.txt)
#endif
#ifndef PSS_SPLIT_TARGET
#define PSS_SPLIT_TARGET 2.0
#endif

struct V2xSpPlan {               // one window length
    const uint4 *seg;            // (q, L, -, -) per segment, phase after phase
    const float2 *mv;            // (expected words, their variance) to reach step 64 i, i <= W / 64 + 1
    uint32_t W, nph, nt, qend;   // k2 draws, phases, twists generated, first word of the remainder
    float K;                     // interval margin, standard deviations
    uint32_t ph[kSpPh + 1];      // first segment of each phase; ph[nph] = segments
};
struct V2xSp {
    V2xSpPlan pl[2];             // windows 0 .. S-2 (W = B), the last window
    uint32_t S, B, P, kb1, nsegmax;
    uint32_t nwp;                // words per window in `words`
    uint32_t *words;             // raw (untempered) MT words [window][nwp]
    uint2 *rec;                  // [window][nsegmax][kSpRec]
    uint2 *ss;                   // [window][nsegmax] start (role, j); role 2: the stream had ended
    uint32_t *anc;               // [window][kSpPh + 1][4]: (role, j, ended) at each phase's start
    uint32_t *K1, *K2;           // the slot's draws (V1: J [window][B] and the bucket counts [window][nbk])
    int64_t w0;                  // V1: the window of job 0
    uint32_t nbk;                // V1: buckets per window
};
template <bool kV1>
__device__ __forceinline__ uint32_t sp_nd(uint32_t W) { return kV1 ? (W ? W - 1u : 0u) : W; }   // draws of a stream

// one block of a stream exactly, emitting (the lanes below nval hold words): V2's pair_block, or
// V1's draw_block at draw i2 (bound W - d)
template <bool kV1, class Emit>
__device__ __forceinline__ void sp_block(uint32_t word, uint32_t nval, uint32_t W, uint32_t P, uint32_t kb1,
                                         uint32_t &st, uint32_t &i1, uint32_t &i2, Emit &emit) {
    if constexpr (kV1) {
        auto bound = [&](uint32_t d) { return W - d; };
        auto em = [&](uint32_t d, uint32_t r) { emit(true, d, r); };
        i2 += draw_block(word, (int)nval, i2, sp_nd<true>(W), bound, em);
    } else {
        pair_block(word, (uint32_t)(threadIdx.x & 63) < nval, W, P, kb1, st, i1, i2, emit);
    }
}
__device__ __forceinline__ const V2xSpPlan &sp_plan(const V2xSp &a, uint32_t s) {
    return a.pl[s + 1u == a.S ? 1 : 0];
}
__device__ __forceinline__ uint32_t sp_phases(const V2xSpPlan &pl) { return pl.nph ? pl.nph : 1u; }

// the wave's minimum, uniform: DPP row shifts and row broadcasts (lanes without a source keep
// ~0), then lane 63 -- no LDS round trip (a shuffle per step cost ~100 clocks each)
template <int CTRL, int ROWMASK>
__device__ __forceinline__ uint32_t dpp_min_step(uint32_t x) {
    const uint32_t y = (uint32_t)__builtin_amdgcn_update_dpp((int)0xFFFFFFFF, (int)x, CTRL, ROWMASK, 0xF, false);
    return y < x ? y : x;
}
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t x) {
    x = dpp_min_step<0x111, 0xF>(x);
    x = dpp_min_step<0x112, 0xF>(x);
    x = dpp_min_step<0x114, 0xF>(x);
    x = dpp_min_step<0x118, 0xF>(x);
    x = dpp_min_step<0x142, 0xA>(x);
    x = dpp_min_step<0x143, 0xC>(x);
    return (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
}

// pair_block's verdicts for one full block at one start (st, i2), without emitting: advances
// (st, i2) and returns in delta the largest d such that the block makes the same verdicts from
// (st, i2 + d) -- every k2 lane's index shifts by d: an accepted word r at bound n = W - j stays
// accepted while d < n - r, a rejected one stays rejected, and the bound keeps its bit length
// while d <= n - 2^(k-1)
__device__ __forceinline__ void pair_eval(uint32_t word, uint32_t W, uint32_t P, uint32_t kb1, uint32_t &st,
                                          uint32_t &i2, uint32_t &delta) {
    const int lane = threadIdx.x & 63;
    const uint64_t below = lanemask_lt();
    const bool a1 = (word >> (32u - kb1)) < P;
    uint32_t j = 0, role = 0, Fx = 0;
    bool a2 = false;
    auto pass = [&](uint32_t n2, uint32_t rr) {
        a2 = rr < n2;
        const uint32_t f = ((a1 != a2) ? 2u : 0u) | (a1 ? 1u : 0u);
        Fx = wave_role_scan(f);
        const uint32_t Fp = wave_prev_lane(Fx);
        role = lane ? role_apply(Fp, st) : st;
        const uint64_t m2 = __ballot(role == 1u && a2);
        j = i2 + (uint32_t)__popcll(m2 & below);
    };
    const uint32_t jl = i2 + ((uint32_t)lane + 1u) / 2u;
    const uint32_t nhi = i2 < W ? W - i2 : 1u, nlo = jl < W ? W - jl : 1u;
    const uint32_t kbh = 32u - (uint32_t)__builtin_clz(nhi);
    const uint32_t rh = word >> (32u - kbh);
    const bool sure = kbh == 32u - (uint32_t)__builtin_clz(nlo) && (rh < nlo || rh >= nhi);
    if (__ballot(!sure) == 0) {
        pass(nlo, rh);
    } else {
        uint32_t jg = i2 + (uint32_t)lane / 3u;
        for (;;) {
            const uint32_t n2 = jg < W ? W - jg : 1u;
            pass(n2, word >> (32u - (32u - (uint32_t)__builtin_clz(n2))));
            if (__ballot(j != jg) == 0) break;
            jg = j;
        }
    }
    uint32_t lim = 0xFFFFFFFFu;
    if (role == 1u) {
        const uint32_t n = j < W ? W - j : 1u;
        const uint32_t kb = 32u - (uint32_t)__builtin_clz(n);
        const uint32_t r = word >> (32u - kb);
        lim = n - (1u << (kb - 1u));
        if (r < n && n - r - 1u < lim) lim = n - r - 1u;
        if (j >= W) lim = 0u;
    }
    delta = wave_min_u32(lim);
    i2 += (uint32_t)__popcll(__ballot(role == 1u && a2));
    st = role_apply((uint32_t)__builtin_amdgcn_readlane((int)Fx, 63), st);
}
// V1: one block's draws at draw index i2 (bound W - d, a single role), without emitting: advances
// i2 and returns the largest shift under which every verdict stays (as pair_eval's k2 lanes)
__device__ __forceinline__ void draw_eval(uint32_t word, uint32_t W, uint32_t &i2, uint32_t &delta) {
    const int lane = threadIdx.x & 63;
    const uint64_t below = lanemask_lt();
    uint32_t j = 0;
    bool acc = false;
    // lane l's draw index lies in [i2, i2 + l]: where every verdict is the same over its range, one pass
    const uint32_t jl = i2 + (uint32_t)lane;
    const uint32_t nhi = i2 < W ? W - i2 : 1u, nlo = jl < W ? W - jl : 1u;
    const uint32_t kbh = 32u - (uint32_t)__builtin_clz(nhi);
    const uint32_t rh = word >> (32u - kbh);
    const bool sure = kbh == 32u - (uint32_t)__builtin_clz(nlo) && (rh < nlo || rh >= nhi);
    if (__ballot(!sure) == 0) {
        acc = rh < nlo;
        j = i2 + (uint32_t)__popcll(__ballot(acc) & below);
    } else {
        uint32_t jg = i2 + (uint32_t)lane / 2u;
        for (;;) {
            const uint32_t n2 = jg < W ? W - jg : 1u;
            acc = (word >> (32u - (32u - (uint32_t)__builtin_clz(n2)))) < n2;
            j = i2 + (uint32_t)__popcll(__ballot(acc) & below);
            if (__ballot(j != jg) == 0) break;
            jg = j;
        }
    }
    const uint32_t n = j < W ? W - j : 1u;
    const uint32_t kb = 32u - (uint32_t)__builtin_clz(n);
    const uint32_t r = word >> (32u - kb);
    uint32_t lim = n - (1u << (kb - 1u));
    if (r < n && n - r - 1u < lim) lim = n - r - 1u;
    if (j >= W) lim = 0u;
    delta = wave_min_u32(lim);
    i2 += (uint32_t)__popcll(__ballot(acc));
}
}  // namespace

// ---- generation: a workgroup per window (its raw words), the tail draws on the other blocks ----
// Thread t (< 227) owns words t, t + 227 and t + 454 of every twist: new[k] needs old[k],
// old[k + 1] and either old[k + 397] (k < 227) or new[k - 227] -- the same thread's previous
// word -- so a twist's three dependent steps run in the thread's registers, and only the previous
// twist's words cross threads: the state goes through LDS once per twist (double-buffered, one
// barrier).  new[623] also needs new[0]: its thread computes new[0] again from the old state.
// (One wave over the whole state ran ~1200 clocks a twist, four waves stepping 227 words at a
// time with a barrier per step ~900: 2.9 / 2.2 ms for C5's 5.7K twists a window.)
constexpr int kSpGenThreads = 256;
// Twists [t0, t1) of every window (a chunk: the phases that need only the words before t1 run
// while later chunks are generated); the first chunk seeds and carries the tail draws, a later one
// resumes from the last twist's words (the state).
template <bool kV1>
__global__ __launch_bounds__(kSpGenThreads) void k_v2x_sp_gen(V2xSp a, V2xGeo x, int64_t epoch, uint32_t t0,
                                                              uint32_t t1) {
    __shared__ uint32_t sm[4 * kMtN];   // a window's double-buffered state, or four tail waves' MT
    const uint32_t b = blockIdx.x;
    const int tid = threadIdx.x;
    const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane(tid >> 6);
    if (b >= a.S) {   // the tail: a wave per 64 tail steps
        const uint32_t j0 = ((b - a.S) * 4u + wv) * 64u;
        if (j0 < x.P) v2x_tail_block(x, epoch, 0u, j0, a.K1, sm + kMtN * wv);
        return;
    }
    const uint32_t s = b;
    const V2xSpPlan &pl = sp_plan(a, s);
    if (t0 == 0 && tid < 4)   // phase 0 starts at (k1, 0) -- V1: its one role, (1, 0)
        a.anc[(size_t)s * (kSpPh + 1) * 4 + tid] = kV1 && tid == 0 ? 1u : 0u;
    if (t1 > pl.nt) t1 = pl.nt;
    if (t0 >= t1) return;
    // the generator is a latency chain: it issues first on its SIMDs
    __builtin_amdgcn_s_setprio(3);
    uint32_t *wbase = a.words + (size_t)s * a.nwp;
    uint32_t *sm0 = sm + (t0 & 1u) * kMtN;   // the state the first twist reads
    if (t0 == 0) {
        if (wv == 0) {
            int64_t seed;
            if constexpr (kV1) {   // V1:102,165-171: window w seeds epoch + w * 10000
                const int64_t w = a.w0 + (int64_t)s;
                seed = w == 0 ? epoch : epoch + w * 10000;
            } else {               // V2:107-109,147
                seed = s == 0 ? epoch + 2 : epoch + (int64_t)(s - 1) * 10000;
            }
            mt_seed_int(sm0, seed);
        }
    } else {
        for (int i = tid; i < kMtN; i += kSpGenThreads) sm0[i] = wbase[(size_t)(t0 - 1u) * kMtN + (uint32_t)i];
    }
    __syncthreads();
    constexpr int D = kMtN - kMtM;   // 227
    const bool own = tid < D, own2 = tid < kMtN - 2 * D;   // words t, t + 227 (all), t + 454 (t < 170)
    const bool last = tid == kMtN - 1 - 2 * D;            // t = 169: word 623
    uint32_t o0 = 0u, o1 = 0u, o2 = 0u;
    if (own) { o0 = sm0[tid]; o1 = sm0[tid + D]; }
    if (own2) o2 = sm0[tid + 2 * D];
    uint32_t *dst = wbase + (uint32_t)tid;
    for (uint32_t t = t0; t < t1; t++) {
        const uint32_t *st = sm + (t & 1u) * kMtN;        // the previous twist's words
        uint32_t *sn = sm + ((t + 1u) & 1u) * kMtN;
        if (own) {
            const uint32_t b0 = st[tid + 1], c0 = st[tid + kMtM], b1 = st[tid + D + 1];
            const uint32_t b2 = own2 && !last ? st[tid + 2 * D + 1] : 0u;
            uint32_t z0 = 0u, z1 = 0u, z397 = 0u;
            if (last) { z0 = st[0]; z1 = st[1]; z397 = st[kMtM]; }
            const uint32_t n0 = mt_twist_word(o0, b0, c0);
            const uint32_t n1 = mt_twist_word(o1, b1, n0);
            uint32_t n2 = 0u;
            if (own2) n2 = last ? mt_twist_word(o2, mt_twist_word(z0, z1, z397), n1) : mt_twist_word(o2, b2, n1);
            uint32_t *dt = dst + (size_t)t * kMtN;
            dt[0] = n0;
            dt[D] = n1;
            if (own2) dt[2 * D] = n2;
            sn[tid] = n0;
            sn[tid + D] = n1;
            if (own2) sn[tid + 2 * D] = n2;
            o0 = n0; o1 = n1; o2 = n2;
        }
        __syncthreads();
    }
}

// the interval of a segment's start: the expected k2 index after (q - qa) words from the
// phase's anchor A (the plan's table of expected words per step, linearly interpolated) +-
// PSS_SPLIT_K standard deviations of the renewal count, + 16
__device__ __forceinline__ void sp_interval(const V2xSpPlan &pl, uint32_t A, uint32_t dq, bool v1, uint32_t &lo,
                                            uint32_t &hi) {
    const uint32_t nt = pl.W / 64u + 1u;   // table entries - 1
    auto at = [&](float j, float &m, float &v, float &e) {
        float fi = j * (1.0f / 64.0f);
        if (fi > (float)nt - 1.0f) fi = (float)nt - 1.0f;
        const uint32_t i = (uint32_t)fi;
        const float fr = fi - (float)i;
        const float2 x0 = pl.mv[i], x1 = pl.mv[i + 1];
        m = x0.x + fr * (x1.x - x0.x);
        v = x0.y + fr * (x1.y - x0.y);
        e = (x1.x - x0.x) * (1.0f / 64.0f);
    };
    float mA, vA, eA;
    at((float)A, mA, vA, eA);
    const float target = mA + (float)dq;
    uint32_t l = 0, h = nt;   // the last entry whose expected words stay below the target
    while (h - l > 1u) {
        const uint32_t md = (l + h) / 2u;
        if (pl.mv[md].x <= target) l = md;
        else h = md;
    }
    const float x0 = pl.mv[l].x, x1 = pl.mv[l + 1].x;
    float je = 64.0f * ((float)l + (x1 > x0 ? (target - x0) / (x1 - x0) : 0.0f));
    if (je < (float)A) je = (float)A;
    float mj, vj, ej;
    at(je, mj, vj, ej);
    const float var = vj - vA > 0.0f ? vj - vA : 0.0f;
    const float m = pl.K * __builtin_sqrtf(var + 1.0f) / (ej > 1.0f ? ej : 1.0f) + 16.0f;
    const float flo = je - m, fhi = je + m + 1.0f;
    lo = flo > (float)A ? (uint32_t)flo : A;
    const uint32_t cap = A + (v1 ? dq : dq / 2u) + 1u;   // at most one k2 per two words (V1: a draw a word)
    hi = fhi < (float)cap ? (uint32_t)fhi : cap;
    if (lo > hi) lo = hi;
}

// ---- level 1: the pieces of one (segment, start role) per wave -------------------------------
// The branch list lives across the lanes: lane i holds piece i's low end a_i, its role and its
// count offset c_i (pieces are contiguous: piece i ends at a_{i+1} - 1, the last at hi).
template <bool kV1>
__global__ __launch_bounds__(256) void k_v2x_sp_lvl1(V2xSp a, uint32_t phase) {
    const uint32_t s = blockIdx.y;
    const V2xSpPlan &pl = sp_plan(a, s);
    if (phase >= pl.nph) return;
    const int lane = threadIdx.x & 63;
    const uint32_t item = blockIdx.x * 4u + (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    // (V1: one role -- the record's role-0 half stays empty)
    const uint32_t g = pl.ph[phase] + (kV1 ? item : item / 2u), r0 = kV1 ? 1u : item & 1u;
    if (g >= pl.ph[phase + 1]) return;
    const uint32_t *an = a.anc + ((size_t)s * (kSpPh + 1) + phase) * 4;
    const uint32_t ai2 = an[1], aend = an[2];
    const uint4 sg = pl.seg[g];
    uint2 *rec = a.rec + ((size_t)s * a.nsegmax + g) * kSpRec;
    uint32_t lo, hi;
    sp_interval(pl, ai2, sg.x - pl.seg[pl.ph[phase]].x, kV1, lo, hi);
    uint32_t cnt = kSpOver;
    uint32_t la = lo, lst = r0, lc = 0u;
#ifdef PSS_DIAG_SP_PRINT
    const uint64_t dg_t0 = __builtin_amdgcn_s_memtime();
    uint32_t dg_evals = 0, dg_maxn = 0;
#endif
    if (!aend) {
        const uint32_t W = pl.W, P = a.P, kb1 = a.kb1;
        const uint32_t *wsrc = a.words + (size_t)s * a.nwp + sg.x;
        uint32_t n = 1u;
        bool over = false;
        uint32_t w8[8];   // the next 8 blocks' words, loaded together
        for (uint32_t bq = 0; bq < sg.y && !over; bq += 64u) {
            const uint32_t u8 = (bq >> 6) & 7u;
            if (u8 == 0u) {
#pragma unroll
                for (int u = 0; u < 8; u++) w8[u] = bq + 64u * u < sg.y ? wsrc[bq + 64u * u + (uint32_t)lane] : 0u;
            }
            uint32_t wr = w8[0];
#pragma unroll
            for (int u = 1; u < 8; u++) wr = u8 == (uint32_t)u ? w8[u] : wr;
            const uint32_t word = mt_temper(wr);
            uint32_t na = 0u, nst = 0u, nc = 0u, nn = 0u, lstl = 0u, lcl = 0u;
            for (uint32_t i = 0; i < n && !over; i++) {
                uint32_t ba = (uint32_t)__builtin_amdgcn_readlane((int)la, (int)i);
                const uint32_t bb = i + 1u < n ? (uint32_t)__builtin_amdgcn_readlane((int)la, (int)(i + 1u)) - 1u : hi;
                const uint32_t bst = (uint32_t)__builtin_amdgcn_readlane((int)lst, (int)i);
                const uint32_t bc = (uint32_t)__builtin_amdgcn_readlane((int)lc, (int)i);
                for (;;) {
                    uint32_t st2 = bst, j2 = ba + bc, d = 0u;
                    if (j2 + 64u >= sp_nd<kV1>(W)) { over = true; break; }
                    if constexpr (kV1) draw_eval(word, W, j2, d);
                    else pair_eval(word, W, P, kb1, st2, j2, d);
#ifdef PSS_DIAG_SP_PRINT
                    dg_evals++;
#endif
                    const uint32_t e = d >= bb - ba ? bb : ba + d;
                    const uint32_t c2 = j2 - ba;
                    if (!(nn && lstl == st2 && lcl == c2)) {   // else: the last piece extends to e
                        // (far more pieces than a record keeps -- a bound crossing a power of two
                        // inside the segment makes one per k2 word -- : the walk runs it exactly)
                        if (nn == (uint32_t)kSpPieces) { over = true; break; }
                        if ((uint32_t)lane == nn) { na = ba; nst = st2; nc = c2; }
                        nn++;
                        lstl = st2;
                        lcl = c2;
                    }
                    if (e == bb) break;
                    ba = e + 1u;
                }
            }
            la = na; lst = nst; lc = nc; n = nn;
#ifdef PSS_DIAG_SP_PRINT
            dg_maxn = n > dg_maxn ? n : dg_maxn;
#endif
        }
        if (!over && n <= (uint32_t)kSpPieces) cnt = n;
    }
#ifdef PSS_DIAG_SP_PRINT
    {
        const uint64_t dg = __builtin_amdgcn_s_memtime() - dg_t0;
        if (lane == 0 && s == 0 && (dg > 200000u || (g & 255u) == 0u))
            printf("sp_lvl1 phase %u g %u r0 %u L %u hi-lo %u evals %u maxn %u cnt %u clocks %lu\n", phase, g, r0, sg.y,
                   hi - lo, dg_evals, dg_maxn, cnt, (unsigned long)dg);
    }
#endif
    const uint32_t base = r0 ? (uint32_t)kSpPieces : 0u;
    if (cnt != kSpOver && (uint32_t)lane < cnt) rec[base + (uint32_t)lane] = make_uint2(la, lst | (lc << 1));
    if (lane == 0) {
        reinterpret_cast<uint32_t *>(rec + kSpRecCnt)[r0] = cnt;
        if (kV1) reinterpret_cast<uint32_t *>(rec + kSpRecCnt)[0] = kSpOver;
        if (r0 == (kV1 ? 1u : 0u)) {
            rec[kSpRecLoHi] = make_uint2(lo, hi);
            rec[kSpRecQL] = make_uint2(sg.x, sg.y);
        }
    }
}

// ---- the walk: one wave per window over one phase's segments ----------------------------------
template <bool kV1>
__global__ __launch_bounds__(64) void k_v2x_sp_walk(V2xSp a, uint32_t phase) {
    __shared__ uint32_t mt[kMtN];
    const uint32_t s = blockIdx.x;
    const V2xSpPlan &pl = sp_plan(a, s);
    if (phase >= sp_phases(pl)) return;
    __builtin_amdgcn_s_setprio(3);
    const int lane = threadIdx.x & 63;
    const uint32_t W = pl.W, P = a.P, kb1 = a.kb1;
    uint32_t *an = a.anc + ((size_t)s * (kSpPh + 1) + phase) * 4;
    // the state is wave-uniform: in scalar registers (a vector copy would make every use wait on
    // the outstanding record loads)
    uint32_t st = (uint32_t)__builtin_amdgcn_readfirstlane((int)an[0]);
    uint32_t i2 = (uint32_t)__builtin_amdgcn_readfirstlane((int)an[1]);
    uint32_t ended = (uint32_t)__builtin_amdgcn_readfirstlane((int)an[2]);
    const uint32_t g0 = pl.ph[phase], g1 = pl.nph ? pl.ph[phase + 1] : 0u;
    const uint2 *rec = a.rec + (size_t)s * a.nsegmax * kSpRec;
    uint2 *ss = a.ss + (size_t)s * a.nsegmax;
    const uint32_t *wsrc = a.words + (size_t)s * a.nwp;
    auto noemit = [](bool, uint32_t, uint32_t) {};
    // The records come through LDS in batches of 64 segments (one bulk load of the next batch in
    // flight while this one is walked), lane k = segment k of the batch, and a batch resolves by
    // guess and verify: every lane guesses where its segment starts (first the middle of its
    // interval, then where the last pass put it), takes its pieces' transfer at the guess for
    // either start role, and one inclusive scan of those transfers (the role maps composed, the
    // k2 counts added) gives every lane a start.  Lanes up to the first one whose actual start
    // lies in a piece of another transfer are then exact; that lane's start is exact too, so it
    // becomes the next pass's first lane with an exact guess (or, outside its interval or with
    // too many pieces, it runs exactly).  Each pass settles at least one lane, almost always all.
    // (Walking the segments one by one cost ~550 clocks a segment: a chain of lane reads and
    // scalar branches; ~900 with the records loaded from HBM per segment.)
    constexpr uint32_t kBatch = 64, kPad = kSpRec + 1;   // (odd record pitch: lane k's reads spread over the banks)
    __shared__ uint2 rl[2][kBatch * kPad];
    uint4 v[16];
    auto load_batch = [&](uint32_t gb) {
        const uint4 *src = reinterpret_cast<const uint4 *>(rec + (size_t)gb * kSpRec);
#pragma unroll
        for (int i = 0; i < 16; i++) {
            const uint32_t idx = (uint32_t)lane + 64u * (uint32_t)i;
            v[i] = gb + (idx >> 4) < g1 ? src[idx] : make_uint4(0u, 0u, 0u, 0u);
        }
    };
    auto store_batch = [&](int buf) {
#pragma unroll
        for (int i = 0; i < 16; i++) {
            const uint32_t idx = (uint32_t)lane + 64u * (uint32_t)i;
            uint2 *d = rl[buf] + (idx >> 4) * kPad + 2u * (idx & 15u);
            d[0] = make_uint2(v[i].x, v[i].y);
            d[1] = make_uint2(v[i].z, v[i].w);
        }
        wave_lds_order();
    };
    // an exact run of segment words [q, q + L) from (st, i2), 8 blocks' words loaded at a time
    const uint32_t nd = sp_nd<kV1>(W);
    auto run_exact = [&](uint32_t q, uint32_t L) {
        uint32_t i1 = i2 + st;
        for (uint32_t bq = 0; bq < L && i2 < nd; bq += 512u) {
            uint32_t w8[8];
#pragma unroll
            for (int u = 0; u < 8; u++) w8[u] = bq + 64u * u < L ? wsrc[q + bq + 64u * u + (uint32_t)lane] : 0u;
#pragma unroll
            for (int u = 0; u < 8; u++)
                if (bq + 64u * u < L && i2 < nd) sp_block<kV1>(mt_temper(w8[u]), 64u, W, P, kb1, st, i1, i2, noemit);
        }
        if (i2 >= nd) ended = 1u;
    };
#ifdef PSS_DIAG_SP_PRINT   // timing / diagnostic build: passes and exact runs per walk
    uint32_t dg_pass = 0, dg_exact = 0;
    const uint64_t dg_t0 = __builtin_amdgcn_s_memtime();
#endif
    if (g0 < g1) {
        load_batch(g0);
        store_batch(0);
    }
    int buf = 0;
    for (uint32_t gb = g0; gb < g1; gb += kBatch, buf ^= 1) {
        const bool more = gb + kBatch < g1;
        if (more) load_batch(gb + kBatch);
        const uint32_t nb = g1 - gb < kBatch ? g1 - gb : kBatch;
        const uint32_t ul = (uint32_t)lane;
        const uint2 *mr = rl[buf] + (ul < nb ? ul : 0u) * kPad;   // this lane's record
        const uint32_t lo = mr[kSpRecLoHi].x, hi = mr[kSpRecLoHi].y;
        const uint32_t c0 = mr[kSpRecCnt].x, c1 = mr[kSpRecCnt].y;
        auto valid = [&](uint32_t r, uint32_t j) { return (r ? c1 : c0) <= (uint32_t)kSpPieces && j >= lo && j <= hi; };
        // this lane's pieces in registers (low ends past the count: ~0), read once per batch
        uint32_t pa[2][kSpPieces], pk[2][kSpPieces];
#pragma unroll
        for (int r = 0; r < 2; r++) {
            const uint32_t n = r ? c1 : c0;
#pragma unroll
            for (int q = 0; q < kSpPieces; q++) {
                const uint2 e = mr[r * kSpPieces + q];
                pa[r][q] = (uint32_t)q < n ? e.x : 0xFFFFFFFFu;
                pk[r][q] = e.y;
            }
        }
        // the batch's largest piece count bounds the lookups (uniform)
        uint32_t nmax = 1u;
        {
            const uint32_t m0 = ul < nb && c0 <= (uint32_t)kSpPieces ? c0 : 1u, m1 = ul < nb && c1 <= (uint32_t)kSpPieces ? c1 : 1u;
            uint32_t mm = m0 > m1 ? m0 : m1;
#pragma unroll
            for (int o = 32; o; o >>= 1) {
                const uint32_t y = (uint32_t)__shfl_xor((int)mm, o);
                mm = y > mm ? y : mm;
            }
            nmax = (uint32_t)__builtin_amdgcn_readfirstlane((int)mm);
        }
        auto lookup = [&](uint32_t r, uint32_t j) {   // the transfer (role | c << 1) of the piece holding j
            uint32_t t = r ? pk[1][0] : pk[0][0];
#pragma unroll
            for (int q = 1; q < kSpPieces; q++) {
                if ((uint32_t)q >= nmax) break;
                const uint32_t aq = r ? pa[1][q] : pa[0][q];
                t = aq <= j ? (r ? pk[1][q] : pk[0][q]) : t;
            }
            return t;
        };
        uint32_t guess = lo + (hi - lo) / 2u;       // where this lane's segment starts, guessed
        uint32_t sst = 0u, si2 = 0u;                // its start, once settled
        uint32_t f = 0;                             // lanes below f are settled
        while (f < nb && !ended) {
#ifdef PSS_DIAG_SP_PRINT
            dg_pass++;
#endif
            // transfers at the guesses (identity outside [f, nb))
            const bool act = ul >= f && ul < nb;
            const uint32_t p0 = valid(0u, guess) ? lookup(0u, guess) : 0u;
            const uint32_t p1 = valid(1u, guess) ? lookup(1u, guess) : 2u;
            const uint32_t r0 = p0 & 1u, r1 = p1 & 1u;
            uint32_t tF = act ? (r0 == r1 ? 2u | r0 : r0) : 0u;
            uint32_t t0 = act ? p0 >> 1 : 0u, t1 = act ? p1 >> 1 : 0u;
            // inclusive scan, (earlier) then (this), on DPP row shifts and row broadcasts (lanes
            // without a source read the identity, 0): no LDS round trip per step
            auto step = [&](uint32_t pF, uint32_t q0c, uint32_t q1c) {
                const uint32_t a0 = role_apply(pF, 0u), a1 = role_apply(pF, 1u);
                const uint32_t n0 = q0c + (a0 ? t1 : t0), n1 = q1c + (a1 ? t1 : t0);
                tF = role_compose(tF, pF);
                t0 = n0;
                t1 = n1;
            };
            step(dpp_role<0x111, 0xF>(tF), dpp_role<0x111, 0xF>(t0), dpp_role<0x111, 0xF>(t1));
            step(dpp_role<0x112, 0xF>(tF), dpp_role<0x112, 0xF>(t0), dpp_role<0x112, 0xF>(t1));
            step(dpp_role<0x114, 0xF>(tF), dpp_role<0x114, 0xF>(t0), dpp_role<0x114, 0xF>(t1));
            step(dpp_role<0x118, 0xF>(tF), dpp_role<0x118, 0xF>(t0), dpp_role<0x118, 0xF>(t1));
            step(dpp_role<0x142, 0xA>(tF), dpp_role<0x142, 0xA>(t0), dpp_role<0x142, 0xA>(t1));
            step(dpp_role<0x143, 0xC>(tF), dpp_role<0x143, 0xC>(t0), dpp_role<0x143, 0xC>(t1));
            const uint32_t eF = (uint32_t)__shfl_up((int)tF, 1), e0 = (uint32_t)__shfl_up((int)t0, 1);
            const uint32_t e1 = (uint32_t)__shfl_up((int)t1, 1);
            const uint32_t bst = ul == f ? st : role_apply(eF, st);
            const uint32_t bi2 = i2 + (ul == f ? 0u : (st ? e1 : e0));
            const bool vstart = valid(bst, bi2);
            const bool ok = vstart && valid(bst, guess) && lookup(bst, bi2) == lookup(bst, guess);
            const uint64_t bad = __ballot(act && !ok);
            const uint32_t g = bad ? (uint32_t)__ffsll((long long)bad) - 1u : nb;
            if (ul >= f && ul < g) { sst = bst; si2 = bi2; }
            if (g >= nb) {   // all settled: the state after the batch
                const uint32_t lF = (uint32_t)__builtin_amdgcn_readlane((int)tF, (int)(nb - 1u));
                const uint32_t l0 = (uint32_t)__builtin_amdgcn_readlane((int)t0, (int)(nb - 1u));
                const uint32_t l1 = (uint32_t)__builtin_amdgcn_readlane((int)t1, (int)(nb - 1u));
                i2 += st ? l1 : l0;
                st = role_apply(lF, st);
                f = nb;
                break;
            }
            // lane g starts exactly there
            st = (uint32_t)__builtin_amdgcn_readlane((int)bst, (int)g);
            i2 = (uint32_t)__builtin_amdgcn_readlane((int)bi2, (int)g);
            if (!__builtin_amdgcn_readlane((int)vstart, (int)g)) {   // outside its interval: run it
#ifdef PSS_DIAG_SP_PRINT
                dg_exact++;
#endif
                if (ul == g) { sst = st; si2 = i2; }
                run_exact((uint32_t)__builtin_amdgcn_readlane((int)mr[kSpRecQL].x, (int)g),
                          (uint32_t)__builtin_amdgcn_readlane((int)mr[kSpRecQL].y, (int)g));
                st = (uint32_t)__builtin_amdgcn_readfirstlane((int)st);
                i2 = (uint32_t)__builtin_amdgcn_readfirstlane((int)i2);
                f = g + 1u;
            } else {
                f = g;
            }
            if (ul >= f) guess = bi2;
        }
        if (ended)   // the stream ended inside a segment: every later one is marked
            if (ul >= f) { sst = 2u; si2 = i2; }
        if (ul < nb) ss[gb + ul] = make_uint2(sst, si2);
        if (more) store_batch(buf ^ 1);
    }
    if (lane == 0) { an[4] = st; an[5] = i2; an[6] = ended; }
#ifdef PSS_DIAG_SP_PRINT
    if (lane == 0 && s == 0)
        printf("sp_walk phase %u segs %u passes %u exact %u clocks %lu i2 %u W %u\n", phase, g1 - g0, dg_pass, dg_exact,
               (unsigned long)(__builtin_amdgcn_s_memtime() - dg_t0), i2, W);
#endif
    if (phase + 1u != sp_phases(pl)) return;
    // the rest of the window, exactly, emitting
    const size_t t0 = (size_t)s * a.B;
    uint32_t *k1 = a.K1 + t0, *k2 = a.K2 + t0;
    auto emit = [&](bool second, uint32_t i, uint32_t r) {
        if constexpr (kV1) {   // J[n - 1 - d] (the buckets are counted afterwards: k_v1x_sp_count)
            k1[W - 1u - i] = r;
        } else {
            if (second) k2[i] = r;
            else k1[i] = r;
        }
    };
    if (!ended) {
        uint32_t i1 = i2 + st, q = pl.qend;
        const uint32_t nw = pl.nt * (uint32_t)kMtN;
        while (i2 < nd && q < nw) {   // 8 blocks' words loaded at a time
            uint32_t w8[8];
#pragma unroll
            for (int u = 0; u < 8; u++) {
                const uint32_t qu = q + 64u * u + (uint32_t)lane;
                w8[u] = qu < nw ? wsrc[qu] : 0u;
            }
#pragma unroll
            for (int u = 0; u < 8; u++) {
                if (i2 >= nd || q >= nw) break;
                const uint32_t nval = nw - q < 64u ? nw - q : 64u;
                const bool valid = (uint32_t)lane < nval;
                sp_block<kV1>(valid ? mt_temper(w8[u]) : 0u, nval, W, P, kb1, st, i1, i2, emit);
                q += nval;
            }
        }
        if (i2 < nd) {   // past the generated words: the stream continues from its state (the last twist)
            for (int i = lane; i < kMtN; i += 64) mt[i] = wsrc[nw - (uint32_t)kMtN + (uint32_t)i];
            wave_lds_order();
            while (i2 < nd) {
                mt_twist(mt);
                for (int q0 = 0; q0 < kMtN && i2 < nd; q0 += 64) {
                    const int nval = kMtN - q0 < 64 ? kMtN - q0 : 64;
                    const bool valid = lane < nval;
                    sp_block<kV1>(valid ? mt_temper(mt[q0 + lane]) : 0u, (uint32_t)nval, W, P, kb1, st, i1, i2, emit);
                }
            }
        }
    }
    if (!kV1)
        for (uint32_t u = W + (uint32_t)lane; u < a.B; u += 64u) k2[u] = 0u;   // padding steps
}

// ---- emission: one wave per segment from its start ---------------------------------------------
template <bool kV1>
__global__ __launch_bounds__(256) void k_v2x_sp_emit(V2xSp a) {
    const uint32_t s = blockIdx.y;
    const V2xSpPlan &pl = sp_plan(a, s);
    const uint32_t g = blockIdx.x * 4u + (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    if (g >= pl.ph[pl.nph]) return;
    const uint2 st0 = a.ss[(size_t)s * a.nsegmax + g];
    if (st0.x > 1u) return;
    const int lane = threadIdx.x & 63;
    const uint4 sg = pl.seg[g];
    const uint32_t W = pl.W, P = a.P, kb1 = a.kb1;
    const uint32_t *wsrc = a.words + (size_t)s * a.nwp + sg.x;
    const size_t t0 = (size_t)s * a.B;
    uint32_t *k1 = a.K1 + t0, *k2 = a.K2 + t0;
    auto emit = [&](bool second, uint32_t i, uint32_t r) {
        if constexpr (kV1) {   // J[n - 1 - d]
            k1[W - 1u - i] = r;
        } else {
            if (second) k2[i] = r;
            else k1[i] = r;
        }
    };
    const uint32_t nd = sp_nd<kV1>(W);
    uint32_t st = st0.x, i2 = st0.y, i1 = i2 + st;
    for (uint32_t bq = 0; bq < sg.y && i2 < nd; bq += 512u) {   // 8 blocks' words loaded together
        uint32_t w8[8];
#pragma unroll
        for (int u = 0; u < 8; u++) w8[u] = bq + 64u * u < sg.y ? wsrc[bq + 64u * u + (uint32_t)lane] : 0u;
#pragma unroll
        for (int u = 0; u < 8; u++)
            if (bq + 64u * u < sg.y && i2 < nd) sp_block<kV1>(mt_temper(w8[u]), 64u, W, P, kb1, st, i1, i2, emit);
    }
}

// V1: the draws' bucket counts (j >> 11 of J[1 .. n), pss_v1exact.hip kV1bShift) once J is
// written -- per-draw atomics on a window's few hundred counters in the emission took 1.7 ms at C5;
// here an LDS histogram per 16K entries, then one atomic per (workgroup, bucket)
constexpr uint32_t kSpCountPer = 16384, kSpCountLds = 8192;
__global__ __launch_bounds__(256) void k_v1x_sp_count(V2xSp a) {
    __shared__ uint32_t h[kSpCountLds];
    const uint32_t s = blockIdx.y;
    const uint32_t n = sp_plan(a, s).W;
    const uint32_t i0 = blockIdx.x * kSpCountPer;
    if (i0 >= n) return;
    const uint32_t *j = a.K1 + (size_t)s * a.B;
    uint32_t *bc = a.K2 + (size_t)s * a.nbk;
    const uint32_t i1 = i0 + kSpCountPer < n ? i0 + kSpCountPer : n;
    const bool lds = a.nbk <= kSpCountLds;
    if (lds) {
        for (uint32_t b = threadIdx.x; b < a.nbk; b += 256u) h[b] = 0u;
        __syncthreads();
    }
    for (uint32_t i = (i0 ? i0 : 1u) + threadIdx.x; i < i1; i += 256u) {
        const uint32_t b = j[i] >> 11;
        if (lds) atomicAdd(&h[b], 1u);
        else atomicAdd(&bc[b], 1u);
    }
    if (lds) {
        __syncthreads();
        for (uint32_t b = threadIdx.x; b < a.nbk; b += 256u)
            if (h[b]) atomicAdd(&bc[b], h[b]);
    }
}

namespace {
// ---- host: the plan of one window length (cached per device, W and P) -----------------------
struct SpPlanHost {
    std::vector<uint4> seg;
    uint32_t W = 0, nph = 0, nt = 0, qend = 0;
    double K = PSS_SPLIT_K;
    uint32_t ph[kSpPh + 1] = {};
    double words = 0;            // expected words of the window
    std::vector<float2> mv;      // expected words / variance to reach step 64 i
    uint4 *dseg = nullptr;
    float2 *dmv = nullptr;
};

static uint32_t sp_bitlen(uint64_t n) { return n ? 64u - (uint32_t)__builtin_clzll(n) : 0u; }

static void sp_plan_build(uint32_t W, uint32_t P, bool v1, SpPlanHost &h) {
    h.W = W;
    h.K = v1 ? PSS_SPLIT_K_V1 : PSS_SPLIT_K;
    const uint32_t kb1 = sp_bitlen(P);
    const double a1 = v1 ? 1.0 : (double)P / (double)(1ull << kb1);   // (V1: no k1 draws)
    // words per step j (a k1 then a k2 draw at bound W - j) and their variance; running sums
    std::vector<double> M(W + 1), V(W + 1), E(W ? W : 1);
    M[0] = V[0] = 0.0;
    for (uint32_t j = 0; j < W; j++) {
        const uint32_t n = W - j;
        const double a2 = (double)n / (double)(1ull << sp_bitlen(n));
        E[j] = (v1 ? 0.0 : 1.0 / a1) + 1.0 / a2;
        M[j + 1] = M[j] + E[j];
        V[j + 1] = V[j] + (1.0 - a1) / (a1 * a1) + (1.0 - a2) / (a2 * a2);
    }
    h.words = W ? M[W] : 0.0;
    for (uint32_t i = 0; i <= W / 64u + 1u; i++) {
        const uint32_t j = 64u * i < W ? 64u * i : W;
        h.mv.push_back(make_float2((float)M[j], (float)V[j]));
    }
    auto jat = [&](double q) {   // the step whose expected word offset reaches q
        const size_t i = (size_t)(std::lower_bound(M.begin(), M.end(), q) - M.begin());
        return i < W ? i : (size_t)(W ? W - 1 : 0);
    };
    uint32_t q = 0;
    for (int p = 0; p < kSpPh && W; p++) {
        const uint32_t qa = q;
        const size_t ja = jat(qa), n0 = h.seg.size();
        for (;;) {
            const size_t je = jat(q);
            const double sd = std::sqrt(V[je] - V[ja] + 1.0) / E[je];
            const double m = h.K * sd + 16.0, width = 2.0 * m + 1.0;
            const double nmin = (double)W - (double)je - m - 64.0;
            if (nmin <= 4.0 * width) break;
            const uint32_t kk = sp_bitlen((uint64_t)nmin);
            const double f2 = ((double)(1ull << kk) / nmin) / E[je];   // k2 share of the words (upper bound)
            auto splits = [&](uint32_t L) { return L * f2 * width / (double)(1ull << (kk - 1)); };
            uint32_t L = 4096;
            while (L > 64 && splits(L) > PSS_SPLIT_TARGET) L >>= 1;
            if (splits(L) > 2.0 * PSS_SPLIT_TARGET || (double)je + m + L >= (double)W - 64.0) break;
            // The bound W - j crossing a power of two inside a segment changes the bit length of
            // every later k2 word, at a point that moves with the start: about one piece per k2
            // word, far more than a record keeps.  So a phase ends ahead of each crossing (the next
            // one re-anchors there, its intervals narrow again) and the segments whose intervals
            // still straddle a crossing are one block long (their exact runs in the walk are short).
            const double jlo = (double)je - 2.0 * m > 0.0 ? (double)je - 2.0 * m : 0.0;
            const double jhi = (double)je + 2.0 * m + (v1 ? (double)L : L / 2.0) + 1.0;
            if (sp_bitlen((uint64_t)((double)W - jlo)) != sp_bitlen((uint64_t)std::max(1.0, (double)W - jhi))) {
                if (m > kSpCrossMargin && h.seg.size() > n0) break;
                L = 64;
            }
            h.seg.push_back(make_uint4(q, L, 0u, 0u));   // (the interval comes from the actual anchor: sp_interval)
            q += L;
        }
        if (h.seg.size() == n0) break;
        h.nph++;
        h.ph[h.nph] = (uint32_t)h.seg.size();
    }
    for (int p = (int)h.nph + 1; p <= kSpPh; p++) h.ph[p] = (uint32_t)h.seg.size();
    h.qend = q;
    double nw = h.words + 12.0 * std::sqrt(W ? V[W] : 0.0) + 2.0 * kMtN;
    if (nw < (double)q + 64.0) nw = (double)q + 64.0;
    h.nt = (uint32_t)std::ceil(nw / (double)kMtN);
}

static const SpPlanHost *sp_plan_get(uint32_t W, uint32_t P, bool v1) {
    static std::mutex mu;
    static std::map<std::tuple<int, uint32_t, uint32_t, bool>, std::unique_ptr<SpPlanHost>> cache;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    std::lock_guard<std::mutex> lk(mu);
    auto &slot = cache[std::make_tuple(dev, W, P, v1)];
    if (!slot) {
        auto h = std::make_unique<SpPlanHost>();
        sp_plan_build(W, P, v1, *h);
        if (!h->seg.empty()) {
            const size_t sb = h->seg.size() * sizeof(uint4), mb = h->mv.size() * sizeof(float2);
            char *d = nullptr;
            if (hipMalloc((void **)&d, sb + mb) != hipSuccess) {
                (void)hipGetLastError();
                return nullptr;   // (not cached: retried on the next call)
            }
            if (hipMemcpy(d, h->seg.data(), sb, hipMemcpyHostToDevice) != hipSuccess ||
                hipMemcpy(d + sb, h->mv.data(), mb, hipMemcpyHostToDevice) != hipSuccess) {
                (void)hipGetLastError();
                (void)hipFree(d);
                return nullptr;
            }
            h->dseg = reinterpret_cast<uint4 *>(d);
            h->dmv = reinterpret_cast<float2 *>(d + sb);
        }
        slot = std::move(h);
    }
    return slot.get();
}

// per device: a stream for the generator chunks and their events (the phases on the caller's
// stream wait on them); the mutex keeps one call's record / wait pairs together
struct SpSide {
    std::mutex mu;
    hipStream_t g = nullptr;
    hipEvent_t start = nullptr, ev[kSpPh + 1] = {};
    bool ok = false;
};
static SpSide *sp_side() {
    static std::mutex mu;
    static std::map<int, std::unique_ptr<SpSide>> per;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    std::lock_guard<std::mutex> lk(mu);
    auto &p = per[dev];
    if (!p) {
        p = std::make_unique<SpSide>();
        int lo = 0, hi = 0;
        bool ok = hipDeviceGetStreamPriorityRange(&lo, &hi) == hipSuccess &&
                  hipStreamCreateWithPriority(&p->g, hipStreamNonBlocking, hi) == hipSuccess &&
                  hipEventCreateWithFlags(&p->start, hipEventDisableTiming) == hipSuccess;
        for (hipEvent_t &e : p->ev) ok = ok && hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess;
        if (!ok) (void)hipGetLastError();
        p->ok = ok;
    }
    return p->ok ? p.get() : nullptr;
}

static V2xSpPlan sp_plan_dev(const SpPlanHost &h) {
    V2xSpPlan p{};
    p.seg = h.dseg;
    p.mv = h.dmv;
    p.W = h.W; p.nph = h.nph; p.nt = h.nt; p.qend = h.qend;
    p.K = (float)h.K;
    for (int i = 0; i <= kSpPh; i++) p.ph[i] = h.ph[i];
    return p;
}
}  // namespace
