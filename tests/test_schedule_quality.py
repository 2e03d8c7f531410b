"""Distribution parity of the counter-based schedule against the reference algorithm.

The GPU reproduces the oracle's counter-based twin bit for bit (tests/test_gpu_parity.py), and
the twin reproduces the reference's assignment and per-rank multisets exactly
(tests/test_oracle_golden.py).  The ORDER inside a pool is drawn from a different random
source than the reference's CPython `random`, so what can be checked is that
it follows the same law.  These tests compare the exact restatement of the reference
(V1:157-172, V2:96-116: CPython MT19937, list.remove pools) with the twin on the same shapes:
displacement quantiles, spread, and short-range order statistics.  CPU only; they also guard
every change to the slot / insertion / tail hash functions.
"""
import numpy as np
import pytest

from oracle import oracle as O

QS = [0.001, 0.01, 0.05, 0.25, 0.5, 0.75, 0.95, 0.99]


def _stats(streams, B):
    d = np.concatenate([(np.arange(len(s)) - s) / B for s in streams])
    up = np.concatenate([np.diff(s) > 0 for s in streams])
    lag = np.concatenate([np.abs(np.diff(s)) < B for s in streams])
    return d, up.mean(), lag.mean()


@pytest.mark.parametrize("B,ns", [(256, 40000), (1000, 60000), (96, 9000)])
def test_v2_displacement_law_matches_reference(B, ns):
    N = 10**12                     # no wrap: the id is the virtual index (old = new = 0)
    # 24 streams a side: at B = 96 the 0.99 quantile moves by ~0.05 between sets of 12
    ex = [O.v2_exact_stream(e, 0, 0, ns, B, N) for e in range(24)]
    ph = [O.v2_philox_stream(O.epoch_key(s, e), r, 0, 0, ns, B, N)
          for s in (0, 3, 5, 9) for e in range(3) for r in range(2)]
    dx, upx, lagx = _stats(ex, B)
    dp, upp, lagp = _stats(ph, B)
    # V2 law: no id earlier than v - 2B; a geometric late tail of scale ~B
    assert dp.min() >= -2.0 and dx.min() >= -2.0
    np.testing.assert_allclose(np.quantile(dp, QS), np.quantile(dx, QS), atol=0.06)
    assert abs(dp.std() / dx.std() - 1) < 0.03
    assert abs(upp - upx) < 0.01          # consecutive outputs: P(increasing) ~ 1/2
    assert abs(lagp - lagx) < 0.01        # consecutive outputs closer than one window


@pytest.mark.parametrize("B,ns", [(512, 20000), (100, 5000)])
def test_v1_window_permutation_is_uniform(B, ns):
    # V1:165-171: each window is a uniform permutation; the element at each position must be
    # uniform over the window (chi-square over many windows), like the reference's shuffle
    N = 10**12
    reps = []
    for s in range(6):
        key = O.epoch_key(s, 7)
        for r in range(4):
            reps.append(O.v1_philox_stream(key, r, 0, ns, B, N))
    x = np.stack(reps)                          # [reps, ns] of ids
    full = (ns // B) * B
    rel = (x[:, :full] % B).reshape(-1, B)      # offset of the element at each window position
    # first window position: offsets uniform over [0, B)
    counts = np.bincount(rel[:, 0] * 8 // B, minlength=8)
    exp = rel.shape[0] / 8
    chi2 = ((counts - exp) ** 2 / exp).sum()
    assert chi2 < 30.0                          # 7 dof, p ~ 1e-4
    # displacement inside the window is |d| < B, mean ~ 0
    d = (np.arange(full)[None, :] % B) - rel.reshape(x.shape[0], -1)
    assert np.abs(d).max() < B
    assert abs(d.mean()) < 0.02 * B


BURST = 32   # steps per burst of a grouped pool (schedule 4; 16 up to schedule 3)


def _burst_stats(streams, B, T):
    """Per aligned run of BURST consecutive outputs among the replacement steps (a grouped
    pool's burst: one 4096-slot group draws all of them): the spread (max - min) / B, and
    |diff| / B of consecutive outputs inside the run."""
    spread, step = [], []
    for s in streams:
        x = np.asarray(s[:T // BURST * BURST], dtype=np.float64).reshape(-1, BURST)
        spread.append((x.max(1) - x.min(1)) / B)
        step.append(np.abs(np.diff(x, axis=1)).ravel() / B)
    return np.concatenate(spread), np.concatenate(step)


@pytest.mark.parametrize("B,ns,nex,atol", [(20000, 160000, 3, 0.02), (65536, 4 * 65536, 4, 0.01),
                                           (1 << 20, 3 << 20, 2, 0.015)])
def test_v2_grouped_pool_law_matches_reference(B, ns, nex, atol):
    """Pools beyond LDS (P1 > 16384) draw in bursts of 32 inside G = ceil(P1 / 4096) slot
    groups.  Against the reference's own single-pool draws (V2:101-106, the
    exact restatement -- rank-select form for the big pools), on the grouped geometries: B =
    20000 (G = 5, groups of 4000: multiply-shift draws), 65536 (G = 16) and C5's 2^20 (G = 256,
    groups of 4096 with paired draws): displacement quantiles, spread, consecutive-output
    statistics, and within-burst statistics (the spread of each run of 32 outputs and the gaps
    inside it) against the same positions of the reference's stream."""
    N = 10**12
    T = ns - B
    ex = [O.v2_exact_stream_rs(e, 0, 0, ns, B, N) for e in range(nex)]
    ph = [O.v2_philox_stream(O.epoch_key(s, e), r, 0, 0, ns, B, N)
          for s in (0, 3) for e in range(2) for r in range(2)][:max(4, 2 * nex)]
    dx, upx, lagx = _stats(ex, B)
    dp, upp, lagp = _stats(ph, B)
    assert dp.min() >= -2.0 and dx.min() >= -2.0
    np.testing.assert_allclose(np.quantile(dp, QS), np.quantile(dx, QS), atol=atol)
    assert abs(dp.std() / dx.std() - 1) < 0.01
    assert abs(upp - upx) < 0.005
    assert abs(lagp - lagx) < 0.005
    sx, gx = _burst_stats(ex, B, T)
    sp, gp = _burst_stats(ph, B, T)
    BQ = [0.05, 0.25, 0.5, 0.75, 0.95]
    np.testing.assert_allclose(np.quantile(sp, BQ), np.quantile(sx, BQ), atol=2 * atol)
    np.testing.assert_allclose(np.quantile(gp, BQ), np.quantile(gx, BQ), atol=2 * atol)
    assert abs(sp.mean() / sx.mean() - 1) < 0.01 and abs(gp.mean() / gx.mean() - 1) < 0.01


# ---- randomness of the counter schedule's primitives ------------------------------------------
def _chi2(counts):
    counts = np.asarray(counts, dtype=np.float64).ravel()
    exp = counts.sum() / counts.size
    return ((counts - exp) ** 2 / exp).sum(), counts.size - 1


def _chi2_ok(counts, z=5.0):
    # chi-square with k dof against its normal approximation: mean k, sd sqrt(2k)
    x, k = _chi2(counts)
    return abs(x - k) < z * np.sqrt(2 * k), (x, k)


@pytest.mark.parametrize("P1", [256, 4096, 100, 3000, 20000, 65536])
def test_slot_draws_are_uniform_per_slot(P1):
    """Every slot is drawn equally often (chi-square over the P1 slots), for paired power-of-two
    pools, multiply-shift pools and both kinds of grouped pools (P1 > 16384)."""
    T = 200 * P1 if P1 <= 4096 else 60 * P1
    k = O.v2_slots(O.epoch_key(5, 1), 3, P1, T)
    ok, stat = _chi2_ok(np.bincount(k, minlength=P1))
    assert ok, stat


@pytest.mark.parametrize("P1", [256, 4096, 65536])
def test_paired_draws_are_independent(P1):
    """Paired draws share one 32-bit hash (steps t and t + 64 in small pools, sub-steps u and
    u + 64 of a group in grouped ones): the joint distribution of the two slots' top 4 bits is
    uniform over the 256 cells, and so is that of consecutive steps."""
    T = 4_000_000
    k = O.v2_slots(O.epoch_key(9, 2), 0, P1, T).astype(np.int64)
    hb = int(np.log2(P1 if P1 <= 16384 else 4096))
    top = (k % (1 << hb)) >> (hb - 4)                    # slot inside the group, top 4 bits
    if P1 <= 16384:
        t = np.arange(T)
        lo = t[(t % 128) < 64]
        pairs = (lo, lo + 64)
    else:
        G = P1 // 4096
        t = np.arange(T)
        g, u = (t // 16) % G, (t // 16 // G) * 16 + t % 16
        sel = (u % 128) < 64
        partner = ((u + 64) // 16 * G + g) * 16 + (u + 64) % 16
        ok_ = sel & (partner < T)
        pairs = (t[ok_], partner[ok_])
    for a, b in (pairs, (np.arange(T - 1), np.arange(1, T))):
        joint = np.bincount(top[a] * 16 + top[b], minlength=256)
        ok, stat = _chi2_ok(joint)
        assert ok, stat


def _pair_counts_expected(n, bins, K):
    """Expected (pi(a), pi(b)) bin counts for K uniform random permutations of [0, n): an
    ordered pair of DISTINCT elements (a permutation never maps two positions to one value)."""
    c = np.bincount(np.arange(n) * bins // n, minlength=bins).astype(np.float64)
    return K * (np.outer(c, c) - np.diag(c)) / (n * (n - 1))


def _chi2_expected_ok(counts, exp, z=5.0):
    counts, exp = np.asarray(counts, np.float64).ravel(), np.asarray(exp, np.float64).ravel()
    m = exp > 0
    x, k = ((counts[m] - exp[m]) ** 2 / exp[m]).sum(), int(m.sum()) - 1
    return abs(x - k) < z * np.sqrt(2 * k), (x, k)


@pytest.mark.parametrize("n", [4, 16, 64, 100, 256, 700, 1024, 4096, 65536, 1 << 18, 300_000, 1 << 20, 5000,
                               3 << 20])
def test_feistel_insertion_order_is_uniform(n):
    """The keyed Feistel bijections (8 fmix32 rounds for halves <= 5 bits, the 16-bit round
    function up to 10 bits, the 24-bit one above; cycle walking when n is not a power of 4): over
    many keys the images of single positions are uniform over [0, n) (chi-square on up to 32
    bins) and the images of two neighbours follow the law of a uniform random permutation
    (chi-square on up to 8 x 8 bins against the distinct-pair law) -- the law of the
    reference's Fisher-Yates windows (V1:169-170).  Before the small-half rounds, n = 16 / 64 /
    256 failed this at z = 74 / 122 / 22."""
    rng = np.random.default_rng(n)
    K = 6000
    keys = rng.integers(0, 2 ** 32, (K, 6), dtype=np.uint64).astype(np.uint32)
    y0 = np.array([O.feistel(0, n, k) for k in keys], dtype=np.int64)
    y1 = np.array([O.feistel(1, n, k) for k in keys], dtype=np.int64)
    y7 = np.array([O.feistel(min(7, n - 1), n, k) for k in keys], dtype=np.int64)
    b1 = min(32, n)
    for y in (y0, y1, y7):
        exp = K * np.bincount(np.arange(n) * b1 // n, minlength=b1) / n
        ok, stat = _chi2_expected_ok(np.bincount(y * b1 // n, minlength=b1), exp)
        assert ok, stat
    b2 = min(8, n)
    for a, b in ((y0, y1), (y1, y7)):
        got = np.bincount((a * b2 // n) * b2 + b * b2 // n, minlength=b2 * b2)
        ok, stat = _chi2_expected_ok(got, _pair_counts_expected(n, b2, K))
        assert ok, stat
    # one key: a permutation of [0, n) whose neighbouring images are uncorrelated
    if 64 <= n <= 65536:
        perm = np.array([O.feistel(i, n, keys[0]) for i in range(n)], dtype=np.int64)
        assert np.array_equal(np.sort(perm), np.arange(n))
        lim = 0.05 if n >= 1024 else 4.0 / np.sqrt(n)
        assert abs(np.corrcoef(perm[:-1], perm[1:])[0, 1]) < lim
        assert abs(np.corrcoef(np.arange(n), perm)[0, 1]) < lim
