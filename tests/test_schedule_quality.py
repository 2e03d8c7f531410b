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
    ex = [O.v2_exact_stream(e, 0, 0, ns, B, N) for e in range(12)]
    ph = [O.v2_philox_stream(O.epoch_key(s, e), r, 0, 0, ns, B, N)
          for s in (0, 3) for e in range(3) for r in range(2)]
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


@pytest.mark.parametrize("B,ns", [(20000, 160000)])
def test_v2_grouped_pool_law_matches_reference(B, ns):
    # pools beyond LDS (P1 > 16384) draw in bursts of 16 inside G = ceil(P1 / 4096) slot groups
    # (DESIGN.md §3.2.1); the displacement law must still be the reference's single-pool law
    N = 10**12
    ex = [O.v2_exact_stream(e, 0, 0, ns, B, N) for e in range(3)]
    ph = [O.v2_philox_stream(O.epoch_key(s, e), r, 0, 0, ns, B, N)
          for s in (0, 3) for e in range(2) for r in range(2)]
    dx, upx, lagx = _stats(ex, B)
    dp, upp, lagp = _stats(ph, B)
    assert dp.min() >= -2.0 and dx.min() >= -2.0
    np.testing.assert_allclose(np.quantile(dp, QS), np.quantile(dx, QS), atol=0.02)
    assert abs(dp.std() / dx.std() - 1) < 0.01
    assert abs(upp - upx) < 0.005
    assert abs(lagp - lagx) < 0.005
