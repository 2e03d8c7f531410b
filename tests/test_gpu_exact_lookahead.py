"""Exact-order draw lookahead (pss_runtime.cpp generate_exact): once an engine generated
consecutive epochs of one call shape, the MT draws of the coming epochs are made ahead on side
streams into draw slots, and the call of a prepared epoch only decodes (V2) / resolves (V1).  The
reference's draws depend on the epoch and the window alone (V1:165-171, V2:107-109,147), so a
prepared epoch must give the same stream as one drawn in its own call: checked here against an
engine that visits the same epochs out of order (never sequential, so it never draws ahead) and
against the exact oracle.
"""
import numpy as np
import pytest

from oracle import oracle as O
from partiallyshuffledistributedsampler_amd.engine import IndexEngine

pytestmark = pytest.mark.gpu

EPOCHS = list(range(11))


def _shape(B, R=3, mult=3.5, pad=2):
    ns = int(mult * B)
    N, F = ns * R - pad, 90
    lens = np.full(F, N // F, dtype=np.int64)
    lens[-1] += N - lens.sum()
    return lens, N, R


def _check_epochs(B, version, order, calls_per_epoch=1, lookahead=None):
    """Every epoch of `order` (rank starts from the engine's own epoch history, which depends on
    the order the epochs are visited in, V2:142-152) against the exact oracle.  Returns the
    engine's lookahead counters (pss_lookahead_stats) and its peak device bytes."""
    lens, N, R = _shape(B)
    eng = IndexEngine(lens, N, R, B, version, device=0, order="exact")
    if lookahead is not None:
        eng.set_lookahead(*lookahead)
    peak = 0
    ns = eng.num_samples
    for e in order:
        eng.init_iter(e)
        if calls_per_epoch == 1:
            got = eng.generate(0, R).cpu().numpy()
        else:   # one call per rank, the last rank in two position ranges
            rows = [eng.generate(r, r + 1).cpu().numpy()[0] for r in range(R - 1)]
            h = ns // 3
            rows.append(np.concatenate([eng.generate(R - 1, R, pos_lo=0, count=h).cpu().numpy()[0],
                                        eng.generate(R - 1, R, pos_lo=h).cpu().numpy()[0]]))
            got = np.stack(rows)
        eng.check()
        old, new = eng.rank_starts()
        for r in range(R):
            ref = (O.v1_exact_stream(e, int(new[r]), ns, B, N) if version == 1 else
                   O.v2_exact_stream_rs(e, int(old[r]), int(new[r]), ns, B, N))
            assert np.array_equal(got[r], ref), ("epoch", e, "rank", r, "B", B, "version", version)
        peak = max(peak, eng.workspace_bytes())
    stats = eng.lookahead_stats()
    eng.close()
    return stats, peak


# V2: B = 4096 chain mode, one wave per pool2 window, and 5000, merge levels (no lookahead for
# the one-wave draws: they check the slot-less path beside it); 2^16 pools beyond one decode
# tile, few long windows (the workgroup draws, eight epochs ahead)
@pytest.mark.parametrize("B", [4096, 5000, 1 << 16])
def test_v2_consecutive_epochs_with_draws_made_ahead(B):
    stats, _ = _check_epochs(B, 2, EPOCHS)
    if B == 1 << 16:   # the prepared path really ran
        assert stats["exact_made"] > 0 and stats["exact_used"] >= len(EPOCHS) - 3, stats


# V1: B = 4096 windows resolved in LDS (no lookahead); 2^17 windows through HBM (workgroup
# draws, 8 ahead)
@pytest.mark.parametrize("B", [4096, 1 << 17])
def test_v1_consecutive_epochs_with_draws_made_ahead(B):
    stats, _ = _check_epochs(B, 1, EPOCHS)
    if B == 1 << 17:
        assert stats["exact_made"] > 0 and stats["exact_used"] >= len(EPOCHS) - 3, stats


def test_epoch_jumps_drop_the_prepared_draws():
    # 0, 1 (queues 2, 3), 5 (not 1 + 1: its own draws, the slots of 2, 3 dropped), 6, 7, 3, 4
    _check_epochs(1 << 16, 2, [0, 1, 5, 6, 7, 3, 4])
    _check_epochs(1 << 17, 1, [0, 1, 5, 6, 7, 3, 4])


@pytest.mark.parametrize("version,B", [(1, 1 << 17), (2, 1 << 16)])
def test_several_calls_per_epoch_keep_the_lookahead_correct(version, B):
    # each call shape (rank 0, rank 1, rank 2's two position ranges) keeps its own history, so the
    # whole-range shapes still draw ahead (one shared "last call" never did)
    stats, _ = _check_epochs(B, version, EPOCHS[:6], calls_per_epoch=3)
    assert stats["exact_used"] > 0, stats


@pytest.mark.parametrize("version,B", [(1, 1 << 17), (2, 1 << 16)])
def test_lookahead_bounds_are_honoured_and_change_nothing(version, B):
    """pss_set_lookahead: depth 0 makes no slot; a byte cap of two slots keeps the draw slots
    within it (the peak device bytes of the capped engine exceed the depth-0 engine's by at most
    the cap); the default draws ahead -- and every epoch equals the exact oracle in all three."""
    s_off, peak_off = _check_epochs(B, version, EPOCHS[:8], lookahead=(0, 1 << 30, -1))
    assert s_off["exact_made"] == 0 and s_off["exact_used"] == 0, s_off
    lens, N, R = _shape(B)
    probe = IndexEngine(lens, N, R, B, version, device=0, order="exact")
    probe.set_lookahead(1, 1 << 30, -1)
    probe.init_iter(0)
    probe.generate(0, R)
    b0 = probe.workspace_bytes()
    probe.init_iter(1)
    probe.generate(0, R)              # queues one slot (epoch 2): its size
    slot = probe.workspace_bytes() - b0
    probe.close()
    assert slot > 0
    # a cap of 2.5 slots: at most two slots (the one a decode reads, one drawn ahead)
    cap = int(2.5 * slot)
    s_cap, peak_cap = _check_epochs(B, version, EPOCHS[:8], lookahead=(-1, cap, -1))
    assert s_cap["exact_used"] > 0, s_cap
    assert peak_cap - peak_off <= cap, (peak_cap, peak_off, cap)
    s_def, _ = _check_epochs(B, version, EPOCHS[:8])
    assert s_def["exact_used"] > 0, s_def


def test_leaving_the_exact_order_drops_the_slots_and_coming_back_restarts():
    B = 1 << 16
    lens, N, R = _shape(B)
    eng = IndexEngine(lens, N, R, B, 2, device=0, order="exact")
    ns = eng.num_samples

    def check(e):
        eng.init_iter(e)
        got = eng.generate(0, R).cpu().numpy()
        eng.check()
        old, new = eng.rank_starts()
        for r in range(R):
            ref = O.v2_exact_stream_rs(e, int(old[r]), int(new[r]), ns, B, N)
            assert np.array_equal(got[r], ref), ("epoch", e, "rank", r)

    for e in (0, 1, 2):          # 2 from a slot, 3.. queued
        check(e)
    eng.set_order_mode("counter")
    eng.init_iter(3)
    c = eng.generate(0, R).cpu().numpy()
    eng.check()
    assert c.shape == (R, ns) and c.min() >= 0 and c.max() < N
    eng.set_order_mode("exact")
    for e in (4, 5, 6):          # 4: own draws (the slots went), 5 queued by 4 ... 6 from a slot
        check(e)
    eng.close()


@pytest.mark.parametrize("B", [1000, 4096])
def test_v2_exact_odd_num_samples_several_ranks(B):
    """an odd num_samples puts the chain-mode decode's virtual indices (VV, after
    the odd-length per-position arrays) at an address that is not 16-byte aligned; the fan-out's
    16-byte loads must then take their scalar form.  R = 3, ns odd, with and without draw slots,
    against the exact oracle."""
    R = 3
    ns = 2 * B + 2 * (B // 3) + 1                     # odd
    N = ns * R - 1
    F = 37
    lens = np.full(F, N // F, dtype=np.int64)
    lens[-1] += N - lens.sum()
    for depth in (0, -1):
        eng = IndexEngine(lens, N, R, B, 2, device=0, order="exact")
        eng.set_lookahead(depth, 1 << 30, -1)
        assert eng.num_samples == ns and ns % 2 == 1
        for e in range(4):
            eng.init_iter(e)
            got = eng.generate(0, R).cpu().numpy()
            eng.check()
            old, new = eng.rank_starts()
            for r in range(R):
                ref = O.v2_exact_stream_rs(e, int(old[r]), int(new[r]), ns, B, N)
                assert np.array_equal(got[r], ref), ("epoch", e, "rank", r, "depth", depth)
        eng.close()
