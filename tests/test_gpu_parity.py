"""GPU parity: the HIP path (through the C-ABI) against the CPU oracle.

  * Philox schedule: GPU streams == oracle/pss_oracle.c twin, bit for bit;
  * reference parity: file order / blocks / start_num == the reference's (goldens + oracle),
    per-rank epoch multiset == the reference's exact stream's multiset;
  * coverage: all ranks together cover [0, N) plus the pad, no duplicates or drops;
  * id -> (file, offset) map and file -> rank partition == oracle.
"""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from tests.golden_util import fixture_params, load, scenario_names

pytestmark = pytest.mark.gpu

pss = pytest.importorskip("partiallyshuffledistributedsampler_amd.engine")


class _Checked(pss.IndexEngine):
    """IndexEngine whose every generate / map is followed by pss_check (device error flag)."""

    def generate(self, *a, **kw):
        out = super().generate(*a, **kw)
        self.check(kw.get("stream"))
        return out

    def map(self, *a, **kw):
        r = super().map(*a, **kw)
        self.check(kw.get("stream"))
        return r


def _engine(lengths, N, R, B, version, shuffle=True, seed=0, order="counter"):
    return _Checked(lengths, N, R, B, version, shuffle=shuffle, seed=seed, device=0, order=order)


def _oracle_stream(version, key, rank, old, new, ns, B, N, shuffle=True):
    if version == 1:
        return O.v1_philox_stream(key, rank, new, ns, B, N, shuffle)
    return O.v2_philox_stream(key, rank, old, new, ns, B, N)


def test_dpp_wave_scan():
    from partiallyshuffledistributedsampler_amd import _lib
    import ctypes
    rng = np.random.default_rng(1)
    x = rng.integers(0, 2 ** 40, 64 * 37, dtype=np.int64)
    xin = torch.from_numpy(x).cuda()
    out = torch.empty(2 * len(x), dtype=torch.int64, device="cuda")
    _lib.call("pss_debug_wave_scan", ctypes.c_void_p(xin.data_ptr()), ctypes.c_void_p(out.data_ptr()),
              len(x), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    got = out.cpu().numpy().reshape(-1, 2)
    ref64 = np.cumsum(x.reshape(-1, 64).astype(np.uint64), axis=1).reshape(-1)
    ref32 = np.cumsum((x.reshape(-1, 64) & 0xFFFFFFFF).astype(np.uint64), axis=1).reshape(-1) & 0xFFFFFFFF
    assert np.array_equal(got[:, 0].astype(np.uint64), ref64)
    assert np.array_equal(got[:, 1].astype(np.uint64), ref32)


CONFIGS = [
    # (F, len lo/hi, R, B)
    (64, (100, 300), 2, 64),
    (37, (1, 900), 7, 40),
    (200, (50, 2000), 4, 4096),
    (50, (1000, 5000), 3, 3000),
    (40, (2000, 9000), 2, 8192),
    (10, (10000, 40000), 2, 16384),
    (13, (1, 50), 5, 100),        # ns < B
    (9, (20, 40), 2, 70),         # B < ns < 2B
    (100, (1, 3), 8, 7),          # tiny windows
    (20, (5000, 20000), 2, 20000),      # pools beyond LDS: HBM multi-pass sort / HBM slot table
    (12, (50000, 100000), 3, 70001),    # ... odd pool size, partial last window
    (6, (1000, 3000), 2, 100000),       # ns < B with a big pool: tail only
]


@pytest.mark.parametrize("version", [1, 2])
@pytest.mark.parametrize("cfg", CONFIGS)
def test_streams_match_oracle_twin(version, cfg):
    F, (lo, hi), R, B = cfg
    rng = np.random.default_rng(F * 1000 + R)
    lengths = rng.integers(lo, hi, F)
    N = int(lengths.sum())
    eng = _engine(lengths, N, R, B, version, seed=1234)
    ns = eng.num_samples
    for epoch in (0, 3):
        eng.init_iter(epoch)
        old, new = eng.rank_starts()
        out = eng.generate(0, R).cpu().numpy()
        key = O.epoch_key(1234, epoch)
        for r in range(R):
            ref = _oracle_stream(version, key, r, int(old[r]), int(new[r]), ns, B, N)
            assert np.array_equal(out[r], ref), (cfg, version, epoch, r)
        # coverage: every id of [0, N) exactly once, plus the wrap-around pad (V1:161-163)
        allids = np.sort(out.reshape(-1))
        pad = ns * R - N
        expect = np.sort(np.concatenate([np.arange(N), np.arange(pad)]))
        assert np.array_equal(allids, expect)


@pytest.mark.parametrize("F,lo,hi,R,B", [(200, 50, 2000, 4, 4096), (64, 100, 300, 2, 64),
                                        (30, 20000, 60000, 3, 1000),
                                        (20, 20000, 60000, 2, 20000),    # pools beyond LDS
                                        (8, 100000, 200000, 2, 65536)])
def test_v2_epoch_lookahead_matches_oracle(F, lo, hi, R, B):
    """Consecutive epochs of one shape take their last-occurrence pass from the lookahead queued
    on the side stream by the previous generate; skipped / repeated epochs and shape changes in
    between must fall back to the full launch.  Every stream == the oracle twin."""
    rng = np.random.default_rng(F + B)
    lengths = rng.integers(lo, hi, F)
    N = int(lengths.sum())
    eng = _engine(lengths, N, R, B, 2, seed=77)
    ns = eng.num_samples
    # (epoch, ranks, emit path): "probe" calls take the unsplit path between lookaheads
    plan = [(0, 0, R, "xchg"), (1, 0, R, "xchg"), (2, 0, R, "xchg"), (3, 0, R, "xchg"),
            (5, 0, R, "xchg"), (6, 0, R, "xchg"), (6, 0, R, "xchg"), (7, 1, R, "xchg"),
            (8, 0, R, "xchg"), (9, 0, R, "xchg"), (10, 0, R, "probe"), (11, 0, R, "xchg"),
            (12, 0, R, "xchg"), (13, 0, R, "xchg"), (14, 1, R, "xchg"), (15, 0, R, "xchg"),
            (16, 1, R, "xchg")] + [(e, 0, R, "xchg") for e in range(17, 25)]
    outs = []
    for epoch, r0, r1, path in plan:
        eng.set_emit_path(path)
        eng.init_iter(epoch)
        old, new = eng.rank_starts()
        outs.append((epoch, r0, r1, eng.generate(r0, r1), np.asarray(old).copy(), np.asarray(new).copy()))
    torch.cuda.synchronize()
    for epoch, r0, r1, out, old, new in outs:
        out = out.cpu().numpy()
        key = O.epoch_key(77, epoch)
        for r in range(r0, r1):
            ref = _oracle_stream(2, key, r, int(old[r]), int(new[r]), ns, B, N)
            assert np.array_equal(out[r - r0], ref), (epoch, r)


@pytest.mark.parametrize("version", [1, 2])
def test_position_ranges_and_resume(version):
    rng = np.random.default_rng(5)
    lengths = rng.integers(500, 3000, 60)
    N, R, B = int(lengths.sum()), 4, 1000
    eng = _engine(lengths, N, R, B, version)
    eng.init_iter(2)
    full = eng.generate(0, R).cpu().numpy()
    ns = eng.num_samples
    for pos_lo, count in ((0, 1), (1, 999), (999, 2), (1234, 4321), (ns - 7, 100), (ns - B - 3, B + 3)):
        part = eng.generate(1, 3, pos_lo, count).cpu().numpy()
        c = min(count, ns - pos_lo)
        assert np.array_equal(part[:, :c], full[1:3, pos_lo:pos_lo + c]), (pos_lo, count)


@pytest.mark.parametrize("name", scenario_names("v1") + scenario_names("v2"))
def test_reference_assignment_and_multiset(name):
    """Against the reference's recorded goldens: file order, blocks, start_num bit-exact;
    per-rank epoch multiset == the reference's stream multiset."""
    fx = load(name)
    files, lengths, fl, N, R, B, bs, shuffle = fixture_params(fx)
    version = 1 if fx["version"] == "v1" else 2
    lens = [fl.get(p, lengths[p]) if fl else lengths[p] for p in files]
    eng = _engine(lens, N, R, B, version, shuffle=shuffle)
    for ep_i, er0 in enumerate(fx["ranks"][0]["epochs"]):
        eng.init_iter(er0["epoch"])
        order = eng.file_order()
        assert [files[i] for i in order] == er0["files"]
        assert eng.blocks().tolist() == er0["blocks"]
        old, new = eng.rank_starts()
        out = eng.generate(0, R).cpu().numpy()
        for rrec in fx["ranks"]:
            r = rrec["rank"]
            er = rrec["epochs"][ep_i]
            assert int(new[r]) == er["start_num"] and int(old[r]) == er["old_start"]
            if er.get("resume_step") is not None:
                continue  # resume multiset differs by design (V1 lossy resume), tested elsewhere
            if version == 1:
                ref = O.v1_exact_stream(er["epoch"], er["start_num"], eng.num_samples, B, N, shuffle)
            else:
                ref = O.v2_exact_stream(er["epoch"], er["old_start"], er["start_num"], eng.num_samples, B, N)
            assert np.array_equal(np.sort(out[r]), np.sort(ref)), (name, r)
            if not shuffle and version == 1:   # identity order: sequence parity too
                rec = [x for b in er["batches"] for x in b]
                assert out[r][:len(rec)].tolist() == rec


@pytest.mark.parametrize("F,hi", [(300, 500), (4096, 40), (4097, 40), (20_000, 60)])
def test_map_and_partition_match_oracle(F, hi):
    # one scan chunk (F <= 4096) and several (two-pass scan); empty files included
    rng = np.random.default_rng(11 + F)
    lengths = rng.integers(0, hi, F)
    N, R, B = int(lengths.sum()), 6, 256
    for version in (1, 2):
        eng = _engine(lengths, N, R, B, version)
        eng.init_iter(7)
        order = eng.file_order()
        prefix = np.concatenate([[0], np.cumsum(lengths[order])])
        ids = eng.generate(0, R)
        fpos, off = eng.map(ids.reshape(-1))
        rf, ro = O.map_ids(prefix, ids.cpu().numpy().reshape(-1))
        assert np.array_equal(fpos.cpu().numpy(), rf)
        assert np.array_equal(off.cpu().numpy(), ro)
        seg_off, sf, sl, sh = eng.partition(0, R)
        idsn = ids.cpu().numpy()
        for r in range(R):
            segs = set()
            for k in range(seg_off[r], seg_off[r + 1]):
                segs.add(int(sf[k]))
                assert 0 <= sl[k] < sh[k] <= lengths[order[sf[k]]]
            f_r, _ = O.map_ids(prefix, idsn[r])
            assert segs == set(f_r.tolist())
            assert sum(int(sh[k] - sl[k]) for k in range(seg_off[r], seg_off[r + 1])) == eng.num_samples


def test_map_reflection_flags():
    lengths = np.array([5, 7, 3])
    eng = _engine(lengths, 20, 2, 4, 1)   # N=20 > T=15: ids >= 15 reflect
    eng.init_iter(0)
    ids = torch.tensor([0, 14, 15, 16, 19], dtype=torch.int64, device="cuda")
    fpos, off = eng.map(ids)
    order = eng.file_order()
    prefix = np.concatenate([[0], np.cumsum(lengths[order])])
    T = prefix[-1]
    for i, x in enumerate([0, 14, 15, 16, 19]):
        refl = x >= T
        y = 2 * T - x if refl else x
        if refl and y == T:
            y = T - 1
        f = int(np.searchsorted(prefix, y, side="right") - 1)
        while prefix[f + 1] == prefix[f]:
            f += 1
        assert int(fpos[i]) == (-1 - f if refl else f)
        assert int(off[i]) == y - prefix[f]


def test_digest_matches_oracle():
    rng = np.random.default_rng(3)
    x = rng.integers(0, 2 ** 40, 100_003, dtype=np.int64)
    acc = pss.digest(torch.from_numpy(x).cuda())
    assert pss.as_u64(acc) == O.digest(x)
    acc = pss.digest_range(5, 1_000_005, 0)
    assert pss.as_u64(acc) == O.digest_range(5, 1_000_005)


def test_v2_displacement_bounds():
    # an id of virtual index v is emitted no earlier than position v - 2B (V2:96-116)
    rng = np.random.default_rng(8)
    lengths = rng.integers(1000, 3000, 100)
    N, R, B = int(lengths.sum()), 2, 512
    eng = _engine(lengths, N, R, B, 2)
    eng.init_iter(1)
    old, new = eng.rank_starts()
    out = eng.generate(0, R).cpu().numpy()
    ns = eng.num_samples
    for r in range(R):
        v = np.where((out[r] - old[r]) % N < 2 * B, (out[r] - old[r]) % N, (out[r] - new[r]) % N)
        pos = np.arange(ns)
        assert (pos - v).min() >= -2 * B
        assert np.array_equal(np.sort(v), np.arange(ns))


def test_exchange_emit_path_is_the_default():
    # MI355X passes the start-up lane-order check -- the synthetic exchange patterns AND the
    # replay cross-check (k_v2_emit_x == the order-free probe replay k_v2_emit on two real
    # geometries, pss_v2.hip xchg_replay_crosscheck): the one-exchange-per-step kernel runs
    eng = _engine(np.full(10, 1000), 10000, 2, 256, 2)
    assert eng.emit_path() == "xchg"


@pytest.mark.parametrize("path", ["xchg", "probe"])
@pytest.mark.parametrize("B,R,F,lo,hi", [(4096, 3, 40, 5000, 9000), (1000, 4, 60, 500, 3000),
                                         (300, 2, 30, 100, 900), (64, 5, 20, 10, 200),
                                         (2048, 2, 8, 10000, 40000)])
def test_v2_emit_paths_match_oracle(path, B, R, F, lo, hi):
    # both replay kernels, full epochs and ragged position ranges, against the oracle twin
    rng = np.random.default_rng(B + R)
    lengths = rng.integers(lo, hi, F)
    N = int(lengths.sum())
    eng = _engine(lengths, N, R, B, 2, seed=99)
    eng.set_emit_path(path)
    ns = eng.num_samples
    eng.init_iter(4)
    old, new = eng.rank_starts()
    full = eng.generate(0, R).cpu().numpy()
    key = O.epoch_key(99, 4)
    for r in range(R):
        assert np.array_equal(full[r], O.v2_philox_stream(key, r, int(old[r]), int(new[r]), ns, B, N)), r
    for pos_lo, count in ((0, 63), (5, 300), (B - 1, 2 * B + 7), (ns // 2, 999), (ns - 100, 100)):
        part = eng.generate(0, R, pos_lo, count).cpu().numpy()
        c = min(count, ns - pos_lo)
        assert np.array_equal(part[:, :c], full[:, pos_lo:pos_lo + c]), (pos_lo, count)


@pytest.mark.parametrize("F,lo,hi,R,B,extra", [
    (40, 5000, 9000, 3, 4096, 0),      # many tiles, a few files per staged interval
    (3000, 1, 6, 2, 256, 0),           # hundreds of tiny files per interval: global fallback
    (60, 500, 3000, 4, 1000, 777),     # N past the files' total: reflected ids (fallback)
    (50, 100, 400, 5, 64, 0),          # tiny windows
    (13, 1, 50, 5, 100, 0),            # ns < B: tail only
    (8, 20000, 60000, 2, 16384, 0),    # the largest LDS pool
    (20, 5000, 20000, 2, 20000, 0),    # grouped pools (P1 > 16384): mapped in the grouped replay
    (12, 50000, 100000, 3, 70001, 555),  # ... odd pool, partial last window, reflected ids
    (40, 20000, 20001, 2, 65536, 0)])  # ... groups of 4096 slots (paired draws, run loop)
def test_v2_fused_mapping_matches_generate_then_map(F, lo, hi, R, B, extra):
    """pss_generate_mapped maps inside the V2 replay (pools that fit LDS: the per-tile LDS
    segment map, global bucketed map outside it; grouped pools: the global bucketed map in the
    grouped replay): equal to generate + pss_map for full epochs, ragged and tail-only position
    ranges, and consecutive epochs served by the lookahead."""
    rng = np.random.default_rng(F + B + extra)
    lengths = rng.integers(lo, hi, F)
    N = int(lengths.sum()) + extra
    eng = _engine(lengths, N, R, B, 2, seed=5)
    ns = eng.num_samples
    for epoch in (0, 1, 2, 3):
        eng.init_iter(epoch)
        ids = eng.generate(0, R)
        fpos, off = eng.map(ids.reshape(-1))
        fpos, off = fpos.reshape(R, -1), off.reshape(R, -1)
        for r0, r1, pos_lo, count in ((0, R, 0, ns), (1, R, 7, 3 * B + 5), (0, R - 1, ns // 2, 999),
                                      (0, R, max(0, ns - 5), 5), (0, R, max(0, ns - B - 3), B + 9)):
            f2, o2 = eng.generate_mapped(r0, r1, pos_lo, count)
            eng.check()
            c = min(count, ns - pos_lo)
            assert torch.equal(f2[:, :c].cpu(), fpos[r0:r1, pos_lo:pos_lo + c].cpu()), (epoch, r0, pos_lo, count)
            assert torch.equal(o2[:, :c].long().cpu(), off[r0:r1, pos_lo:pos_lo + c].cpu()), (epoch, r0, pos_lo, count)
        # the full epoch again as the first call of the epoch (the lookahead's replay stage)
        eng.init_iter(epoch + 10)
        f3, o3 = eng.generate_mapped(0, R)
        ids3 = eng.generate(0, R)
        fp3, of3 = eng.map(ids3.reshape(-1))
        assert torch.equal(f3.cpu(), fp3.reshape(R, -1).cpu()) and torch.equal(o3.long().cpu(), of3.reshape(R, -1).cpu())


@pytest.mark.parametrize("path", ["xchg", "probe"])
@pytest.mark.parametrize("B,R,F,lo,hi", [(20000, 3, 30, 5000, 20000), (65536, 2, 40, 10000, 30000),
                                         (16385, 4, 20, 3000, 9000), (131072, 2, 12, 40000, 80000),
                                         (20000, 8, 60, 19000, 21000)])   # 16 tiles: XCD-grouped replay
def test_v2_large_pool_paths_match_oracle(path, B, R, F, lo, hi):
    # pools beyond the LDS slot table: slot-chunked replay ("xchg") and the HBM slot table
    # ("probe"), full epochs and ragged position ranges, against the oracle twin
    rng = np.random.default_rng(B + R + F)
    lengths = rng.integers(lo, hi, F)
    N = int(lengths.sum())
    eng = _engine(lengths, N, R, B, 2, seed=5)
    eng.set_emit_path(path)
    ns = eng.num_samples
    assert ns > B
    for epoch in (0, 2):
        eng.init_iter(epoch)
        old, new = eng.rank_starts()
        full = eng.generate(0, R).cpu().numpy()
        key = O.epoch_key(5, epoch)
        for r in range(R):
            ref = O.v2_philox_stream(key, r, int(old[r]), int(new[r]), ns, B, N)
            assert np.array_equal(full[r], ref), (epoch, r, int(np.argmax(full[r] != ref)))
    for pos_lo, count in ((0, 100), (B - 5, 3 * B), (ns // 3, 12345), (ns - B - 10, 50), (ns - 7, 7)):
        part = eng.generate(0, R, pos_lo, count).cpu().numpy()
        c = min(count, ns - pos_lo)
        assert np.array_equal(part[:, :c], full[:, pos_lo:pos_lo + c]), (pos_lo, count)


# ---- exact-order mode (V1): the reference's own CPython-MT window shuffles ----------------
@pytest.mark.parametrize("name", scenario_names("v1"))
def test_v1_exact_order_matches_reference_streams(name):
    """order="exact": every rank's id stream equals the stream the reference itself produced
    (tests/golden, captured from V1:178), not only its multiset."""
    fx = load(name)
    files, lengths, fl, N, R, B, bs, shuffle = fixture_params(fx)
    lens = [fl.get(p, lengths[p]) if fl else lengths[p] for p in files]
    eng = _engine(lens, N, R, B, 1, shuffle=shuffle, seed=0, order="exact")
    assert eng.order_mode() == "exact"
    for ep_i, er0 in enumerate(fx["ranks"][0]["epochs"]):
        eng.init_iter(er0["epoch"])
        out = eng.generate(0, R).cpu().numpy()
        for rrec in fx["ranks"]:
            er = rrec["epochs"][ep_i]
            if er.get("resume_step") is not None:
                continue   # the reference's lossy resume (V1:139) is not reproduced
            # the reference's recorded raw stream (its batches, in order) is a prefix of ours
            rec = [x for b in er["batches"] for x in b]
            assert out[rrec["rank"]][:len(rec)].tolist() == rec, (name, rrec["rank"], er["epoch"])
            ref = O.v1_exact_stream(er["epoch"], er["start_num"], eng.num_samples, B, N, shuffle)
            assert np.array_equal(out[rrec["rank"]], ref), (name, rrec["rank"], er["epoch"])


@pytest.mark.parametrize("F,lo,hi,R,B,epochs", [
    (64, 10000, 10001, 2, 4096, (0, 1)),            # C1 (BASELINE configs[0])
    (37, 1, 900, 7, 40, (0, 5)),
    (50, 1000, 5000, 3, 3000, (2,)),                # partial last window
    (40, 2000, 9000, 2, 8192, (1,)),
    (30, 5000, 9000, 2, 12345, (3,)),               # partial last window, odd size
    (40, 5000, 9000, 2, 16000, (1,)),               # largest exact window in LDS
    (40, 5000, 9000, 2, 16001, (1,)),               # smallest window of the HBM path
    (40, 5000, 9000, 2, 16384, (0, 1)),             # HBM path, partial last window
    (30, 20000, 60000, 3, 65536, (2,)),
    (70, 100000, 100001, 2, 1 << 20, (0, 2 ** 32 - 3)),   # C5's pool: B = 2^20, 3.3 windows per rank
    (13, 1, 50, 5, 100, (0, 9)),                    # ns < B
    (100, 1, 3, 8, 7, (0,)),                        # tiny windows
    (30, 100, 400, 3, 257, (2 ** 32 - 30000,)),     # window seeds cross 2^32 (two-word MT keys)
])
def test_v1_exact_order_matches_exact_oracle(F, lo, hi, R, B, epochs):
    rng = np.random.default_rng(F + B)
    lengths = rng.integers(lo, hi, F)
    N = int(lengths.sum())
    eng = _engine(lengths, N, R, B, 1, seed=7, order="exact")
    ns = eng.num_samples
    for epoch in epochs:
        eng.init_iter(epoch)
        _, new = eng.rank_starts()
        out = eng.generate(0, R).cpu().numpy()
        for r in range(R):
            ref = O.v1_exact_stream(epoch, int(new[r]), ns, B, N, True)
            assert np.array_equal(out[r], ref), (F, B, epoch, r)
        if ns > 3:   # position sub-ranges come out of the same windows
            lo_p, cnt = ns // 3, ns // 2
            part = eng.generate(1, R, lo_p, cnt).cpu().numpy()
            assert np.array_equal(part, out[1:, lo_p:lo_p + cnt])


def test_exact_order_unsupported_configs():
    """The GPU exact orders' bounds (pss.h): V1 shuffle_buffer < 2^31, V2 num_samples < 2^31
    and shuffle_buffer < 2^30; the handle refuses others at pss_set_order_mode (no launch)."""
    from partiallyshuffledistributedsampler_amd import _lib
    lengths = np.full(10, 1000)
    with pytest.raises(_lib.PSSError):
        pss.IndexEngine(lengths, 10000, 2, 2 ** 31, 1, device=0, order="exact")     # V1, B >= 2^31
    with pytest.raises(_lib.PSSError):
        pss.IndexEngine(lengths, 10000, 2, 2 ** 30, 2, device=0, order="exact")     # V2, B >= 2^30
    big = np.full(4, 2 ** 30)
    with pytest.raises(_lib.PSSError):
        pss.IndexEngine(big, 2 ** 32, 2, 4096, 2, device=0, order="exact")          # V2, ns = 2^31
    pss.IndexEngine(lengths, 10000, 2, 2 ** 20, 1, device=0, order="exact").close()  # V1 big windows: accepted


@pytest.mark.parametrize("name", scenario_names("v2"))
def test_v2_exact_order_matches_reference_streams(name):
    """order="exact" on V2: each rank's id stream equals the one the reference produced
    (tests/golden, captured at V2:181) and the exact oracle's."""
    fx = load(name)
    files, lengths, fl, N, R, B, bs, shuffle = fixture_params(fx)
    lens = [fl.get(p, lengths[p]) if fl else lengths[p] for p in files]
    eng = _engine(lens, N, R, B, 2, seed=0, order="exact")
    for ep_i, er0 in enumerate(fx["ranks"][0]["epochs"]):
        eng.init_iter(er0["epoch"])
        out = eng.generate(0, R).cpu().numpy()
        for rrec in fx["ranks"]:
            er = rrec["epochs"][ep_i]
            ref = O.v2_exact_stream(er["epoch"], er["old_start"], er["start_num"], eng.num_samples, B, N)
            assert np.array_equal(out[rrec["rank"]], ref), (name, rrec["rank"], er["epoch"])
            if er.get("resume_step") is not None:
                continue   # the recorded batches start at the resume point
            rec = [x for b in er["batches"] for x in b]
            assert out[rrec["rank"]][:len(rec)].tolist() == rec, (name, rrec["rank"], er["epoch"])


@pytest.mark.parametrize("F,lo,hi,R,B,epochs", [
    (37, 1, 900, 7, 40, (0, 5)),
    (50, 1000, 5000, 3, 3000, (2,)),                # partial last pool2 window
    (40, 2000, 9000, 2, 4096, (1,)),                # pool2 windows of one decode tile
    (13, 1, 50, 5, 100, (0, 9)),                    # ns < B: tail only
    (9, 20, 40, 2, 70, (3,)),                       # B < ns < 2B
    (100, 1, 3, 8, 7, (0,)),                        # tiny pools
    (64, 3000, 3001, 2, 1000, (4,)),                # many global decode levels (ns = 96000)
    (40, 2000, 9000, 2, 4097, (1,)),                # windows beyond one decode tile
    (30, 2000, 4000, 3, 5000, (0, 2)),              # ... partial last window (padded steps)
    (60, 3000, 4000, 2, 20000, (3,)),               # pool1 > 4096: table-free global levels
    (25, 3000, 9000, 1, 70001, (1,)),               # a big pool, one rank, few windows
])
def test_v2_exact_order_matches_exact_oracle(F, lo, hi, R, B, epochs):
    rng = np.random.default_rng(F * 7 + B)
    lengths = rng.integers(lo, hi, F)
    N = int(lengths.sum())
    eng = _engine(lengths, N, R, B, 2, seed=7, order="exact")
    ns = eng.num_samples
    for epoch in epochs:
        eng.init_iter(epoch)
        old, new = eng.rank_starts()
        out = eng.generate(0, R).cpu().numpy()
        for r in range(R):
            ref = O.v2_exact_stream(epoch, int(old[r]), int(new[r]), ns, B, N)
            assert np.array_equal(out[r], ref), (F, B, epoch, r)
        if ns > 3:
            lo_p, cnt = ns // 3, ns // 2
            part = eng.generate(1, R, lo_p, cnt).cpu().numpy()
            assert np.array_equal(part, out[1:, lo_p:lo_p + cnt])


@pytest.mark.parametrize("version", [1, 2])
@pytest.mark.parametrize("cfg", CONFIGS + [(10_000, (10_000, 10_001), 8, 1 << 20)])
def test_gpu_equals_cpu_mode(version, cfg):
    """north_star: the internal CPU mode of the counter schedule matches the GPU bit for bit
    (same engine API, device="cpu" vs the HIP kernels), including the C5 pool (B = 2^20)."""
    F, (lo, hi), R, B = cfg
    rng = np.random.default_rng(F * 1000 + R + 1)
    lengths = rng.integers(lo, hi, F)
    N = int(lengths.sum())
    gpu = _engine(lengths, N, R, B, version, seed=99)
    cpu = pss.IndexEngine(lengths, N, R, B, version, seed=99, device="cpu")
    for epoch in (1, 2):
        gpu.init_iter(epoch)
        cpu.init_iter(epoch)
        a = gpu.generate(0, R).cpu().numpy()
        b = cpu.generate(0, R).numpy()
        assert np.array_equal(a, b), (cfg, version, epoch)
