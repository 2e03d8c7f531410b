"""The fused (file, offset) hand-off, pss_generate_mapped, against pss_generate + pss_map on the
same epoch (V1:181-221: the reference's id -> (file, offset) walk, restated by pss_map and pinned
by the map tests against the oracle), over the map's every path:

  * pair slots in the V2 exchange replay (MapArgs::pack: (file << pob) | offset in 31 bits),
    with windows of one, two and three files, windows that escape (three or more boundaries,
    tiny files; a block that wraps at N; ids past the files' total, reflected) and slot values
    older than the constants' reach;
  * the segment map (shapes whose pairs do not fit 31 bits: a huge file among many);
  * the uniform-length shortcut (every file the same length: file = id / L by a magic);
  * V1's one-shot kernel with per-window map segments (and its global-map fallback);
  * consecutive epochs (the V2 lookahead and the double-buffered epoch tables), partial ranges.
"""
import zlib

import numpy as np
import pytest
import torch

from partiallyshuffledistributedsampler_amd.engine import IndexEngine

pytestmark = pytest.mark.gpu


def _lengths(kind, rng):
    if kind == "uniform":
        return np.full(40, 7000, dtype=np.int64)
    if kind == "varied":
        return rng.integers(3000, 12000, 40)
    if kind == "tiny":                       # hundreds of files per window: every window escapes
        return rng.integers(1, 9, 4000)
    if kind == "mixed":                      # 1-3 files per window, some windows with 3+
        return np.concatenate([rng.integers(1500, 6000, 30), rng.integers(1, 300, 60)])
    if kind == "empty":                      # empty files between non-empty ones
        ln = rng.integers(2000, 9000, 50)
        ln[rng.integers(0, 50, 12)] = 0
        return ln
    if kind == "huge":                       # (F - 1) << 21 > 2^31: no pair slots
        ln = rng.integers(1, 40, 1200)
        ln[7] = 1_500_000
        return ln
    raise ValueError(kind)


def _check(eng, R, ns, r0, r1, pos_lo, count, fpos, off):
    f2, o2 = eng.generate_mapped(r0, r1, pos_lo, count)
    eng.check()
    c = min(count, ns - pos_lo)
    assert torch.equal(f2[:, :c].cpu(), fpos[r0:r1, pos_lo:pos_lo + c].cpu()), (r0, r1, pos_lo, count)
    assert torch.equal(o2[:, :c].long().cpu(), off[r0:r1, pos_lo:pos_lo + c].cpu()), (r0, r1, pos_lo, count)


@pytest.mark.parametrize("version", [1, 2])
@pytest.mark.parametrize("kind,R,B,extra", [
    ("uniform", 4, 4096, 0),
    ("uniform", 3, 4096, 1234),     # ids past the files' total: reflected (escapes)
    ("varied", 4, 4096, 0),
    ("varied", 5, 1024, 0),
    ("varied", 3, 1000, 0),         # B not a power of 4: cycle-walking windows
    ("tiny", 3, 2048, 0),
    ("mixed", 4, 4096, 0),
    ("empty", 4, 4096, 0),
    ("huge", 2, 4096, 0),
    ("uniform", 2, 65536, 0),       # grouped pools (V2) / big windows (V1)
    ("varied", 2, 20000, 0),
])
def test_generate_mapped_equals_generate_then_map(version, kind, R, B, extra):
    rng = np.random.default_rng(zlib.crc32(repr((kind, R, B, extra)).encode()))
    lengths = _lengths(kind, rng)
    N = int(lengths.sum()) + extra
    eng = IndexEngine(lengths, N, R, B, version, seed=11, device=0)
    ns = eng.num_samples
    for epoch in (0, 1, 2, 3, 4):
        eng.init_iter(epoch)
        ids = eng.generate(0, R)
        fpos, off = eng.map(ids.reshape(-1))
        fpos, off = fpos.reshape(R, -1), off.reshape(R, -1)
        _check(eng, R, ns, 0, R, 0, ns, fpos, off)
        if epoch in (1, 3):
            for r0, r1, pos_lo, count in ((1, R, 7, 3 * B + 5), (0, R - 1, ns // 2, 999),
                                          (0, R, max(0, ns - B - 3), B + 9)):
                _check(eng, R, ns, r0, r1, pos_lo, count, fpos, off)
    eng.close()


def test_mapped_consecutive_epochs_lookahead_and_tables():
    """Eight consecutive whole-epoch calls (the V2 pass of e + 1, e + 2 queued ahead, the epoch
    tables of e built beside e - 1's replay), each checked afterwards against generate + map
    of a fresh engine replaying the same history."""
    rng = np.random.default_rng(5)
    lengths = rng.integers(4000, 11000, 60)
    N, R, B = int(lengths.sum()), 4, 4096
    for version in (1, 2):
        a = IndexEngine(lengths, N, R, B, version, seed=3, device=0)
        outs = []
        for e in range(8):
            a.init_iter(e)
            outs.append(a.generate_mapped(0, R))
        torch.cuda.synchronize()
        b = IndexEngine(lengths, N, R, B, version, seed=3, device=0)
        for e in range(8):
            b.init_iter(e)
            ids = b.generate(0, R)
            f, o = b.map(ids.reshape(-1))
            assert torch.equal(outs[e][0].cpu(), f.reshape(R, -1).cpu()), (version, e)
            assert torch.equal(outs[e][1].long().cpu(), o.reshape(R, -1).cpu()), (version, e)
        a.close()
        b.close()


@pytest.mark.parametrize("v2_depth", [0, 1, 2])
def test_v2_lookahead_depths_give_the_same_streams(v2_depth):
    """pss_set_lookahead's V2 depth (0: the last-occurrence pass in line; 1, 2 epochs queued
    ahead): ids and the fused hand-off over consecutive epochs equal a default engine's, and the
    counters show the queued passes used (or none at depth 0)."""
    rng = np.random.default_rng(9)
    lengths = rng.integers(3000, 9000, 50)
    N, R, B = int(lengths.sum()), 3, 4096
    a = IndexEngine(lengths, N, R, B, 2, seed=2, device=0)
    b = IndexEngine(lengths, N, R, B, 2, seed=2, device=0)
    b.set_lookahead(-1, 1 << 30, v2_depth)
    for e in range(7):
        a.init_iter(e)
        b.init_iter(e)
        assert torch.equal(a.generate(0, R).cpu(), b.generate(0, R).cpu()), (v2_depth, e)
    for e in range(7, 12):
        a.init_iter(e)
        b.init_iter(e)
        fa, oa = a.generate_mapped(0, R)
        fb, ob = b.generate_mapped(0, R)
        assert torch.equal(fa.cpu(), fb.cpu()) and torch.equal(oa.cpu(), ob.cpu()), (v2_depth, e)
    st = b.lookahead_stats()
    if v2_depth == 0:
        assert st["v2_queued"] == 0 and st["v2_used"] == 0, st
    else:
        assert st["v2_used"] >= 8, st
    a.close()
    b.close()
