"""Bench-scale reference goldens (tests/golden/big, made by tools/gen_golden_big.py from the
reference itself), CPU side:

  * the oracle's exact restatements reproduce every recorded reference stream -- V1 windows up
    to B = 2^20 (C5's pool, 12 windows per rank), V2 at B = 4096 / 400 / 65536 (incl. the
    per-step reseeding tail and two-word MT seeds) and the first 20480 draws at C5's B = 2^20;
  * the library's host history (pss_init_iter, the file -> rank assignment) reproduces the
    reference's file order / blocks / start_num at C3 (100K files, R = 1024) and C4 (Zipf,
    R = 4096) over init_iter(0, 1, 1, 9) -- V1:113-125, V2:142-152;
  * the product's CPU mode (device="cpu"): order="exact" == the reference stream, and the
    default counter order has the reference's per-rank epoch multiset.

The GPU side of the same fixtures is tests/test_gpu_golden_big.py."""
import numpy as np
import pytest

from oracle import oracle as O
from tests.golden_util import (big_lengths, big_names, check_multiset, check_stream, load_big,
                               load_big_streams, sha256_i64)

pss = pytest.importorskip("partiallyshuffledistributedsampler_amd.engine")

STREAMS = big_names("stream") + big_names("prefix")


def _walk(fx, eng):
    """Replay the fixture's init_iter sequence on `eng`, yielding (rank, epoch record) after
    checking the engine's (old, new) start of each recorded rank."""
    ranks = fx["ranks"]
    for i, er0 in enumerate(ranks[0]["epochs"]):
        eng.init_iter(er0["epoch"])
        old, new = eng.rank_starts()
        for rr in ranks:
            er = rr["epochs"][i]
            r = rr["rank"]
            assert (int(old[r]), int(new[r])) == (er["old_start"], er["start_num"]), (r, er["epoch"])
            yield r, er


def _oracle_stream(fx, er, ns, N):
    B, e = fx["B"], er["epoch"]
    if fx["version"] == 1:
        return O.v1_exact_stream(e, er["start_num"], ns, B, N)
    if fx["kind"] == "prefix":
        return O.v2_exact_prefix(e, er["old_start"], er["start_num"], ns, B, N, fx["prefix"])
    if B > 20000:
        return O.v2_exact_stream_rs(e, er["old_start"], er["start_num"], ns, B, N)
    return O.v2_exact_stream(e, er["old_start"], er["start_num"], ns, B, N)


@pytest.mark.parametrize("name", STREAMS)
def test_oracle_reproduces_reference_stream(name):
    fx = load_big(name)
    lens = big_lengths(fx)
    N, R = int(lens.sum()), fx["R"]
    ns = O.num_samples(N, R)
    full = load_big_streams(name) if fx.get("full_npz") else {}
    for rr in fx["ranks"]:
        assert rr["num_samples"] == ns
        h = O.RefHistory(fx["version"], len(lens), R, rr["rank"], N)
        for er in rr["epochs"]:
            h.init_iter(er["epoch"])
            assert (h.old_start, h.start) == (er["old_start"], er["start_num"])
            got = _oracle_stream(fx, er, ns, N)
            what = "%s r%d e%d" % (name, rr["rank"], er["epoch"])
            check_stream(got, er, fx, what)
            key = "r%d_e%d" % (rr["rank"], er["epoch"])
            if key in full:
                assert np.array_equal(got, full[key]), what


@pytest.mark.parametrize("name", big_names("assignment"))
def test_host_assignment_matches_reference_at_scale(name):
    """pss_init_iter's CPython-MT file order, blocks and start_num (old and new) == the
    reference's, for every rank, over the cumulative init_iter(0, 1, 1, 9) history."""
    fx = load_big(name)
    lens = big_lengths(fx)
    N, R, B = int(lens.sum()), fx["R"], fx["B"]
    assert N == fx["N"]
    for ver in (1, 2):
        eng = pss.IndexEngine(lens, N, R, B, ver, device="cpu")
        ns = eng.num_samples
        for rec in fx["versions"]["v%d" % ver]:
            eng.init_iter(rec["epoch"])
            assert ns == rec["num_samples"]
            order = eng.file_order().astype(np.int64)
            assert order[:32].tolist() == rec["order_head"], (ver, rec["epoch"])
            assert sha256_i64(order) == rec["order_sha256"], (ver, rec["epoch"])
            blocks = eng.blocks().astype(np.int64)
            assert sha256_i64(blocks) == rec["blocks_sha256"], (ver, rec["epoch"])
            old, new = eng.rank_starts()
            assert sha256_i64(new) == rec["start_sha256"], (ver, rec["epoch"])
            if ver == 2:    # V2's first two pools come from the previous start_num (V2:135-138)
                assert sha256_i64(old // ns) == rec["prev_blocks_sha256"], rec["epoch"]
        eng.close()


@pytest.mark.parametrize("name", STREAMS)
def test_cpu_mode_exact_order_is_reference_stream(name):
    fx = load_big(name)
    lens = big_lengths(fx)
    N = int(lens.sum())
    eng = pss.IndexEngine(lens, N, fx["R"], fx["B"], fx["version"], device="cpu", order="exact")
    count = fx["prefix"] if fx["kind"] == "prefix" else None
    for r, er in _walk(fx, eng):
        got = eng.generate(r, r + 1, 0, count).numpy()[0]
        check_stream(got, er, fx, "%s r%d e%d" % (name, r, er["epoch"]))
    eng.close()


@pytest.mark.parametrize("name", big_names("stream"))
def test_cpu_mode_counter_order_has_reference_multiset(name):
    fx = load_big(name)
    lens = big_lengths(fx)
    N = int(lens.sum())
    eng = pss.IndexEngine(lens, N, fx["R"], fx["B"], fx["version"], device="cpu")
    for r, er in _walk(fx, eng):
        check_multiset(eng.generate(r, r + 1).numpy()[0], er, "%s r%d e%d" % (name, r, er["epoch"]))
    eng.close()


def test_partition_oracle_reads_what_the_reference_streams_read():
    """oracle.partition_segments (the checker of pss_partition) against the reference itself:
    for every rank-epoch of the Zipf fixtures (whole reference streams, both versions), the
    segments' per-file lengths == the per-file counts of the reference stream mapped through the
    reference's own file order (RefHistory, pinned above) and V1:181-221's map."""
    for name in ("zipf_v1", "zipf_v2"):
        fx = load_big(name)
        lens = big_lengths(fx)
        N, R, B = int(lens.sum()), fx["R"], fx["B"]
        ns = O.num_samples(N, R)
        full = load_big_streams(name)
        for rr in fx["ranks"]:
            h = O.RefHistory(fx["version"], len(lens), R, rr["rank"], N)
            for er in rr["epochs"]:
                h.init_iter(er["epoch"])
                prefix = np.concatenate([[0], np.cumsum(lens[h.order])]).astype(np.int64)
                f, _ = O.map_ids(prefix, full["r%d_e%d" % (rr["rank"], er["epoch"])])
                sf, sl, sh = O.partition_segments(fx["version"], prefix, h.old_start, h.start, ns, B, N)
                seg = np.zeros(len(lens), dtype=np.int64)
                np.add.at(seg, sf, sh - sl)
                assert np.array_equal(np.bincount(f, minlength=len(lens)), seg), (name, rr["rank"])


@pytest.mark.parametrize("version", [2, 1])
def test_cpu_mode_partition_at_c4_matches_oracle(version):
    """pss_partition (CPU mode) of all 4096 ranks at C4 (Zipf, N > 2^31) == the oracle's
    segments, over the reference-pinned file order (assign_c4)."""
    import workloads as W
    lengths, N, R, B, _ = W.shape("c4")
    fx = load_big("assign_c4")
    eng = pss.IndexEngine(lengths, N, R, B, version, device="cpu")
    ns = eng.num_samples
    rec = fx["versions"]["v%d" % version][1]
    eng.init_iter(0)
    eng.init_iter(rec["epoch"])
    order = eng.file_order()
    assert sha256_i64(order.astype(np.int64)) == rec["order_sha256"]
    prefix = np.concatenate([[0], np.cumsum(lengths[order])]).astype(np.int64)
    old, new = eng.rank_starts()
    seg_off, sf, sl, sh = eng.partition(0, R)
    for r in range(R):
        a, b = int(seg_off[r]), int(seg_off[r + 1])
        wf, wl, wh = O.partition_segments(version, prefix, int(old[r]), int(new[r]), ns, B, N)
        assert np.array_equal(sf[a:b], wf) and np.array_equal(sl[a:b], wl) and np.array_equal(sh[a:b], wh), r
    eng.close()
