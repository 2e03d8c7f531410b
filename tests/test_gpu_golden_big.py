"""Bench-scale reference goldens on the GPU, through the C-ABI (tests/golden/big, captured from
the reference itself by tools/gen_golden_big.py; the CPU side is tests/test_golden_big.py).

  * order="exact": each recorded rank-epoch stream is reproduced bit for bit (whole-stream
    sha256) -- V1 at B = 4096 and at C5's B = 2^20 (windows far beyond LDS, 12 per rank), V2 at
    B = 400 / 4096 / 65536 (pool2 refills, the per-step reseeding tail, two-word MT seeds) and
    the first 20480 draws of C5's B = 2^20 pools (V1:157-172, V2:96-116);
  * the default counter order: every rank-epoch has the reference's id multiset (sorted-stream
    sha256), over the same cumulative init_iter history;
  * the mapped hand-off (pss_generate_mapped) equals generate + map on the exact streams.
"""
import numpy as np
import pytest
import torch

from tests.golden_util import big_lengths, big_names, check_multiset, check_stream, load_big

pytestmark = pytest.mark.gpu

pss = pytest.importorskip("partiallyshuffledistributedsampler_amd.engine")

STREAMS = big_names("stream") + big_names("prefix")


def _walk(fx, eng):
    ranks = fx["ranks"]
    for i, er0 in enumerate(ranks[0]["epochs"]):
        eng.init_iter(er0["epoch"])
        old, new = eng.rank_starts()
        for rr in ranks:
            er = rr["epochs"][i]
            r = rr["rank"]
            assert (int(old[r]), int(new[r])) == (er["old_start"], er["start_num"]), (r, er["epoch"])
            yield r, er


def _engine(fx, order):
    lens = big_lengths(fx)
    return pss.IndexEngine(lens, int(lens.sum()), fx["R"], fx["B"], fx["version"], device=0,
                           order=order)


@pytest.mark.parametrize("name", STREAMS)
def test_gpu_exact_order_is_reference_stream(name):
    fx = load_big(name)
    eng = _engine(fx, "exact")
    count = fx["prefix"] if fx["kind"] == "prefix" else None
    for r, er in _walk(fx, eng):
        got = eng.generate(r, r + 1, 0, count)
        eng.check()
        check_stream(got.cpu().numpy()[0], er, fx, "%s r%d e%d" % (name, r, er["epoch"]))
    eng.close()


@pytest.mark.parametrize("name", big_names("stream"))
def test_gpu_counter_order_has_reference_multiset(name):
    fx = load_big(name)
    eng = _engine(fx, "counter")
    for r, er in _walk(fx, eng):
        got = eng.generate(r, r + 1)
        eng.check()
        check_multiset(got.cpu().numpy()[0], er, "%s r%d e%d" % (name, r, er["epoch"]))
    eng.close()


@pytest.mark.parametrize("name", ["c1_v1", "c1_v2", "zipf_v2", "v2_b65536_r0_e5", "v1_c5_r0"])
def test_gpu_exact_order_mapped_hand_off(name):
    """(file, offset) of the exact streams: pss_generate_mapped == pss_generate + pss_map, for
    all recorded ranks at once and for a ragged position range.  v1_c5_r0: V1 windows of 2^20
    entries, beyond LDS -- the HBM path's k_v1x_out maps each id where it writes it."""
    fx = load_big(name)
    eng = _engine(fx, "exact")
    for r, er in _walk(fx, eng):
        f, o = eng.generate_mapped(r, r + 1)
        eng.check()
        ids = eng.generate(r, r + 1)
        check_stream(ids.cpu().numpy()[0], er, fx, name)
        fr, orr = eng.map(ids.view(-1))
        assert torch.equal(f.view(-1), fr) and torch.equal(o.view(-1).long(), orr), (name, r)
        n = eng.num_samples
        lo, cnt = n // 3 + 7, n // 2
        f2, o2 = eng.generate_mapped(r, r + 1, lo, cnt)
        assert torch.equal(f2.view(-1), fr[lo:lo + cnt]) and torch.equal(o2.view(-1).long(), orr[lo:lo + cnt])
    eng.close()
