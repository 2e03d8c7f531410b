"""Pin the CPU oracle against the reference's own outputs (tests/golden, tools/gen_golden.py).

This is what makes the oracle trustworthy: every function the GPU parity tests rely on is
checked here against vectors recorded from the reference sampler itself.
"""
import numpy as np
import pytest

from oracle import oracle as O
from tests.golden_util import fixture_params, length_of_fn, load, scenario_names


def test_mt_genrand_kats():
    kats = load("mt_kats")
    for rec in kats["genrand"]:
        mt = O.MT(rec["seed"])
        got = [mt.u32() for _ in range(len(rec["u32"]))]
        assert got == rec["u32"], rec["seed"]


def test_mt_shuffle_kats():
    for rec in load("mt_kats")["shuffle"]:
        got = O.seeded_shuffle(rec["seed"], rec["n"]).tolist()
        assert got == rec["perm"], (rec["seed"], rec["n"])
        mt = O.MT(rec["seed"])
        assert mt.shuffle(np.arange(rec["n"])).tolist() == rec["perm"]


def test_mt_randbelow_and_choice_kats():
    k = load("mt_kats")
    mt = O.MT(k["randbelow"]["seed"])
    assert [mt.randbelow(n) for n in k["randbelow"]["n"]] == k["randbelow"]["r"]
    mt = O.MT(k["choice"]["seed"])
    # choice(seq) == seq[_randbelow(len(seq))] (random.py:375-378); seq = range(n) here
    assert [mt.randbelow(n) for n in k["choice"]["n"]] == k["choice"]["r"]


def test_num_samples_float_ceil():
    assert O.num_samples(559, 3) == 187
    assert O.num_samples(2_594_705_250, 4096) == 633_473
    assert O.num_samples(1_000_000_000, 1024) == 976_563
    # above 2**53 the reference's float ceil differs from integer ceil; keep the float one
    big = 2 ** 53 + 1
    assert O.num_samples(big, 1) == 2 ** 53


ALL = [("v1", n) for n in scenario_names("v1")] + [("v2", n) for n in scenario_names("v2")]


@pytest.mark.parametrize("ver,name", ALL)
def test_history_and_exact_streams(ver, name):
    fx = load(name)
    files, lengths, fl, N, R, B, bs, shuffle = fixture_params(fx)
    version = 1 if ver == "v1" else 2
    for rrec in fx["ranks"]:
        rank = rrec["rank"]
        h = O.RefHistory(version, len(files), R, rank, N, shuffle)
        assert rrec["num_samples"] == h.ns and rrec["len"] == h.ns
        assert rrec["ori_total_size"] == N
        for er in rrec["epochs"]:
            ep = er["epoch"]
            assert er["old_start"] == h.start
            h.init_iter(ep)
            assert [files[i] for i in h.order] == er["files"], (name, rank, ep)
            assert h.blocks.tolist() == er["blocks"]
            assert h.start == er["start_num"]
            stream = [x for b in er["batches"] for x in b]
            resume = er.get("resume_step")
            if version == 1:
                pos = resume * bs if resume is not None else -1
                got = O.v1_exact_stream(ep, h.start, h.ns, B, N, shuffle, pos)
            else:
                skip = resume * bs if resume is not None else 0
                got = O.v2_exact_stream(ep, h.old_start, h.start, h.ns, B, N, skip)
                # the rank-select restatement (the checker of big pools) reproduces it too
                got_rs = O.v2_exact_stream_rs(ep, h.old_start, h.start, h.ns, B, N, skip)
                assert np.array_equal(got_rs, got), (name, rank, ep)
            # the recorded stream stops early only via the tmp_count == 1 quirk
            assert got[:len(stream)].tolist() == stream, (name, rank, ep)
            if er["num_batches"] * bs < len(got):
                # stopped early: the last recorded batch mapped exactly one id
                assert len(er["batches"][-1]) >= 1


@pytest.mark.parametrize("ver,name", ALL)
def test_batch_grouping_semantics(ver, name):
    fx = load(name)
    files, lengths, fl, N, R, B, bs, shuffle = fixture_params(fx)
    length_of = length_of_fn(lengths, fl)
    fidx = {p: i for i, p in enumerate(sorted(lengths))}
    for rrec in fx["ranks"]:
        for er in rrec["epochs"]:
            stream = [x for b in er["batches"] for x in b]
            got = list(O.ref_batches(stream, bs, er["files"], length_of))
            assert len(got) == er["num_batches"], (name, rrec["rank"], er["epoch"])
            for (rf, offs), ref in zip(got, er["outputs"]):
                assert rf == ref["read_files"]
                assert offs == ref["off"]
                assert [[fidx[p]] * len(o) for p, o in zip(rf, offs)] == ref["fid"]


def test_v1_multiset_is_rank_block():
    # V1 per-rank epoch multiset = {start + v : v < ns} mod N  (V1:161-163)
    for N, R, B in ((559, 3, 16), (1000, 7, 33), (97, 4, 200)):
        ns = O.num_samples(N, R)
        for start in (0, ns, ns * (R - 1)):
            s = O.v1_exact_stream(3, start, ns, B, N)
            ref = (start + np.arange(ns)) % N
            assert np.array_equal(np.sort(s), np.sort(ref))


def test_v2_multiset_old_new_split():
    # V2 per-rank multiset = [old, old+min(2B,ns)) U [new+2B, new+ns) mod N (V2:135-138,110-112)
    for N, R, B in ((559, 3, 16), (1000, 7, 33), (97, 4, 200), (5000, 2, 300)):
        ns = O.num_samples(N, R)
        for old, new in ((0, ns), (ns * (R - 1), 0), (ns, ns)):
            s = O.v2_exact_stream(5, old, new, ns, B, N)
            v = np.arange(ns)
            ref = np.where(v < 2 * B, old + v, new + v) % N
            assert len(s) == ns
            assert np.array_equal(np.sort(s), np.sort(ref))


def test_pyref_loops_reproduce_reference_streams():
    """oracle/pyref.py (bench.py's cpu_baseline restatement of the reference loops) draws the
    reference's own id streams (tests/golden raw batches, captured at V1:178 / V2:181)."""
    import numpy as np
    from oracle.pyref import V1Loop, V2Draws, V2Loop
    for name in ("v1_small", "v1_c1_small", "v1_zipf"):
        fx = load(name)
        files, lengths, fl, N, R, B, bs, shuffle = fixture_params(fx)
        rrec = fx["ranks"][0]
        ns = rrec["num_samples"]
        for er in rrec["epochs"]:
            if er.get("resume_step") is not None:
                continue
            lens = [fl.get(p, lengths[p]) for p in er["files"]]
            loop = V1Loop(er["start_num"], ns, B, N, lens,
                          lambda f: {"x": np.arange(lens[f])}, epoch=er["epoch"], bs=bs, use_gc=False)
            got = []
            while loop.next_batch() is not None:
                got.append(loop.last_indices)
            assert got[:len(er["batches"])] == er["batches"], (name, er["epoch"])
    for name in ("v2_small", "v2_zipf"):
        fx = load(name)
        files, lengths, fl, N, R, B, bs, shuffle = fixture_params(fx)
        for rrec in fx["ranks"]:
            ns = rrec["num_samples"]
            er = rrec["epochs"][0]
            d = V2Draws(er["old_start"], er["start_num"], ns, B, epoch=er["epoch"])
            want = [x for b in er["batches"] for x in b]
            got = [d.get_index() for _ in range(len(want))]
            got = [x - N if x >= N else x for x in got]
            assert got == want, (name, rrec["rank"])
            # the whole __next__ loop (draws + map + gather) on the same rank
            lens = [fl.get(p, lengths[p]) for p in er["files"]]
            loop = V2Loop(er["old_start"], er["start_num"], ns, B, N, lens,
                          lambda f: {"x": np.arange(lens[f])}, epoch=er["epoch"], bs=bs,
                          use_gc=False)
            got = []
            while loop.next_batch() is not None:
                got.append(loop.last_indices)
            assert got[:len(er["batches"])] == er["batches"], (name, rrec["rank"])
    # bench-scale fixture (tests/golden/big): whole rank streams at B = 4096 / 400
    from tests.golden_util import big_lengths, check_stream, load_big
    for name in ("c1_v1", "c1_v2", "zipf_v2"):
        fx = load_big(name)
        lens_ds = big_lengths(fx)
        N, B, bs = int(lens_ds.sum()), fx["B"], fx["bs"]
        rr = fx["ranks"][0]
        h = O.RefHistory(fx["version"], len(lens_ds), fx["R"], rr["rank"], N)
        er = rr["epochs"][0]
        h.init_iter(er["epoch"])
        lens = lens_ds[h.order].tolist()
        data = lambda f: {"x": np.arange(lens[f])}   # noqa: E731
        if fx["version"] == 1:
            loop = V1Loop(h.start, h.ns, B, N, lens, data, epoch=er["epoch"], bs=bs, use_gc=False)
        else:
            loop = V2Loop(h.old_start, h.start, h.ns, B, N, lens, data, epoch=er["epoch"], bs=bs,
                          use_gc=False)
        got = []
        while loop.next_batch() is not None:
            got.extend(loop.last_indices)
        check_stream(got, er, fx, name)


def _rs_cases():
    rng = np.random.default_rng(2024)
    cases = [(300, 2000, 3), (4096, 4096 * 5 + 17, 2), (1, 50, 1), (7, 7, 2), (70, 130, 4),
             (20000, 20000 * 3 + 5, 1), (5000, 4999, 2), (64, 64 * 40, 3), (3, 200, 2)]
    for _ in range(24):
        B = int(np.exp(rng.uniform(0, np.log(20000))))
        ns = int(rng.integers(1, 4 * B + 3))
        cases.append((max(B, 1), ns, int(rng.integers(1, 5))))
    return cases


@pytest.mark.parametrize("B,ns,R", _rs_cases())
def test_v2_rank_select_oracle_equals_list_remove_restatement(B, ns, R):
    """orc_v2_exact_stream_rs (rank-select bitmaps, O(log B) per draw) against the list.remove
    restatement (V2:101-106 verbatim) on random geometries up to B = 20000, including ns < B,
    ns between B and 2B, the per-step reseeding tail, epochs whose seeds need two MT key words,
    resume skips, and ranks whose blocks wrap at N."""
    N = ns * R - (R - 1) if R > 1 else ns
    rng = np.random.default_rng(B * 7919 + ns)
    for _ in range(2):
        old = ns * int(rng.integers(0, R))
        new = ns * int(rng.integers(0, R))
        epoch = int(rng.choice([0, 3, 2 ** 32 - 5, 10 ** 10]))
        skip = int(rng.integers(0, ns)) if rng.random() < 0.3 else 0
        a = O.v2_exact_stream(epoch, old, new, ns, B, N, skip)
        b = O.v2_exact_stream_rs(epoch, old, new, ns, B, N, skip)
        assert len(a) == ns - skip
        assert np.array_equal(a, b), (B, ns, R, old, new, epoch, skip)
