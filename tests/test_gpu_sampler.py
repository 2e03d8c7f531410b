"""End-to-end drop-in facade on the GPU: the sampler classes against the reference goldens
and the oracle, through the C-ABI (ids from the HIP kernels, host assembly on top)."""
import numpy as np
import pytest

from oracle import oracle as O
from tests.golden_util import fixture_params, length_of_fn, load, scenario_names

pytestmark = pytest.mark.gpu

V1mod = pytest.importorskip("partiallyshuffledistributedsampler_amd.DistributedSamplerViaLocallyShuffle")
V2mod = pytest.importorskip("partiallyshuffledistributedsampler_amd.DistributedSamplerViaLocallyShuffleV2")


class Dataset:
    def __init__(self, files):
        self.files = list(files)
        self.resets = 0

    def reset(self):
        self.resets += 1


def reader_for(lengths):
    index = {p: i for i, p in enumerate(sorted(lengths))}

    def reader(path, get_data=False):
        n = lengths[path]
        if not get_data:
            return n
        return {"fid": np.full(n, index[path], dtype=np.int64),
                "off": np.arange(n, dtype=np.int64)}, n
    return reader


def make(fx, rank, **kw):
    files, lengths, fl, N, R, B, bs, shuffle = fixture_params(fx)
    cls = (V1mod if fx["version"] == "v1" else V2mod).DistributedSamplerViaLocallyShuffle
    use_fl = fx["config"].get("files_len", True)
    return cls(Dataset(files), reader_for(lengths), num_replicas=R, rank=rank, shuffle=shuffle,
               shuffle_buffer=B, total_size=fx["config"].get("total_size", 1), batch_size=bs,
               files_len=(fl if use_fl else None), **kw)


def batches_of(it):
    # next() on the iterator: a `for` loop would call __iter__ again, which -- as in the
    # reference -- runs one more (cumulative) init_iter
    out = []
    while True:
        try:
            out.append(next(it))
        except StopIteration:
            return out


@pytest.mark.parametrize("name", scenario_names("v1") + scenario_names("v2"))
def test_sampler_matches_reference_semantics(name):
    fx = load(name)
    files, lengths, fl, N, R, B, bs, shuffle = fixture_params(fx)
    length_of = length_of_fn(lengths, fl)
    for rrec in fx["ranks"]:
        s = make(fx, rrec["rank"])
        assert len(s) == rrec["len"]
        for er in rrec["epochs"]:
            if er.get("resume_step") is not None:
                s.set_epoch(er["epoch"])
                s.find_ckpt_position(er["resume_step"])
            else:
                s.set_epoch(er["epoch"])
            it = iter(s)
            assert s.files == er["files"] and s.blocks == er["blocks"]
            assert s.start_num == er["start_num"]
            got = batches_of(it)
            stream = s.indices()
            if er.get("resume_step") is not None:
                stream = stream[er["resume_step"] * bs:]
            # grouping/mapping semantics of the reference applied to our own stream
            ref = list(O.ref_batches(stream, bs, er["files"], length_of))
            assert len(got) == len(ref)
            for (tg, none, rf), (rrf, roffs) in zip(got, ref):
                assert rf == rrf and [d["off"].tolist() for d in tg] == roffs
            if fx["version"] == "v1" and not shuffle:
                # identity order: the batches must be the reference's, bit for bit
                assert len(got) == er["num_batches"]
                for (tg, _, rf), r in zip(got, er["outputs"]):
                    assert rf == r["read_files"] and [d["off"].tolist() for d in tg] == r["off"]


def test_sampler_errors_match_reference():
    fx = load("v1_small")
    files, lengths, fl, N, R, B, bs, shuffle = fixture_params(fx)
    C1 = V1mod.DistributedSamplerViaLocallyShuffle
    C2 = V2mod.DistributedSamplerViaLocallyShuffle
    with pytest.raises(AssertionError):
        C1(Dataset(files), reader_for(lengths), num_replicas=2, rank=0, shuffle_buffer=4)
    with pytest.raises(TypeError):
        C1(Dataset(files), reader_for(lengths), num_replicas=2, rank=0, total_size=10)
    s2 = C2(Dataset(files), reader_for(lengths), num_replicas=2, rank=0, total_size=10)
    with pytest.raises(TypeError):
        iter(s2)


def test_resume_is_exact_skip_ahead():
    rng = np.random.default_rng(4)
    lens = rng.integers(50, 400, 40)
    files = ["f%02d" % i for i in range(40)]
    lengths = dict(zip(files, lens.tolist()))
    for mod in (V1mod, V2mod):
        kw = dict(num_replicas=3, rank=1, shuffle_buffer=64, total_size=1, batch_size=32,
                  files_len=lengths)
        a = mod.DistributedSamplerViaLocallyShuffle(Dataset(files), reader_for(lengths), **kw)
        a.set_epoch(5)
        full = [b[2] for b in a]          # `for` = one __iter__ = one init_iter
        ids_full = a.indices()
        b = mod.DistributedSamplerViaLocallyShuffle(Dataset(files), reader_for(lengths), **kw)
        b.set_epoch(5)
        b.find_ckpt_position(7)
        rest = [x[2] for x in b]          # warm start: __iter__ skips init_iter
        assert rest == full[7:]
        assert np.array_equal(b.indices(), ids_full)


def test_device_handoff_and_multiset():
    rng = np.random.default_rng(9)
    lens = rng.integers(1000, 5000, 100)
    files = ["f%03d" % i for i in range(100)]
    lengths = dict(zip(files, lens.tolist()))
    N = int(lens.sum())
    R = 4
    for mod, ver in ((V1mod, 1), (V2mod, 2)):
        allids = []
        for r in range(R):
            s = mod.DistributedSamplerViaLocallyShuffle(Dataset(files), reader_for(lengths),
                                                        num_replicas=R, rank=r, shuffle_buffer=4096,
                                                        total_size=1, batch_size=256, files_len=lengths)
            s.set_epoch(2)
            iter(s)
            ids, fpos, off = s.device_indices()
            assert ids.is_cuda and ids.numel() == len(s)
            allids.append(ids.cpu().numpy())
        allids = np.sort(np.concatenate(allids))
        pad = len(s) * R - N
        assert np.array_equal(allids, np.sort(np.concatenate([np.arange(N), np.arange(pad)])))
