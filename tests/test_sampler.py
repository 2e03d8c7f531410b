"""End-to-end drop-in facade: the sampler classes against the reference goldens and the
oracle, through the C-ABI -- on the GPU (ids from the HIP kernels; `-m gpu`) and in the
library's CPU mode (device="cpu", the same schedule on host threads; runs without a GPU)."""
import numpy as np
import pytest

from oracle import oracle as O
from tests.golden_util import fixture_params, length_of_fn, load, scenario_names

DEVICES = [pytest.param("cpu", id="cpu"), pytest.param(0, id="gpu", marks=pytest.mark.gpu)]

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


def make(fx, rank, device, **kw):
    files, lengths, fl, N, R, B, bs, shuffle = fixture_params(fx)
    cls = (V1mod if fx["version"] == "v1" else V2mod).DistributedSamplerViaLocallyShuffle
    use_fl = fx["config"].get("files_len", True)
    return cls(Dataset(files), reader_for(lengths), num_replicas=R, rank=rank, shuffle=shuffle,
               shuffle_buffer=B, total_size=fx["config"].get("total_size", 1), batch_size=bs,
               files_len=(fl if use_fl else None), device=device, **kw)


def batches_of(it):
    # next() on the iterator: a `for` loop would call __iter__ again, which -- as in the
    # reference -- runs one more (cumulative) init_iter
    out = []
    while True:
        try:
            out.append(next(it))
        except StopIteration:
            return out


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("name", scenario_names("v1") + scenario_names("v2"))
def test_sampler_matches_reference_semantics(name, device):
    fx = load(name)
    files, lengths, fl, N, R, B, bs, shuffle = fixture_params(fx)
    length_of = length_of_fn(lengths, fl)
    for rrec in fx["ranks"]:
        s = make(fx, rrec["rank"], device)
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


@pytest.mark.parametrize("device", DEVICES)
def test_sampler_errors_match_reference(device):
    fx = load("v1_small")
    files, lengths, fl, N, R, B, bs, shuffle = fixture_params(fx)
    C1 = V1mod.DistributedSamplerViaLocallyShuffle
    C2 = V2mod.DistributedSamplerViaLocallyShuffle
    with pytest.raises(AssertionError):
        C1(Dataset(files), reader_for(lengths), num_replicas=2, rank=0, shuffle_buffer=4)
    with pytest.raises(TypeError):
        C1(Dataset(files), reader_for(lengths), num_replicas=2, rank=0, total_size=10)
    s2 = C2(Dataset(files), reader_for(lengths), num_replicas=2, rank=0, total_size=10,
            device=device)
    with pytest.raises(TypeError):
        iter(s2)


@pytest.mark.parametrize("device", DEVICES)
def test_resume_is_exact_skip_ahead(device):
    rng = np.random.default_rng(4)
    lens = rng.integers(50, 400, 40)
    files = ["f%02d" % i for i in range(40)]
    lengths = dict(zip(files, lens.tolist()))
    for mod in (V1mod, V2mod):
        kw = dict(num_replicas=3, rank=1, shuffle_buffer=64, total_size=1, batch_size=32,
                  files_len=lengths, device=device)
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


@pytest.mark.parametrize("device", DEVICES)
def test_device_handoff_and_multiset(device):
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
                                                        total_size=1, batch_size=256, files_len=lengths,
                                                        device=device)
            s.set_epoch(2)
            iter(s)
            ids, fpos, off = s.device_indices()
            assert ids.is_cuda == (device != "cpu") and ids.numel() == len(s)
            allids.append(ids.cpu().numpy())
        allids = np.sort(np.concatenate(allids))
        pad = len(s) * R - N
        assert np.array_equal(allids, np.sort(np.concatenate([np.arange(N), np.arange(pad)])))


@pytest.mark.parametrize("device", DEVICES)
def test_rank_block_matches_single_ranks(device):
    """ranks=(lo, hi): one process generates a block of logical ranks in one launch; its rows
    equal the ranks' own streams, and iteration serves `rank`'s batches."""
    rng = np.random.default_rng(12)
    lens = rng.integers(200, 900, 60)
    files = ["f%02d" % i for i in range(60)]
    lengths = dict(zip(files, lens.tolist()))
    R = 8
    for mod in (V1mod, V2mod):
        kw = dict(num_replicas=R, shuffle_buffer=256, total_size=1, batch_size=128,
                  files_len=lengths, device=device)
        blk = mod.DistributedSamplerViaLocallyShuffle(Dataset(files), reader_for(lengths), rank=5,
                                                      ranks=(4, 8), **kw)
        blk.set_epoch(3)
        got = [b[2] for b in blk]
        rows = blk.block_indices().cpu().numpy()
        assert rows.shape == (4, len(blk))
        for r in range(4, 8):
            one = mod.DistributedSamplerViaLocallyShuffle(Dataset(files), reader_for(lengths), rank=r, **kw)
            one.set_epoch(3)
            it = iter(one)
            assert np.array_equal(one.indices(), rows[r - 4])
            if r == 5:
                assert [b[2] for b in batches_of(it)] == got
        with pytest.raises(ValueError):
            mod.DistributedSamplerViaLocallyShuffle(Dataset(files), reader_for(lengths), rank=3,
                                                    ranks=(4, 8), **kw)


@pytest.mark.parametrize("device", DEVICES)
def test_files_view_is_lazy_and_exact(device):
    """self.files is a view over the engine's file order (no per-epoch list rebuild) that
    compares, indexes and slices like the reference's list (V1:122-125)."""
    fx = load("v2_small")
    s = make(fx, 0, device)
    er = fx["ranks"][0]["epochs"][0]
    s.set_epoch(er["epoch"])
    iter(s)
    assert type(s.files).__name__ == "_FileOrder"
    assert s.files == er["files"] and list(s.files) == er["files"]
    assert s.files[3] == er["files"][3] and s.files[2:5] == er["files"][2:5]
    assert len(s.files) == len(er["files"])


def _probe_fixture(ver):
    import json
    import os
    from tests.golden_util import GOLDEN
    with open(os.path.join(GOLDEN, "probes_%s.json" % ver)) as f:
        return json.load(f)


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("order", ["counter", "exact"])
@pytest.mark.parametrize("ver", ["v1", "v2"])
def test_lazy_length_probes_follow_reference_scan(ver, order, device):
    """files missing from files_len are probed with reader(path, get_data=False) in shuffled
    scan order, restarting every epoch (V1:182-190): the probe calls equal the reference's own
    (tests/golden/probes_*.json, tools/gen_golden_probes.py); in exact order the batches' file
    groups are the reference's too."""
    fx = _probe_fixture(ver)
    mod = V1mod if ver == "v1" else V2mod
    for sc in fx["scenarios"]:
        cfg = sc["config"]
        calls = []
        base = reader_for(cfg["lengths"])

        def reader(path, get_data=False):
            if not get_data:
                calls.append(path)
            return base(path, get_data)
        for rrec in sc["ranks"]:
            s = mod.DistributedSamplerViaLocallyShuffle(
                Dataset(cfg["files"]), reader, num_replicas=cfg["R"], rank=rrec["rank"],
                shuffle_buffer=cfg["B"], total_size=cfg["total_size"], batch_size=cfg["bs"],
                files_len=cfg["files_len_dict"], device=device, order=order)
            for er in rrec["epochs"]:
                s.set_epoch(er["epoch"])
                it = iter(s)
                del calls[:]
                got = [b[2] for b in batches_of(it)]
                assert calls == er["probes"], (sc["name"], rrec["rank"], er["epoch"])
                if order == "exact":
                    assert got == er["read_files"], (sc["name"], rrec["rank"], er["epoch"])


@pytest.mark.gpu
def test_device_error_flag_reaches_the_sampler():
    """A kernel that flags the device error word (here: the partition kernel given too little
    segment capacity) makes the drop-in raise at the next batch instead of serving ids from an
    incomplete epoch (pss_error_snapshot), and pss_check reports it by code."""
    import ctypes
    import torch
    from partiallyshuffledistributedsampler_amd import _lib
    fx = load("v2_small")
    s = make(fx, 0, 0)
    s.set_epoch(0)
    it = iter(s)
    next(it)
    eng = s._engine
    seg_off = torch.zeros(eng.num_replicas + 1, dtype=torch.int64, device="cuda")
    one = torch.zeros(1, dtype=torch.int64, device="cuda")
    one32 = torch.zeros(1, dtype=torch.int32, device="cuda")
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    _lib.call("pss_partition", eng._h, 0, eng.num_replicas, ctypes.c_void_p(seg_off.data_ptr()),
              ctypes.c_void_p(one32.data_ptr()), ctypes.c_void_p(one.data_ptr()),
              ctypes.c_void_p(one.data_ptr()), 1, stream)      # capacity 1: the flag is set
    s.set_epoch(1)
    it = iter(s)
    with pytest.raises(RuntimeError, match="device error"):
        next(it)
    with pytest.raises(_lib.PSSError):
        eng.check()
    eng.check()                                   # pss_check cleared the word


@pytest.mark.parametrize("device", DEVICES)
def test_fused_mapping_and_device_gather(device):
    """pss_generate_mapped (V1: fused into the generation kernel; V2: generate + bucket map)
    equals generate + map, and pss_gather returns the rows the host reader would gather
    (V1:243-248), for the rank's whole epoch."""
    import torch
    from partiallyshuffledistributedsampler_amd.engine import IndexEngine
    rng = np.random.default_rng(31)
    lens = rng.integers(0, 700, 90)           # empty files included
    N, R = int(lens.sum()), 5
    dev = torch.device("cpu") if device == "cpu" else torch.device("cuda", 0)
    for ver, B in ((1, 256), (2, 256), (2, 20000), (1, 70000)):
        eng = IndexEngine(lens, N, R, B, ver, seed=4, device=device)
        eng.init_iter(3)
        ids = eng.generate(0, R)
        fpos, off = eng.map(ids.reshape(-1))
        f2, o2 = eng.generate_mapped(1, R, 7, 1000)
        ns = eng.num_samples
        c = min(1000, ns - 7)
        want_f = fpos.reshape(R, -1)[1:, 7:7 + c]
        want_o = off.reshape(R, -1)[1:, 7:7 + c]
        assert torch.equal(f2[:, :c].cpu(), want_f.cpu()) and torch.equal(o2[:, :c].long().cpu(), want_o.cpu())
        # device-resident rows: file f's sample j is the row (f, j); files stored in dataset order
        base = np.concatenate([[0], np.cumsum(lens)[:-1]])
        data = torch.stack([torch.from_numpy(np.repeat(np.arange(len(lens)), lens)),
                            torch.from_numpy(np.concatenate([np.arange(n) for n in lens]))], 1).to(dev)
        rows = eng.gather(data, torch.from_numpy(base), fpos, off)
        order = eng.file_order()
        fp = fpos.cpu().numpy()
        f_abs = np.where(fp < 0, -1 - fp, fp)
        assert np.array_equal(rows[:, 0].cpu().numpy(), order[f_abs])
        assert np.array_equal(rows[:, 1].cpu().numpy(), off.cpu().numpy())
        eng.close()
    # through the sampler: batches gathered on the device == the host reader's batches
    fx = load("v2_small")
    files, lengths, fl, N, R, B, bs, shuffle = fixture_params(fx)
    s = make(fx, 0, device)
    s.set_epoch(0)
    host = batches_of(iter(s))
    s = make(fx, 0, device)            # a fresh sampler: init_iter's history is cumulative
    s.set_epoch(0)
    iter(s)
    lens2 = np.array([lengths[p] for p in files])
    base2 = torch.from_numpy(np.concatenate([[0], np.cumsum(lens2)[:-1]]))
    data2 = torch.from_numpy(np.concatenate([np.arange(n) for n in lens2])).to(dev)
    dev_batches = list(s.device_batches(data2, base2))
    assert len(dev_batches) >= len(host)
    for (tg, _, rf), (rows, f, o) in zip(host, dev_batches):
        assert sorted(np.concatenate([d["off"] for d in tg]).tolist()) == sorted(rows.cpu().tolist())


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("order", ["counter", "exact"])
def test_state_dict_resume_continues_the_same_stream(device, order):
    """state_dict() after some batches of the third epoch (init_iter history 0, 1, 1): a fresh
    sampler's load_state_dict() replays the history, so file order, blocks and the remaining
    batches equal the uninterrupted run's; a different schedule version or seed is refused."""
    rng = np.random.default_rng(8)
    lens = rng.integers(50, 400, 40)
    files = ["f%02d" % i for i in range(40)]
    lengths = dict(zip(files, lens.tolist()))
    for mod in (V1mod, V2mod):
        kw = dict(num_replicas=3, rank=2, shuffle_buffer=64, total_size=1, batch_size=32,
                  files_len=lengths, device=device, order=order)
        a = mod.DistributedSamplerViaLocallyShuffle(Dataset(files), reader_for(lengths), **kw)
        for e in (0, 1):
            a.set_epoch(e)
            batches_of(iter(a))
        it = iter(a)                       # epoch 1 again: a third, cumulative init_iter
        head = [next(it) for _ in range(5)]
        sd = a.state_dict()
        tail = [b[2] for b in batches_of(it)]
        assert sd["history"] == [0, 1, 1] and sd["position"] == 5 * 32 and head
        b = mod.DistributedSamplerViaLocallyShuffle(Dataset(files), reader_for(lengths), **kw)
        b.load_state_dict(sd)
        it2 = iter(b)                      # warm start
        assert b.files == a.files and b.blocks == a.blocks and b.start_num == a.start_num
        assert [x[2] for x in batches_of(it2)] == tail
        assert np.array_equal(b.indices(), a.indices())
        if order == "counter":
            bad = dict(sd, schedule_version=sd["schedule_version"] - 1)
            c = mod.DistributedSamplerViaLocallyShuffle(Dataset(files), reader_for(lengths), **kw)
            with pytest.raises(ValueError):
                c.load_state_dict(bad)
            with pytest.raises(ValueError):
                c.load_state_dict(dict(sd, seed=sd["seed"] + 1))
        c = mod.DistributedSamplerViaLocallyShuffle(Dataset(files), reader_for(lengths), **kw)
        with pytest.raises(ValueError):    # another file count
            c.load_state_dict(dict(sd, num_files=sd["num_files"] + 1))
        if mod is V1mod:                   # V1 with shuffle=False is another permutation
            with pytest.raises(ValueError):
                c.load_state_dict(dict(sd, shuffle=False))
            c = mod.DistributedSamplerViaLocallyShuffle(Dataset(files), reader_for(lengths),
                                                        **dict(kw, shuffle=False))
            with pytest.raises(ValueError):
                c.load_state_dict(sd)
        # a state of a round-4 build (no 'shuffle' / 'num_files', same schedule version) resumes
        old = {k: v for k, v in sd.items() if k not in ("shuffle", "num_files")}
        d = mod.DistributedSamplerViaLocallyShuffle(Dataset(files), reader_for(lengths), **kw)
        d.load_state_dict(old)
        assert [x[2] for x in batches_of(iter(d))] == tail


@pytest.mark.parametrize("device", DEVICES)
def test_lookahead_bounds_and_workspace_bytes(device):
    """lookahead=(exact_depth, exact_max_bytes, v2_depth) reaches pss_set_lookahead and changes
    nothing in the stream; workspace_bytes() reports the engine's device bytes (0 in CPU mode
    and before the first epoch)."""
    fx = load(scenario_names("v2")[0])
    s_ref = make(fx, 0, device)
    s_cap = make(fx, 0, device, lookahead=(0, 1 << 20, 0))
    assert s_cap.workspace_bytes() == 0
    for e in range(3):
        streams = []
        for s in (s_ref, s_cap):
            s.set_epoch(e)
            batches_of(iter(s))
            streams.append(s.indices())
        assert np.array_equal(streams[0], streams[1])
    if device == "cpu":
        assert s_cap.workspace_bytes() == 0
    else:
        assert s_cap.workspace_bytes() > 0
