"""The product's CPU mode (IndexEngine(device="cpu") -> libpss PSS_DEVICE_CPU handles) against
the independent oracle: the counter schedule's twin and the reference's exact order.  The
GPU == CPU-mode comparison is in test_gpu_parity.py; BASELINE configs[0] (C1) runs end to end
here without a GPU."""
import numpy as np
import pytest

from oracle import oracle as O
import workloads as W
from partiallyshuffledistributedsampler_amd import _lib
from partiallyshuffledistributedsampler_amd.engine import IndexEngine, as_u64, digest, digest_range

CONFIGS = [
    # (F, len lo/hi, R, B)
    (64, (100, 300), 2, 64),
    (37, (1, 900), 7, 40),
    (200, (50, 2000), 4, 4096),
    (50, (1000, 5000), 3, 3000),
    (13, (1, 50), 5, 100),        # ns < B
    (9, (20, 40), 2, 70),         # B < ns < 2B
    (100, (1, 3), 8, 7),          # tiny windows
    (20, (5000, 20000), 2, 20000),      # grouped pools (P1 > 16384), non-power-of-two groups
    (12, (50000, 100000), 3, 70001),    # ... odd pool size, partial last window
    (40, (20000, 20001), 2, 65536),     # ... groups of 4096 (paired draws)
    (6, (1000, 3000), 2, 100000),       # ns < B with a big pool: tail only
]


def _twin(version, key, r, old, new, ns, B, N):
    if version == 1:
        return O.v1_philox_stream(key, r, int(new[r]), ns, B, N)
    return O.v2_philox_stream(key, r, int(old[r]), int(new[r]), ns, B, N)


@pytest.mark.parametrize("version", [1, 2])
@pytest.mark.parametrize("cfg", CONFIGS)
def test_cpu_mode_matches_oracle_twin(version, cfg):
    F, (lo, hi), R, B = cfg
    rng = np.random.default_rng(F * 1000 + R)
    lengths = rng.integers(lo, hi, F)
    N = int(lengths.sum())
    eng = IndexEngine(lengths, N, R, B, version, seed=1234, device="cpu")
    assert eng.emit_path() == "cpu"
    ns = eng.num_samples
    for epoch in (0, 3):
        eng.init_iter(epoch)
        old, new = eng.rank_starts()
        out = eng.generate(0, R).numpy()
        key = O.epoch_key(1234, epoch)
        for r in range(R):
            assert np.array_equal(out[r], _twin(version, key, r, old, new, ns, B, N)), (cfg, epoch, r)
        # position sub-ranges come out of the same streams
        for pos_lo, count in ((0, 1), (ns // 3, ns // 2), (max(ns - 5, 0), 100)):
            part = eng.generate(1 % R, R, pos_lo, count).numpy()
            c = min(count, ns - pos_lo)
            assert np.array_equal(part[:, :c], out[1 % R:, pos_lo:pos_lo + c])
    eng.close()


@pytest.mark.parametrize("version", [1, 2])
@pytest.mark.parametrize("F,lo,hi,R,B", [(37, 1, 900, 7, 40), (50, 1000, 5000, 3, 3000),
                                         (13, 1, 50, 5, 100), (9, 20, 40, 2, 70),
                                         (20, 5000, 20000, 2, 20000)])
def test_cpu_mode_exact_order_matches_exact_oracle(version, F, lo, hi, R, B):
    """order="exact" in CPU mode: the reference's CPython-MT draws, any pool size (the GPU's
    exact kernels are bounded by LDS; the CPU mode is not)."""
    rng = np.random.default_rng(F + B)
    lengths = rng.integers(lo, hi, F)
    N = int(lengths.sum())
    eng = IndexEngine(lengths, N, R, B, version, seed=7, device="cpu", order="exact")
    ns = eng.num_samples
    for epoch in (0, 2):
        eng.init_iter(epoch)
        old, new = eng.rank_starts()
        out = eng.generate(0, R).numpy()
        for r in range(R):
            ref = (O.v1_exact_stream(epoch, int(new[r]), ns, B, N, True) if version == 1 else
                   O.v2_exact_stream(epoch, int(old[r]), int(new[r]), ns, B, N))
            assert np.array_equal(out[r], ref), (F, B, epoch, r)


@pytest.mark.parametrize("B", [1 << 16, 1 << 18])
def test_cpu_mode_exact_order_big_pools_match_rank_select_oracle(B):
    """CPU mode's exact V2 (Fenwick trees) against the oracle's rank-select restatement
    (orc_v2_exact_stream_rs) on pools beyond the list.remove restatement's reach: two ranks of
    ns = 3.5 B, the last block wrapping at N."""
    R = 2
    ns = int(3.5 * B)
    N = ns * R - 1
    lengths = np.full(10, N // 10)
    lengths[-1] += N - lengths.sum()
    eng = IndexEngine(lengths, N, R, B, 2, seed=7, device="cpu", order="exact")
    eng.init_iter(4)
    old, new = eng.rank_starts()
    out = eng.generate(0, R).numpy()
    for r in range(R):
        assert np.array_equal(out[r], O.v2_exact_stream_rs(4, int(old[r]), int(new[r]), ns, B, N)), (B, r)
    eng.close()


def test_c1_runs_end_to_end_on_cpu():
    """BASELINE configs[0]: V1, 64 files x 10K, R=2, B=4096 -- every rank's epoch, exact
    coverage, through the drop-in class with device="cpu"."""
    from partiallyshuffledistributedsampler_amd.DistributedSamplerViaLocallyShuffle import \
        DistributedSamplerViaLocallyShuffle
    lengths, N, R, B, ver = W.shape("c1")
    files = ["c1_%02d.npz" % i for i in range(len(lengths))]
    fl = dict(zip(files, lengths.tolist()))

    class DS:
        def __init__(self):
            self.files = list(files)

        def reset(self):
            pass

    def reader(path, get_data=False):
        n = fl[path]
        return n if not get_data else ({"x": np.arange(n, dtype=np.int32)}, n)
    seen = []
    for r in range(R):
        s = DistributedSamplerViaLocallyShuffle(DS(), reader, num_replicas=R, rank=r,
                                                shuffle_buffer=B, total_size=N, batch_size=1024,
                                                files_len=fl, device="cpu")
        s.set_epoch(0)
        nb = 0
        for tgt, _, read_files in s:
            assert sum(len(d["x"]) for d in tgt) <= 1024
            nb += 1
        assert nb == -(-len(s) // 1024)
        seen.append(s.indices())
    allids = np.sort(np.concatenate(seen))
    assert np.array_equal(allids, np.arange(N))


def test_cpu_mode_map_partition_and_digest():
    rng = np.random.default_rng(21)
    lengths = rng.integers(0, 60, 3000)
    N, R, B = int(lengths.sum()), 6, 256
    eng = IndexEngine(lengths, N, R, B, 2, device="cpu")
    eng.init_iter(7)
    order = eng.file_order()
    prefix = np.concatenate([[0], np.cumsum(lengths[order])])
    ids = eng.generate(0, R)
    fpos, off = eng.map(ids.reshape(-1))
    rf, ro = O.map_ids(prefix, ids.numpy().reshape(-1))
    assert np.array_equal(fpos.numpy(), rf) and np.array_equal(off.numpy(), ro)
    seg_off, sf, sl, sh = eng.partition(0, R)
    for r in range(R):
        assert sum(int(sh[k] - sl[k]) for k in range(seg_off[r], seg_off[r + 1])) == eng.num_samples
    assert as_u64(digest(ids.view(-1))) == O.digest(ids.numpy().reshape(-1))
    assert as_u64(digest_range(3, 100_003, "cpu")) == O.digest_range(3, 100_003)


def test_cpu_mode_is_part_of_the_library():
    eng = IndexEngine(np.full(4, 10), 40, 2, 8, 1, device="cpu")
    d = __import__("ctypes").c_int32()
    _lib.call("pss_device", eng._h, __import__("ctypes").byref(d))
    assert d.value == _lib.PSS_DEVICE_CPU
