"""GPU parity at the BASELINE.json shapes (workloads.py), through the C-ABI.

Each configuration is checked at its real size:
  * selected ranks' full epoch streams == the oracle's counter-schedule twin, bit for bit
    (including the ranks whose blocks wrap at N, V1:161-163 / V2:113-114);
  * exact coverage over ALL logical ranks by the commutative (count, digest) check of
    SURVEY.md §8e: sum of splitmix64 over every emitted id == digest([0, N)) + digest([0, pad));
  * the device error flag is read after every generate (eng.check()).
Shapes: C2 (100M, R=8), C3 (1B, R=1024), C4 (Zipf N=2.59e9 > 2^31, R=4096: the pinned-staging
rank upload and ids above 2^31), a wide case (N + ns >= 2^32: the 64-bit id paths) and C5
(B = 2^20: pools beyond LDS) over consecutive epochs (the lookahead ring).
"""
import numpy as np
import pytest
import torch

from oracle import oracle as O
import workloads as W

pytestmark = pytest.mark.gpu

pss = pytest.importorskip("partiallyshuffledistributedsampler_amd.engine")


def _engine(lengths, N, R, B, version, seed=0):
    return pss.IndexEngine(lengths, N, R, B, version, shuffle=True, seed=seed, device=0)


def _gen(eng, lo, hi, **kw):
    out = eng.generate(lo, hi, **kw)
    eng.check()
    return out


def _twin(version, key, r, old, new, ns, B, N):
    if version == 1:
        return O.v1_philox_stream(key, r, int(new[r]), ns, B, N)
    return O.v2_philox_stream(key, r, int(old[r]), int(new[r]), ns, B, N)


def _coverage(eng, N, R, chunk):
    """(count, digest) over every logical rank, generated `chunk` ranks at a time."""
    acc = torch.zeros(1, dtype=torch.int64, device="cuda")
    count = 0
    for lo in range(0, R, chunk):
        hi = min(R, lo + chunk)
        out = _gen(eng, lo, hi)
        pss.digest(out.view(-1), acc)
        count += out.numel()
        del out
    eng.check()
    ns = eng.num_samples
    pad = ns * R - N
    want = (O.digest_range(0, N) + O.digest_range(0, pad)) & 0xFFFFFFFFFFFFFFFF
    return count == ns * R and pss.as_u64(acc) == want


def _wrapping_ranks(new, ns, N):
    return [r for r in range(len(new)) if int(new[r]) + ns > N]


@pytest.mark.parametrize("version", [2, 1])
def test_c2_all_ranks_match_twin(version):
    lengths, N, R, B, _ = W.shape("c2")
    eng = _engine(lengths, N, R, B, version, seed=0)
    ns = eng.num_samples
    for epoch in (0, 1):     # consecutive epochs: the second takes the queued lookahead pass
        eng.init_iter(epoch)
        old, new = eng.rank_starts()
        out = _gen(eng, 0, R).cpu().numpy()
        key = O.epoch_key(0, epoch)
        for r in range(R):
            assert np.array_equal(out[r], _twin(version, key, r, old, new, ns, B, N)), (epoch, r)
        assert _coverage(eng, N, R, R)                   # N = ns * R: no pad
    eng.close()


def test_c3_coverage_and_ranks_match_twin():
    lengths, N, R, B, ver = W.shape("c3")
    eng = _engine(lengths, N, R, B, ver, seed=0)
    ns = eng.num_samples
    eng.init_iter(3)
    old, new = eng.rank_starts()
    assert _coverage(eng, N, R, 256)
    key = O.epoch_key(0, 3)
    picks = sorted({0, 1, 127, 128, 511, 1023} | set(_wrapping_ranks(new, ns, N)))
    for r in picks:
        got = _gen(eng, r, r + 1).cpu().numpy()[0]
        assert np.array_equal(got, _twin(ver, key, r, old, new, ns, B, N)), r
    # one GPU's block of 128 logical ranks at 8 GPUs, against the same ranks generated alone
    blk = _gen(eng, 128, 256).cpu().numpy()
    assert np.array_equal(blk[0], _twin(ver, key, 128, old, new, ns, B, N))
    assert np.array_equal(blk[127], _gen(eng, 255, 256).cpu().numpy()[0])
    eng.close()


def test_c4_zipf_4096_ranks():
    lengths, N, R, B, ver = W.shape("c4")
    assert N == 2_594_705_250 and R > 1024      # ids above 2^31; staging upload of R > 1024
    eng = _engine(lengths, N, R, B, ver, seed=0)
    ns = eng.num_samples
    assert ns == 633_473
    for epoch in (0, 1):
        eng.init_iter(epoch)
        old, new = eng.rank_starts()
        key = O.epoch_key(0, epoch)
        wrap = _wrapping_ranks(new, ns, N) + [r for r in range(R) if int(old[r]) + 2 * B > N]
        hi_ids = [r for r in range(R) if int(new[r]) > 2 ** 31][:2]
        picks = sorted(set([0, 1, 1024, 2047, 4095] + wrap + hi_ids))
        for r in picks:
            got = _gen(eng, r, r + 1).cpu().numpy()[0]
            assert np.array_equal(got, _twin(ver, key, r, old, new, ns, B, N)), (epoch, r)
        assert int(_gen(eng, hi_ids[0], hi_ids[0] + 1).max()) > 2 ** 31
        assert _coverage(eng, N, R, 512)
    eng.close()


@pytest.mark.parametrize("version", [2, 1])
def test_wide_ids_beyond_2_32(version):
    """N + ns >= 2^32: the kernels' 64-bit id instantiations (every id of the 32-bit fast
    paths fits below 2^32 only when N + ns < 2^32)."""
    F, L, R, B = 2000, 2_200_000, 4096, 4096
    lengths = np.full(F, L, dtype=np.int64)
    N = F * L
    assert N > 2 ** 32
    eng = _engine(lengths, N, R, B, version, seed=11)
    ns = eng.num_samples
    eng.init_iter(2)
    old, new = eng.rank_starts()
    key = O.epoch_key(11, 2)
    top = [r for r in range(R) if int(new[r]) > 2 ** 32][:2]
    picks = sorted(set([0, 7] + top + _wrapping_ranks(new, ns, N)))
    for r in picks:
        got = _gen(eng, r, r + 1).cpu().numpy()[0]
        assert np.array_equal(got, _twin(version, key, r, old, new, ns, B, N)), r
    assert int(_gen(eng, top[0], top[0] + 1).max()) > 2 ** 32
    assert _coverage(eng, N, R, 512)
    eng.close()


def test_c5_big_pool_consecutive_epochs():
    lengths, N, R, B, ver = W.shape("c5")
    eng = _engine(lengths, N, R, B, ver, seed=0)
    ns = eng.num_samples
    outs = []
    for epoch in range(4):   # sequential epochs cycle the lookahead buffers
        eng.init_iter(epoch)
        old, new = eng.rank_starts()
        outs.append((epoch, old.copy(), new.copy(), _gen(eng, 0, R)))
    for epoch, old, new, out in outs:
        key = O.epoch_key(0, epoch)
        o = out.cpu().numpy()
        for r in sorted({epoch % R, R - 1}):
            assert np.array_equal(o[r], _twin(ver, key, r, old, new, ns, B, N)), (epoch, r)
    del outs
    eng.init_iter(9)
    assert _coverage(eng, N, R, R)
    eng.close()


def test_c5_hundred_consecutive_epochs_cover_exactly():
    """BASELINE configs[4] as stated: B = 2^20 pools with the per-epoch set_epoch reseed over 100
    epochs.  Epochs 0..99 run back to back through the lookahead ring (each epoch's key table /
    pre-pass queued on the side stream during the previous replay); every epoch's (count,
    digest) over all 8 ranks equals [0, N)'s, and two epochs' rank streams equal the twin."""
    lengths, N, R, B, ver = W.shape("c5")
    eng = _engine(lengths, N, R, B, ver, seed=0)
    ns = eng.num_samples
    want = O.digest_range(0, N) & 0xFFFFFFFFFFFFFFFF       # N = ns * R: no pad
    out = torch.empty((R, ns), dtype=torch.int64, device="cuda")
    accs = torch.zeros(100, dtype=torch.int64, device="cuda")
    twin_at = {37: None, 99: None}
    for epoch in range(100):
        eng.init_iter(epoch)
        if epoch in twin_at:
            twin_at[epoch] = eng.rank_starts()
        eng.generate(0, R, out=out)
        pss.digest(out.view(-1), accs[epoch:epoch + 1])
        if epoch in twin_at:
            twin_at[epoch] = (twin_at[epoch], out[epoch % R].cpu().numpy())
    eng.check()
    got = [int(x) & 0xFFFFFFFFFFFFFFFF for x in accs.cpu().tolist()]
    bad = [e for e in range(100) if got[e] != want]
    assert not bad, "epochs whose digest differs: %s" % bad
    for epoch, ((old, new), row) in twin_at.items():
        key = O.epoch_key(0, epoch)
        assert np.array_equal(row, _twin(ver, key, epoch % R, old, new, ns, B, N)), epoch
    eng.close()


def test_c5_fused_mapping_equals_generate_then_map():
    """pss_generate_mapped at C5 (B = 2^20, the grouped replay maps each id in-kernel): equal to
    generate + pss_map over all 8 ranks, for two consecutive epochs (the second replay takes the
    lookahead's key table) and a ragged position range."""
    lengths, N, R, B, ver = W.shape("c5")
    eng = _engine(lengths, N, R, B, ver, seed=0)
    ns = eng.num_samples
    for epoch in (0, 1):
        eng.init_iter(epoch)
        f, o = eng.generate_mapped(0, R)
        eng.check()
        ids = _gen(eng, 0, R)
        fr, orr = eng.map(ids.view(-1))
        assert torch.equal(f.view(-1), fr) and torch.equal(o.view(-1).long(), orr), epoch
        del ids, fr, orr
    f2, o2 = eng.generate_mapped(2, 5, 123_457, 3 * B + 11)
    eng.check()
    assert torch.equal(f2, f[2:5, 123_457:123_457 + 3 * B + 11])
    assert torch.equal(o2, o[2:5, 123_457:123_457 + 3 * B + 11])
    eng.close()


@pytest.mark.parametrize("B", [1 << 16, 1 << 18, 1 << 20])
def test_big_pool_exact_order_matches_rank_select_oracle(B):
    """order="exact" (the reference's MT19937 draws, V2:96-116) on pools far beyond the
    list.remove restatement's reach, up to C5's B = 2^20: two ranks of ns = 3.5 B steps -- three
    pool2 windows of B steps (the last partial) decoded through the global merge levels, and a
    B-step tail whose reseeds take two-word MT keys.  Every rank's stream == the exact oracle's
    rank-select restatement (oracle/pss_oracle.c orc_v2_exact_stream_rs, itself checked against
    the list.remove restatement and the reference's goldens in tests/test_oracle_golden.py)."""
    R = 2
    ns = int(3.5 * B)
    N, F = ns * R - 1, 70          # one pad id: the last rank's block wraps at N
    lengths = np.full(F, N // F)
    lengths[-1] += N - lengths.sum()
    gpu = pss.IndexEngine(lengths, N, R, B, 2, device=0, shuffle=True, seed=3, order="exact")
    assert gpu.num_samples == ns
    for epoch in (5, 2 ** 32 - 2):
        gpu.init_iter(epoch)
        old, new = gpu.rank_starts()
        a = _gen(gpu, 0, R).cpu().numpy()
        for r in range(R):
            ref = O.v2_exact_stream_rs(epoch, int(old[r]), int(new[r]), ns, B, N)
            assert np.array_equal(a[r], ref), (B, epoch, r, int(np.argmax(a[r] != ref)))
    gpu.close()


@pytest.mark.parametrize("B,ns_mult", [(300_007, 2.6), ((1 << 17) + 3, 4.3)])
def test_split_draws_odd_pools_match_rank_select_oracle(B, ns_mult):
    """The split draws of long pool2 windows (pss_v2split.h, DESIGN 4.4: per-segment piecewise
    transfers, the guess-and-verify walk, phases re-anchored ahead of the power-of-two crossings
    of the k2 bound) at pools that are not powers of two -- the k1 bound's acceptance is not 1/2,
    so the plan's rates and the crossings differ from C5's -- with a last window of another
    length (a second plan), over two consecutive epochs and an epoch jump (cold calls: the
    split form; a prepared next epoch: the workgroup form).  == the exact oracle (V2:96-116)."""
    R = 2
    ns = int(ns_mult * B)
    N, F = ns * R - 1, 53             # one pad id: the last rank's block wraps at N
    lengths = np.full(F, N // F)
    lengths[-1] += N - lengths.sum()
    gpu = pss.IndexEngine(lengths, N, R, B, 2, device=0, shuffle=True, seed=11, order="exact")
    assert gpu.num_samples == ns
    for epoch in (3, 4, 9):
        gpu.init_iter(epoch)
        old, new = gpu.rank_starts()
        a = _gen(gpu, 0, R).cpu().numpy()
        for r in range(R):
            ref = O.v2_exact_stream_rs(epoch, int(old[r]), int(new[r]), ns, B, N)
            assert np.array_equal(a[r], ref), (B, epoch, r, int(np.argmax(a[r] != ref)))
    gpu.close()


def test_split_draws_two_engines_on_threads():
    """Two engines on two host threads and two streams, each drawing cold exact epochs of long
    pool2 windows at the same time: the split form (pss_v2split.h) shares one generator side
    stream and its events per device, one call's record / wait pairs kept together by a mutex.
    Epochs are not consecutive (no draws made ahead: every call draws for itself).  Each engine's
    streams == the exact oracle (V2:96-116)."""
    from concurrent.futures import ThreadPoolExecutor
    B, R = 1 << 18, 2
    ns = int(2.5 * B)
    N, F = ns * R - 1, 31
    lengths = np.full(F, N // F)
    lengths[-1] += N - lengths.sum()
    engs = [pss.IndexEngine(lengths, N, R, B, 2, device=0, shuffle=True, seed=sd, order="exact") for sd in (5, 6)]
    streams = [torch.cuda.Stream(device=0) for _ in engs]

    def run(k):
        eng, st, res = engs[k], streams[k], []
        for epoch in (11, 3, 40):
            eng.init_iter(epoch)
            old, new = eng.rank_starts()
            out = eng.generate(0, R, stream=st)
            st.synchronize()
            eng.check(st)
            res.append((epoch, old, new, out.cpu().numpy()))
        return res

    with ThreadPoolExecutor(2) as ex:
        results = list(ex.map(run, range(2)))
    for res in results:
        for epoch, old, new, a in res:
            for r in range(R):
                ref = O.v2_exact_stream_rs(epoch, int(old[r]), int(new[r]), ns, B, N)
                assert np.array_equal(a[r], ref), (epoch, r, int(np.argmax(a[r] != ref)))
    for eng in engs:
        eng.close()


def test_c5_pool_exact_order_equals_cpu_mode():
    """The same C5 pool (B = 2^20) through the product's CPU mode (Fenwick trees,
    pss_cpu.cpp): GPU == CPU mode bit for bit (both are checked against the rank-select oracle
    above and in tests/test_cpu_mode.py)."""
    R, B = 2, 1 << 20
    ns = int(3.5 * B)
    N, F = ns * R, 70
    lengths = np.full(F, N // F)
    lengths[-1] += N - lengths.sum()
    kw = dict(shuffle=True, seed=3, order="exact")
    gpu = pss.IndexEngine(lengths, N, R, B, 2, device=0, **kw)
    cpu = pss.IndexEngine(lengths, N, R, B, 2, device="cpu", **kw)
    gpu.init_iter(5)
    cpu.init_iter(5)
    a = _gen(gpu, 0, R).cpu().numpy()
    assert np.array_equal(a, cpu.generate(0, R).numpy())


def test_exact_order_launch_sizes_beyond_2_32_threads():
    """Exact V2 with tiny pools over long streams: B = 2 makes every rank ~1.1M pool2 windows,
    i.e. 1.1M decode-tile blocks of 1024 threads per rank -- more than 2^32 threads for the
    four ranks together, which the launches must split.  GPU == CPU mode."""
    R, B, ns = 4, 2, 2_200_001
    N = ns * R
    lengths = np.full(9, N // 9)
    lengths[-1] += N - lengths.sum()
    kw = dict(shuffle=True, seed=1, order="exact")
    gpu = pss.IndexEngine(lengths, N, R, B, 2, device=0, **kw)
    cpu = pss.IndexEngine(lengths, N, R, B, 2, device="cpu", **kw)
    gpu.init_iter(0)
    cpu.init_iter(0)
    a = _gen(gpu, 0, R).cpu().numpy()
    assert np.array_equal(a, cpu.generate(0, R).numpy())
    gpu.close()


@pytest.mark.parametrize("cfg,version,pad", [("c2", 2, 0), ("c2", 2, 3), ("c2", 1, 3),
                                             ("c5", 2, 0), ("c5", 2, 3), ("c5", 1, 3)])
def test_exact_order_at_bench_shape_matches_exact_oracle(cfg, version, pad):
    """order="exact" at the shapes bench.py reports it on: C2 (R = 8, ns = 12.5M, B = 4096: the
    V2 chain mode, ~3000 chunks linked per rank) and C5 (B = 2^20: 12 pool2 windows through
    the global merge levels; V1 windows through HBM).  pad = 3 drops three samples from the last
    file so that ns * R - N = 3 and the block at 7 * ns wraps at N (V1:161-163, V2:113-114).
    Two ranks per epoch (rank 0 and the wrapping / last block) == the exact oracle (V2: the
    rank-select restatement), over two consecutive epochs; all 8 ranks are generated at once."""
    from concurrent.futures import ThreadPoolExecutor
    lengths, N, R, B, _ = W.shape(cfg)
    lengths = lengths.copy()
    lengths[-1] -= pad
    N -= pad
    eng = pss.IndexEngine(lengths, N, R, B, version, device=0, shuffle=True, order="exact")
    ns = eng.num_samples
    assert ns * R - N == pad
    with ThreadPoolExecutor(4) as ex:           # the oracle calls release the GIL
        for epoch in (0, 1):
            eng.init_iter(epoch)
            old, new = eng.rank_starts()
            last = int(np.argmax(new))              # the block at 7 * ns: wraps when pad > 0
            picks = sorted({0, last})
            if version == 1:
                futs = [ex.submit(O.v1_exact_stream, epoch, int(new[r]), ns, B, N) for r in picks]
            else:
                futs = [ex.submit(O.v2_exact_stream_rs, epoch, int(old[r]), int(new[r]), ns, B, N)
                        for r in picks]
            out = _gen(eng, 0, R).cpu().numpy()
            for r, f in zip(picks, futs):
                ref = f.result()
                assert np.array_equal(out[r], ref), (cfg, version, pad, epoch, r,
                                                     int(np.argmax(out[r] != ref)))
            if pad:
                assert int(out[last].min()) < pad <= ns   # wrapped ids present
            del out
    eng.close()
