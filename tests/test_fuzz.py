"""Seeded random geometries for the counter schedule, beyond the hand-picked CONFIGS.

Each case draws a file-length law (uniform, tiny files with zeros, Zipf, large files), a file
count, a rank count, a pool size B (log-uniform over 1 .. 300 000, so LDS pools, grouped pools
beyond 16384 and B > ns all occur), shuffle on/off, a seed and a start epoch.

  * CPU (`-m "not gpu"`): the library's CPU mode == the oracle twin (oracle/pss_oracle.c) for
    every rank, plus full coverage of [0, N) and the wrap-around pad (V1:161-163);
  * exact order (`order="exact"`, the reference's MT19937 draws) on the GPU == CPU mode at every
    pool size (V1 windows beyond 16000 take the HBM-staged resolution);
  * GPU (`-m gpu`): the HIP kernels (through the C-ABI) == CPU mode over three consecutive
    epochs (the V2 epoch lookahead), on both V2 emit paths, for random (rank, position)
    sub-ranges, the id -> (file, offset) map and the fused mapped generation, with the device
    error word checked after every call.
"""
import numpy as np
import pytest
import torch

from oracle import oracle as O

pss = pytest.importorskip("partiallyshuffledistributedsampler_amd.engine")

N_CPU_CASES = 96
N_GPU_CASES = 200
N_EXACT_CASES = 48
MAX_N = 2_000_000


def _geometry(i):
    rng = np.random.default_rng(90_000 + i)
    F = int(rng.choice([1, 2, 5, 17, 64, 300, 1000, 3000]))
    law = i % 4
    if law == 0:
        lengths = rng.integers(1, 2000, F)
    elif law == 1:
        lengths = rng.integers(0, 50, F)                      # empty and tiny files
    elif law == 2:
        lengths = np.minimum(rng.zipf(1.5, F), 200_000)       # skewed, as C4
    else:
        lengths = rng.integers(5000, 50_000, F)
    lengths = lengths.astype(np.int64)
    lengths[0] = max(int(lengths[0]), 1)
    while lengths.sum() > MAX_N:
        lengths = np.maximum(lengths // 2, 1)
    N = int(lengths.sum())
    R = int(min(rng.choice([1, 2, 3, 8, 13, 64, 130]), N))
    B = int(np.exp(rng.uniform(0.0, np.log(300_000))))
    if i % 6 == 5:          # a pool beyond 16384 slots that refills many times (C5's shape)
        lengths = rng.integers(20_000, 60_000, 40).astype(np.int64)
        N = int(lengths.sum())
        R = int(rng.integers(1, 4))
        B = int(rng.integers(16_385, -(-N // R) // 3))
    return dict(lengths=lengths, N=N, R=R, B=max(B, 1), version=1 + i % 2,
                shuffle=bool(rng.random() > 0.15), seed=int(rng.integers(0, 2 ** 31)),
                epoch=int(rng.integers(0, 1000)), path="probe" if rng.random() < 0.25 else "xchg",
                rng=rng)


def _coverage(out, N, R, ns):
    allids = np.sort(out.reshape(-1))
    pad = ns * R - N
    expect = np.sort(np.concatenate([np.arange(N), np.arange(pad)]))
    return np.array_equal(allids, expect)


@pytest.mark.parametrize("i", range(N_CPU_CASES))
def test_cpu_mode_fuzz_matches_twin(i):
    g = _geometry(i)
    eng = pss.IndexEngine(g["lengths"], g["N"], g["R"], g["B"], g["version"], shuffle=g["shuffle"],
                          seed=g["seed"], device="cpu")
    ns, R, N, B = eng.num_samples, g["R"], g["N"], g["B"]
    eng.init_iter(g["epoch"])
    old, new = eng.rank_starts()
    out = eng.generate(0, R).numpy()
    assert _coverage(out, N, R, ns), g
    if g["shuffle"] or g["version"] == 1:
        key = O.epoch_key(g["seed"], g["epoch"])
        for r in sorted({0, R // 2, R - 1}):
            if g["version"] == 1:
                ref = O.v1_philox_stream(key, r, int(new[r]), ns, B, N, g["shuffle"])
            else:
                ref = O.v2_philox_stream(key, r, int(old[r]), int(new[r]), ns, B, N)
            assert np.array_equal(out[r], ref), (i, r)


@pytest.mark.gpu
@pytest.mark.parametrize("i", range(N_GPU_CASES))
def test_gpu_fuzz_equals_cpu_mode(i, device=0):
    g = _geometry(i)
    rng = g["rng"]
    args = (g["lengths"], g["N"], g["R"], g["B"], g["version"])
    kw = dict(shuffle=g["shuffle"], seed=g["seed"])
    gpu = pss.IndexEngine(*args, device=device, **kw)
    cpu = pss.IndexEngine(*args, device="cpu", **kw)
    if g["version"] == 2:
        gpu.set_emit_path(g["path"])
    ns, R, N = gpu.num_samples, g["R"], g["N"]
    for epoch in range(g["epoch"], g["epoch"] + 3):
        gpu.init_iter(epoch)
        cpu.init_iter(epoch)
        assert np.array_equal(gpu.file_order(), cpu.file_order())
        a = gpu.generate(0, R)
        gpu.check()
        b = cpu.generate(0, R).numpy()
        a_host = a.cpu().numpy()
        assert np.array_equal(a_host, b), (i, epoch)
        assert _coverage(b, N, R, ns), (i, epoch)
        # a random (rank, position) window: the skip-ahead path
        r0 = int(rng.integers(0, R))
        r1 = int(rng.integers(r0 + 1, R + 1))
        p0 = int(rng.integers(0, ns))
        cnt = int(rng.integers(1, ns - p0 + 1))
        part = gpu.generate(r0, r1, p0, cnt)
        gpu.check()
        assert np.array_equal(part.cpu().numpy(), b[r0:r1, p0:p0 + cnt]), (i, epoch, r0, r1, p0, cnt)
        # id -> (file, offset), and the fused mapped generation
        fg, og = gpu.map(a.reshape(-1))
        gpu.check()
        fc, oc = cpu.map(torch.from_numpy(b).reshape(-1))
        assert np.array_equal(fg.cpu().numpy(), fc.numpy()) and np.array_equal(og.cpu().numpy(), oc.numpy())
        if ns * (r1 - r0) > 0:
            mf, mo = gpu.generate_mapped(r0, r1, p0, cnt)
            gpu.check()
            ref_f = fc.numpy().reshape(R, ns)[r0:r1, p0:p0 + cnt]
            ref_o = oc.numpy().reshape(R, ns)[r0:r1, p0:p0 + cnt]
            assert np.array_equal(mf.cpu().numpy(), ref_f) and np.array_equal(mo.cpu().numpy(), ref_o)


@pytest.mark.gpu
@pytest.mark.parametrize("i", range(N_EXACT_CASES))
def test_gpu_fuzz_exact_order_equals_cpu_mode(i, device=0):
    g = _geometry(i)
    args = (g["lengths"], g["N"], g["R"], g["B"], g["version"])
    kw = dict(shuffle=g["shuffle"], seed=g["seed"], order="exact")
    gpu = pss.IndexEngine(*args, device=device, **kw)
    cpu = pss.IndexEngine(*args, device="cpu", **kw)
    R, N, B = g["R"], g["N"], g["B"]
    ns = gpu.num_samples
    for epoch in (g["epoch"], g["epoch"] + 1):
        gpu.init_iter(epoch)
        cpu.init_iter(epoch)
        old, new = gpu.rank_starts()
        a = gpu.generate(0, R)
        gpu.check()
        a = a.cpu().numpy()
        assert np.array_equal(a, cpu.generate(0, R).numpy()), (i, epoch)
        # and the exact oracle (the reference's algorithm restated, oracle/pss_oracle.c), which
        # the golden fixtures pin to the reference itself (tests/test_oracle_golden.py)
        for r in sorted({0, R - 1}):
            if g["version"] == 1:
                ref = O.v1_exact_stream(epoch, int(new[r]), ns, B, N, g["shuffle"])
            else:
                ref = O.v2_exact_stream_rs(epoch, int(old[r]), int(new[r]), ns, B, N)
            assert np.array_equal(a[r], ref), (i, epoch, r)


@pytest.mark.parametrize("i", range(N_EXACT_CASES))
def test_cpu_mode_fuzz_exact_order_matches_exact_oracle(i):
    """The CPU mode's exact order (CPythonMT windows, Fenwick-tree V2) == the exact oracle on
    the same random geometries the GPU's exact order is checked on."""
    g = _geometry(i)
    cpu = pss.IndexEngine(g["lengths"], g["N"], g["R"], g["B"], g["version"], shuffle=g["shuffle"],
                          seed=g["seed"], device="cpu", order="exact")
    R, N, B, ns = g["R"], g["N"], g["B"], cpu.num_samples
    cpu.init_iter(g["epoch"])
    old, new = cpu.rank_starts()
    for r in sorted({0, R // 2, R - 1}):
        got = cpu.generate(r, r + 1).numpy()[0]
        if g["version"] == 1:
            ref = O.v1_exact_stream(g["epoch"], int(new[r]), ns, B, N, g["shuffle"])
        else:
            ref = O.v2_exact_stream_rs(g["epoch"], int(old[r]), int(new[r]), ns, B, N)
        assert np.array_equal(got, ref), (i, r)
