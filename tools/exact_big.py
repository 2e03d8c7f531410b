"""V2 exact order at big pools (up to C5's B = 2^20): GPU == CPU mode, with timings and the
first mismatching positions.  usage: python tools/exact_big.py [B[:epoch] ...]"""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from partiallyshuffledistributedsampler_amd.engine import IndexEngine  # noqa: E402
import torch  # noqa: E402

for arg in (sys.argv[1:] or [str(1 << 20)]):
    B, epoch = (list(map(int, arg.split(":"))) + [5])[:2]          # "B" or "B:epoch"
    R = 2
    ns = int(3.5 * B)                            # 3 pool2 windows, the last partial
    N, F = ns * R, 70
    lengths = np.full(F, N // F)
    lengths[-1] += N - lengths.sum()
    cpu = IndexEngine(lengths, N, R, B, 2, seed=3, device="cpu", order="exact")
    gpu = IndexEngine(lengths, N, R, B, 2, seed=3, device=0, order="exact")
    cpu.init_iter(epoch)
    gpu.init_iter(epoch)
    t = time.time()
    b = cpu.generate(0, R).numpy()
    tc = time.time() - t
    for _ in range(2):
        torch.cuda.synchronize()
        t = time.time()
        a = gpu.generate(0, R)
        gpu.check()
        torch.cuda.synchronize()
        tg = time.time() - t
    a = a.cpu().numpy()
    P, T = B, ns - B
    for r in range(R):
        d = np.nonzero(a[r] != b[r])[0]
        print("B", B, "epoch", epoch, "rank", r, "cpu %.2fs gpu %.3fs" % (tc, tg), "mismatches", len(d),
              "first", d[:4].tolist(), "T", T, "in tail", int((d >= T).sum()), flush=True)
