import time, sys, numpy as np, torch
sys.path.insert(0, '/root/repo')
from partiallyshuffledistributedsampler_amd.engine import IndexEngine
eng = IndexEngine(np.full(10000, 10000), 10**8, 8, 4096, 2, seed=0, device=0)
out = torch.empty((8, eng.num_samples), dtype=torch.int64, device='cuda')
s = torch.cuda.current_stream()
for e in range(3):
    eng.init_iter(e); eng.generate(0, 8, out=out, stream=s)
torch.cuda.synchronize()
ti = tg = 0.0
t0 = time.perf_counter()
for e in range(3, 43):
    a = time.perf_counter(); eng.init_iter(e); b = time.perf_counter(); eng.generate(0, 8, out=out, stream=s); c = time.perf_counter()
    ti += b - a; tg += c - b
torch.cuda.synchronize()
T = time.perf_counter() - t0
print("step us %.1f  host init_iter %.1f  host generate call %.1f" % (T / 40 * 1e6, ti / 40 * 1e6, tg / 40 * 1e6))
