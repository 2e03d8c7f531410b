"""Host cost of one C2 bench step (init_iter + generate enqueue) against its GPU period.
Prints the enqueue-only time per step (no synchronise inside the loop) and the synchronised
time per step."""
import sys, time
import numpy as np
import torch
sys.path.insert(0, ".")
from partiallyshuffledistributedsampler_amd.engine import IndexEngine

F, L, R, B = 10_000, 10_000, 8, 4096
eng = IndexEngine(np.full(F, L, dtype=np.int64), F * L, R, B, 2, shuffle=True, seed=0, device=0)
out = torch.empty((R, eng.num_samples), dtype=torch.int64, device="cuda")
s = torch.cuda.current_stream()
for e in range(5):
    eng.init_iter(e); eng.generate(0, R, out=out, stream=s)
torch.cuda.synchronize()
K = 200
t0 = time.perf_counter(); ti = 0.0
for i in range(K):
    a = time.perf_counter(); eng.init_iter(5 + i); ti += time.perf_counter() - a
    eng.generate(0, R, out=out, stream=s)
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print("enqueue us/step %.1f (init_iter %.1f), synchronised us/step %.1f" % ((t1 - t0) / K * 1e6, ti / K * 1e6, (t2 - t0) / K * 1e6))
