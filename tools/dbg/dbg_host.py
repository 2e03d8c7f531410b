import sys, time, gc
GCLOG = []
def _cb(phase, info):
    GCLOG.append((phase, info.get('generation'), time.perf_counter()))
gc.callbacks.append(_cb)
import numpy as np, torch
sys.path.insert(0, ".")
import workloads as W
from partiallyshuffledistributedsampler_amd.engine import IndexEngine
for cfg, ver in (("c2", 2), ("c2", 1), ("c5", 2)):
    lengths, N, R, B, _ = W.shape(cfg)
    eng = IndexEngine(lengths, N, R, B, ver, seed=0, device=0)
    ns = eng.num_samples
    fp = torch.empty((R, ns), dtype=torch.int32, device="cuda"); of = torch.empty_like(fp)
    for e in range(3):
        eng.init_iter(e); eng.generate_mapped(0, R, out=(fp, of))
    torch.cuda.synchronize()
    ti, tg = [], []
    t00 = time.perf_counter()
    for e in range(3, 33):
        t0 = time.perf_counter(); eng.init_iter(e); t1 = time.perf_counter()
        eng.generate_mapped(0, R, out=(fp, of)); t2 = time.perf_counter()
        ti.append((t1 - t0) * 1e3); tg.append((t2 - t1) * 1e3)
    torch.cuda.synchronize()
    tot = (time.perf_counter() - t00) / 30 * 1e3
    ev = [(p, g, round((t - t00) * 1e3, 2)) for p, g, t in GCLOG if t >= t00]
    GCLOG.clear()
    print('gc events in loop', ev)
    print(cfg, ver, "epoch ms %.3f" % tot, "init_iter ms", np.round(ti, 3).tolist())
    print("   generate_mapped ms", np.round(tg, 3).tolist())
    eng.close()
