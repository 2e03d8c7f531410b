"""Host-side enqueue timing of the C2 bench step (init_iter + generate) against the GPU's
step time: is the host loop ahead of the GPU, or does it pace it?"""
import os, sys, time
import numpy as np
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import workloads as W
from partiallyshuffledistributedsampler_amd.engine import IndexEngine

l1, _, R, B, _ = W.shape("c2")
N = int(l1.sum())
eng = IndexEngine(l1, N, R, B, 2, shuffle=True, seed=0, device=0)
out = torch.empty((R, eng.num_samples), dtype=torch.int64, device="cuda:0")
s = torch.cuda.current_stream()
for e in range(5):
    eng.init_iter(e); eng.generate(0, R, out=out, stream=s)
torch.cuda.synchronize()
K = 200
for mode in ("normal", "init_only", "gen_only"):
    th = np.zeros(K)
    t0 = time.perf_counter()
    for i in range(K):
        a = time.perf_counter()
        if mode != "gen_only":
            eng.init_iter(5 + i)
        if mode != "init_only":
            eng.generate(0, R, out=out, stream=s)
        th[i] = time.perf_counter() - a
    t_enq = time.perf_counter() - t0
    torch.cuda.synchronize()
    t_all = time.perf_counter() - t0
    print(f"{mode}: host per step mean {th.mean()*1e6:.1f} us median {np.median(th)*1e6:.1f} p90 "
          f"{np.percentile(th, 90)*1e6:.1f} max {th.max()*1e6:.1f}; enqueue total {t_enq/K*1e6:.1f} us/step,"
          f" with sync {t_all/K*1e6:.1f} us/step", flush=True)
    if mode == "normal":
        split = np.zeros((K, 2))
        for i in range(K):
            a = time.perf_counter(); eng.init_iter(300 + i); b = time.perf_counter()
            eng.generate(0, R, out=out, stream=s); c = time.perf_counter()
            split[i] = (b - a, c - b)
        torch.cuda.synchronize()
        print(f"split: init_iter mean {split[:,0].mean()*1e6:.1f} us, generate mean {split[:,1].mean()*1e6:.1f} us", flush=True)
