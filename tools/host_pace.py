#!/usr/bin/env python
"""Is the bench step host-paced?  Times, for the C2 V2 / V1 bench shapes on one GPU:
  enqueue  the loop of K steps (init_iter + generate) up to its last launch, no sync
  total    the same loop including the final synchronize
  init     K init_iter calls alone (host: the epoch's file permutation + blocks + starts)
  gen      K generate calls of one epoch (no epoch change: no host epoch work)
If enqueue ~ total, the GPU waited on the host (the gaps between steps' kernels)."""
import json, os, sys, time
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from partiallyshuffledistributedsampler_amd.engine import IndexEngine  # noqa: E402

def run(ver, K=200):
    lengths = np.full(10_000, 10_000, dtype=np.int64)
    eng = IndexEngine(lengths, int(lengths.sum()), 8, 4096, ver, shuffle=True, seed=0, device=0)
    out = torch.empty((8, eng.num_samples), dtype=torch.int64, device="cuda")
    for e in range(5):
        eng.init_iter(e); eng.generate(0, 8, out=out)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(K):
        eng.init_iter(5 + i); eng.generate(0, 8, out=out)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    for i in range(K):
        eng.init_iter(5 + K + i)
    t3 = time.perf_counter()
    torch.cuda.synchronize()
    t4 = time.perf_counter()
    for i in range(K):
        eng.generate(0, 8, out=out)
    t5 = time.perf_counter()
    torch.cuda.synchronize()
    t6 = time.perf_counter()
    eng.close()
    us = lambda a, b: (b - a) / K * 1e6
    print(json.dumps({"version": ver, "enqueue_us": us(t0, t1), "total_us": us(t0, t2),
                      "init_iter_us": us(t2, t3), "gen_enqueue_us": us(t4, t5), "gen_total_us": us(t4, t6)}),
          flush=True)

for v in (2, 1):
    run(v)
