#!/usr/bin/env python
"""Per-config generation throughput on one GPU (BASELINE.json configs[1..4]).

Not the driver's bench line (that is bench.py, C2); this measures the other configurations the
survey names, each as the share one of 8 GPUs would generate:
  c1     V1, 64 files x 10K, R=2 (BASELINE configs[0])              B=4096
  c1x    C1 with order="exact" (the reference's CPython-MT window order)
  c2     V2, 10K files x 10K, R=8 (all 8 ranks)                      B=4096
  c2v1   V1 on the same files                                        B=4096
  c2v1x  c2v1 with order="exact"
  c2x    c2 with order="exact" (the reference's own V2 stream)
  c3     V2, 100K files x 10K = 1B, R=1024 -> ranks [0, 128)         B=4096
  c4     V2, Zipf(1.5)*150 files (N=2.59e9 > 2^31), R=4096 -> [0, 512)  B=4096
  c5     V2, C2 files, B=2^20 (HBM slot-table path), 100 epochs       (reports per-epoch mean)
  c5x    c5 with order="exact"
  c5v1x  V1 on c5's shape (B=2^20 windows, HBM-staged resolution) with order="exact"
Prints one JSON line per config: ids per step, ms per step, G idx/s, per-kernel ms.  Steps are
consecutive epochs after 2 warm-up epochs: the exact configs run with their draws made ahead
(the exact lookahead, PSS_EXACT_LOOKAHEAD=0 to compare).
"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from partiallyshuffledistributedsampler_amd.engine import IndexEngine  # noqa: E402


def run(name, lengths, R, r_hi, B, ver, steps, warmup=2, order="counter"):
    N = int(lengths.sum())
    eng = IndexEngine(lengths, N, R, B, ver, seed=0, device=0, order=order)
    ns = eng.num_samples
    out = torch.empty((r_hi, ns), dtype=torch.int64, device="cuda")
    for e in range(warmup):
        eng.init_iter(e)
        eng.generate(0, r_hi, out=out)
    torch.cuda.synchronize()
    eng.profile(True)
    t0 = time.perf_counter()
    for i in range(steps):
        eng.init_iter(warmup + i)
        eng.generate(0, r_hi, out=out)
    # the caller's stream: the draws of the epochs after the timed ones, made ahead on side
    # streams (exact order), belong to those epochs
    torch.cuda.current_stream().synchronize()
    dt = (time.perf_counter() - t0) / steps
    torch.cuda.synchronize()
    prof = eng.profile_read()
    eng.close()
    ids = r_hi * ns
    print(json.dumps({"config": name, "N": N, "R": R, "ranks_generated": r_hi, "B": B,
                      "version": ver, "order": order, "ids_per_step": ids, "ms_per_step": dt * 1e3,
                      "G_idx_per_s": ids / dt / 1e9,
                      "kernels_ms": {k: v[0] / steps for k, v in prof.items()}}), flush=True)


def main():
    which = sys.argv[1:] or ["c1", "c1x", "c2", "c2x", "c2v1", "c2v1x", "c3", "c4", "c5"]
    c2 = np.full(10_000, 10_000, dtype=np.int64)
    for w in which:
        if w == "c1":      # BASELINE configs[0]: V1, 64 files x 10K, R=2
            run(w, np.full(64, 10_000, dtype=np.int64), 2, 2, 4096, 1, 50)
        elif w == "c1x":   # C1 in the reference's exact order (CPython MT per window)
            run(w, np.full(64, 10_000, dtype=np.int64), 2, 2, 4096, 1, 50, order="exact")
        elif w == "c2x":   # C2 in the reference's exact order (CPython MT, rank-deletion decode)
            run(w, c2, 8, 8, 4096, 2, 12, order="exact")
        elif w == "c2v1x":
            run(w, c2, 8, 8, 4096, 1, 12, order="exact")
        elif w == "c2":
            run(w, c2, 8, 8, 4096, 2, 20)
        elif w == "c2v1":
            run(w, c2, 8, 8, 4096, 1, 20)
        elif w == "c3":
            run(w, np.full(100_000, 10_000, dtype=np.int64), 1024, 128, 4096, 2, 20)
        elif w == "c4":
            z = np.clip(np.random.default_rng(0).zipf(1.5, 100_000) * 150, 1, 2_000_000).astype(np.int64)
            run(w, z, 4096, 512, 4096, 2, 10)
        elif w == "c5":
            run(w, c2, 8, 8, 1 << 20, 2, 100)
        elif w == "c5x":
            run(w, c2, 8, 8, 1 << 20, 2, 12, order="exact")
        elif w == "c5v1x":
            run(w, c2, 8, 8, 1 << 20, 1, 12, order="exact")


if __name__ == "__main__":
    main()
