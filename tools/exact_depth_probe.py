"""Steady exact C5 (V2 and V1) ms per epoch against the exact lookahead depth (pss_set_lookahead):
consecutive epochs after 10 warm-up epochs, 12 timed."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import workloads as W  # noqa: E402
from partiallyshuffledistributedsampler_amd.engine import IndexEngine  # noqa: E402

lengths, N, R, B, _ = W.shape("c5")
for ver in (2, 1):
    for depth in (0, 2, 4, 8):
        eng = IndexEngine(lengths, N, R, B, ver, seed=0, device=0, order="exact")
        eng.set_lookahead(exact_depth=depth)
        out = torch.empty((R, eng.num_samples), dtype=torch.int64, device="cuda")
        for e in range(10):
            eng.init_iter(e)
            eng.generate(0, R, out=out)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for e in range(10, 22):
            eng.init_iter(e)
            eng.generate(0, R, out=out)
        torch.cuda.current_stream().synchronize()
        ms = (time.perf_counter() - t0) / 12 * 1e3
        torch.cuda.synchronize()
        eng.close()
        print(json.dumps({"version": ver, "exact_depth": depth, "ms_per_epoch": round(ms, 3)}), flush=True)
