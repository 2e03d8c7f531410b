"""Cold exact epochs (each call draws for itself) at C2's files and 8 ranks for several pool sizes:
ms per epoch, V2 and V1; run once as is and once with PSS_EXACT_SPLIT=0 (tools/gpu_split.sh)."""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from partiallyshuffledistributedsampler_amd.engine import IndexEngine  # noqa: E402

lengths = np.full(10_000, 10_000, dtype=np.int64)
N, R = int(lengths.sum()), 8
for ver in (2, 1):
    for B in (1 << 14, 1 << 16, 1 << 18):
        eng = IndexEngine(lengths, N, R, B, ver, seed=0, device=0, order="exact")
        out = torch.empty((R, eng.num_samples), dtype=torch.int64, device="cuda")
        eng.init_iter(0)
        eng.generate(0, R, out=out)
        torch.cuda.synchronize()
        ts = []
        for e in (5, 9, 13, 17):   # never consecutive: no draws made ahead
            t0 = time.perf_counter()
            eng.init_iter(e)
            eng.generate(0, R, out=out)
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        eng.close()
        print(json.dumps({"version": ver, "B": B, "split_env": os.environ.get("PSS_EXACT_SPLIT", "default"),
                          "cold_ms": round(float(np.median(ts)), 3)}), flush=True)
