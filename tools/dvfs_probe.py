"""Is the C2 replay's drift (135 us on the first launches, ~170-250 us later) power/clock or overlap?
Runs C2 epochs (all 8 ranks) in three phases under rocprofv3 --kernel-trace: 40 back to back,
40 with a synchronise + 3 ms idle after each, 40 back to back again; tools/dvfs_summary.py splits
the replay launches by phase."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import workloads as W  # noqa: E402
from partiallyshuffledistributedsampler_amd.engine import IndexEngine  # noqa: E402

lengths, N, R, B, ver = W.shape("c2")
eng = IndexEngine(lengths, N, R, B, ver, seed=0, device=0)
out = torch.empty((R, eng.num_samples), dtype=torch.int64, device="cuda")
e = 0
for phase, idle in (("b2b", 0.0), ("idle3ms", 0.003), ("b2b2", 0.0)):
    torch.cuda.synchronize()
    print("phase", phase, time.perf_counter(), flush=True)
    for i in range(40):
        eng.init_iter(e)
        eng.generate(0, R, out=out)
        e += 1
        if idle:
            torch.cuda.synchronize()
            time.sleep(idle)
    torch.cuda.synchronize()
eng.close()
print("done", flush=True)
