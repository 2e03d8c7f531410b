"""Exact order at C3 (100K files, 1B samples, R = 1024, B = 4096): all 1024 ranks per call, a few
consecutive epochs after two warm-up epochs -- run under rocprofv3 --kernel-trace to see where an
exact C3 epoch goes.   usage: python tools/prof_exact_c3.py [--epochs 4]"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import workloads as W  # noqa: E402
from partiallyshuffledistributedsampler_amd.engine import IndexEngine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=4)
    a = ap.parse_args()
    lengths, N, R, B, _ = W.shape("c3")
    eng = IndexEngine(lengths, N, R, B, 2, seed=0, device=0, order="exact")
    ns = eng.num_samples
    out = torch.empty((R, ns), dtype=torch.int64, device="cuda")
    for e in range(2):
        eng.init_iter(e)
        eng.generate(0, R, out=out)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for e in range(a.epochs):
        eng.init_iter(2 + e)
        eng.generate(0, R, out=out)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / a.epochs * 1e3
    eng.check()
    eng.close()
    print(json.dumps({"exact_c3_ms_per_epoch": ms, "ids": R * ns}), flush=True)


if __name__ == "__main__":
    main()
