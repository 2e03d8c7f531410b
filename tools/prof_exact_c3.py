"""Exact order at C3 (100K files, 1B samples, R = 1024, B = 4096; --cfg c2: C2's 8 ranks): all
ranks per call, a few consecutive epochs after two warm-up epochs -- run under rocprofv3
--kernel-trace to see where an exact epoch goes.
usage: python tools/prof_exact_c3.py [--epochs 4] [--cfg c3]"""
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
    ap.add_argument("--cfg", default="c3")
    ap.add_argument("--version", type=int, default=2)
    a = ap.parse_args()
    lengths, N, R, B, _ = W.shape(a.cfg)
    eng = IndexEngine(lengths, N, R, B, a.version, seed=0, device=0, order="exact")
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
    print(json.dumps({"cfg": a.cfg, "version": a.version, "exact_ms_per_epoch": ms, "ids": R * ns}), flush=True)


if __name__ == "__main__":
    main()
