"""Measurement behind DESIGN.md A.R6's rank-shared counter decode estimate:
at C2 V2 (counter order) the replay of ONE rank's stream spread over the chip (pss_generate for
ranks [0, 1): the tile plan fills the chip for any rank count) -- the decode a rank-shared
schedule would run once per epoch -- beside the replay of all 8 ranks, and the exact order's
one-shot fan-out k_v2x_fanout (the fan-out such a decode would need).  Run under
rocprofv3 --kernel-trace --stats; tools/trace_by_grid.py splits the kernels by grid.

usage: python tools/ab_rank_shared.py [--epochs 20]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import workloads as W  # noqa: E402
from partiallyshuffledistributedsampler_amd.engine import IndexEngine  # noqa: E402


def timed(eng, lo, hi, out, epochs, e0):
    for e in range(4):
        eng.init_iter(e0 + e)
        eng.generate(lo, hi, out=out)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for e in range(epochs):
        eng.init_iter(e0 + 4 + e)
        eng.generate(lo, hi, out=out)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / epochs * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=20)
    a = ap.parse_args()
    lengths, N, R, B, _ = W.shape("c2")
    eng = IndexEngine(lengths, N, R, B, 2, seed=0, device=0)
    ns = eng.num_samples
    out = torch.empty((R, ns), dtype=torch.int64, device="cuda")
    res = {"one_rank_ms": timed(eng, 0, 1, out, a.epochs, 0),
           "all_ranks_ms": timed(eng, 0, R, out, a.epochs, 100)}
    eng.set_order_mode("exact")
    res["exact_all_ranks_ms"] = timed(eng, 0, R, out, a.epochs, 200)
    eng.check()
    eng.close()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
