"""Profiling driver of the fused hand-off pss_generate_mapped (all 8 logical ranks, 100M
positions -> int32 (file, offset)): for each of C2 V2, C2 V1 and C5 V2, four warm-up epochs (the
V2 lookahead primed, its buffers grown), then `--epochs` consecutive epochs into preallocated outputs; prints one
JSON line of ms per epoch (host clock around the synchronised loop) and, with --events, the
generation kernels' HIP-event spans.  Run under rocprofv3 --kernel-trace --stats to see the
mapped kernels' durations.

usage: python tools/prof_handoff.py [--epochs 20] [--cfg c2v2,c2v1,c5v2] [--events]
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

WARM = 4   # warm-up epochs: the V2 lookahead's VAL ring grows over the first sequential calls
CFGS = {"c2v2": ("c2", 2), "c2v1": ("c2", 1), "c5v2": ("c5", 2)}


def run(name, epochs, events):
    cfg, ver = CFGS[name]
    lengths, N, R, B, _ = W.shape(cfg)
    eng = IndexEngine(lengths, N, R, B, ver, seed=0, device=0)
    ns = eng.num_samples
    # one allocation, the offsets right after the file positions (a PSS_DIAG_PAIR_INTERLEAVED
    # build writes its interleaved (file, offset) pairs over both)
    both = torch.empty((2, R, ns), dtype=torch.int32, device="cuda")
    fpos, off = both[0], both[1]
    for e in range(WARM):
        eng.init_iter(e)
        eng.generate_mapped(0, R, out=(fpos, off))
    torch.cuda.synchronize()
    if events:
        eng.profile(True)
    t0 = time.perf_counter()
    for e in range(epochs):
        eng.init_iter(WARM + e)
        eng.generate_mapped(0, R, out=(fpos, off))
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / epochs * 1e3
    res = {"ms_per_epoch": ms, "G_pos_per_s": R * ns / ms / 1e6,
           "frac_of_8TBps": R * ns * 8 / (ms * 1e-3) / 8e12}
    if events:
        res["kernels_ms_per_launch"] = {k: v[0] / max(1, v[1]) for k, v in eng.profile_read().items()}
        eng.profile(False)
    eng.check()
    eng.close()
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=20)
    ap.add_argument("--cfg", default="c2v2,c2v1,c5v2")
    ap.add_argument("--events", action="store_true")
    a = ap.parse_args()
    out = {n: run(n, a.epochs, a.events) for n in a.cfg.split(",")}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
