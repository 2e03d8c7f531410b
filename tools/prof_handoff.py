"""Profiling driver: pss_generate_mapped on C2 (all 8 ranks, 100M positions) for a few epochs,
V2 then V1; run under rocprofv3 --kernel-trace --stats to see the mapped kernels' durations."""
import sys

import torch

sys.path.insert(0, ".")
import workloads as W  # noqa: E402
from partiallyshuffledistributedsampler_amd.engine import IndexEngine  # noqa: E402


def main():
    lengths, N, R, B, _ = W.shape("c2")
    for ver in (2, 1):
        eng = IndexEngine(lengths, N, R, B, ver, seed=0, device=0)
        for e in range(8):
            eng.init_iter(e)
            eng.generate_mapped(0, R)
        torch.cuda.synchronize()
        eng.close()
    print("done")


if __name__ == "__main__":
    main()
