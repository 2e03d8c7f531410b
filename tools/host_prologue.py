"""Host prologue per epoch at the weak-scaled C2 shapes (F = 10K files per GPU): init_iter
back to back after a short warm-up, i.e. with the file-order permutations prefetched by the
handle's worker threads.  CPU mode (the prologue is the same host code as in GPU mode).
Usage: python tools/host_prologue.py"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import workloads as W  # noqa: E402
from partiallyshuffledistributedsampler_amd.engine import IndexEngine  # noqa: E402


def main():
    l1, _, R1, B, _ = W.shape("c2")
    print("cpus in affinity mask:", len(os.sched_getaffinity(0)))
    for world in (1, 4, 8):
        lengths = np.tile(l1, world)
        eng = IndexEngine(lengths, int(lengths.sum()), R1 * world, B, 2, seed=0, device="cpu")
        for e in range(5):
            eng.init_iter(e)
        t = time.perf_counter()
        for e in range(5, 105):
            eng.init_iter(e)
        print("world %d  F %d  init_iter back to back %.4f ms" %
              (world, len(lengths), (time.perf_counter() - t) / 100 * 1e3))
        eng.close()


if __name__ == "__main__":
    main()
