"""TEST / BENCH INFRASTRUCTURE ONLY -- one CPU-baseline worker process: the reference's
__next__ loop (oracle/pyref.py restatement, pinned to the reference's streams by
tests/test_oracle_golden.py) for ONE logical rank of a BASELINE workload, a bounded number of
batches, timed.  bench.py's cpu_baseline starts one of these per logical rank, all at once (the
reference is single-threaded and GIL-bound: one process per rank is how it runs on a host,
BASELINE.md "CPU-baseline plan").  Prints one JSON line {"ids", "seconds", ...}.

  python -m oracle.cpu_ref <workload> <version> <rank> <batches> <bs> <gc 0|1>
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import workloads as W  # noqa: E402
from oracle import oracle as O  # noqa: E402
from oracle.pyref import V1Loop, V2Loop  # noqa: E402


def run(workload, version, rank, batches, bs, use_gc, epoch=0):
    lengths, N, R, B, _ = W.shape(workload)
    h = O.RefHistory(version, len(lengths), R, rank, N)
    h.init_iter(epoch)                                      # the epoch's file order and blocks
    lens = lengths[h.order].tolist()
    width = int(lengths.max())
    rows = np.arange(width, dtype=np.int64)
    files = {}

    def data(f):        # in-memory reader with the reference's per-sampler file cache
        d = files.get(f)
        if d is None:
            d = files[f] = {"x": rows[:lens[f]].copy()}
        return d

    if version == 1:
        loop = V1Loop(h.start, h.ns, B, N, lens, data, epoch=epoch, bs=bs, use_gc=use_gc)
    else:
        loop = V2Loop(h.old_start, h.start, h.ns, B, N, lens, data, epoch=epoch, bs=bs,
                      use_gc=use_gc)
    n, nb = 0, 0
    w0 = time.time()
    t0 = time.perf_counter()
    while nb < batches:
        out = loop.next_batch()
        if out is None:
            break
        n += len(loop.last_indices)
        nb += 1
    dt = time.perf_counter() - t0
    return {"ids": n, "batches": nb, "seconds": dt, "rank": rank, "ns": h.ns,
            "wall_start": w0, "wall_end": w0 + dt}


if __name__ == "__main__":
    wl, ver, rank, batches, bs, g = sys.argv[1:7]
    print(json.dumps(run(wl, int(ver), int(rank), int(batches), int(bs), g == "1")))
