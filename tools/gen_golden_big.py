#!/usr/bin/env python
"""Reference-captured golden vectors at bench-scale pools and the big BASELINE shapes
(SURVEY.md §8c "Goldens to commit", VERDICT r03 "next" item 1).  Build container only.

Like tools/gen_golden.py this imports the two reference modules read-only from
/root/reference (same harness shims: Sampler.__init__ accepts data_source, the modules' gc is
a no-op) and records what they produce.  The streams here are too long to store whole, so a
fixture keeps per (rank, epoch): the id count, sha256 of the little-endian int64 raw stream, sha256
of the sorted stream (the epoch multiset), head / tail ids, and for V1 per-window sha256.
Short streams (the Zipf scenario) are stored whole in an .npz next to the JSON.

Capture:
  * V2: the raw stream is what `get_index()` returns (V2:96-116), called directly after
    `iter(sampler)` -- exactly the `indices` of V2:176.
  * V1: the generation loop lives inside `__next__` (V1:157-172).  A local trace function
    grabs the `indices` list object when it appears in the frame and then switches tracing off
    for that frame; the loop appends to the same object, so after `__next__` returns it holds
    the batch's raw ids (no line events per id).  The fixtures have complete files_len, so no
    reflection entries (V1:195) are ever appended.

Fixtures (tests/golden/big/):
  c1_v1, c1_v2      64 files of 8000..12000 samples, R=2, B=4096, epochs 0,1,2 (all ranks)
  zipf_v1, zipf_v2  60 Zipf files (N ~ 30K), R=7, B=400, epochs 0,1,2 -- full streams (.npz)
  v2_b65536_*       R=2, ns = 3.5 B (B = 65536), one pad id; epochs 5 and 2^32-2 (two-word seeds)
  v1_c5_r*          C5's files (10K x 10K, R=8), V1 at B = 2^20: whole rank streams, 12 windows
  v2_c5_prefix_r*   C5 (V2, B = 2^20): the first 20480 draws of a rank
  assign_c3, assign_c4   file order / blocks / start_num history over init_iter(0,1,1,9) at
                         C3 (100K files, R=1024) and C4 (Zipf, R=4096), V1 and V2
  v2_c2_r*, v2_c3_r*, v2_c4_r*   whole V2 rank streams at the true BASELINE shapes (B = 4096):
                         C2 ranks 0 and 7 (12.5M ids each, epoch 0); C3 rank 0 and the ranks
                         whose block wraps at N, epochs 0 and 1; C4 rank 0, the wrapping rank
                         and two ranks with every id above 2^31, epoch 0
  v1_c2_r*, v1_c3_r*, v1_c4_r*   whole V1 rank streams at the same shapes (round 6, VERDICT r05
                         item 5): C2 ranks 0 and 7 (epoch 0); C3 rank 0 and the ranks whose
                         block wraps at N, epochs 0 and 1; C4 rank 0, the wrapping rank and a
                         rank whose every id lies above 2^31, epoch 0 -- per-window sha256 too

Usage:  python tools/gen_golden_big.py [job ... | bench_shapes | bench_shapes_v1]
        (default: every job, 6 processes)
"""
import hashlib
import importlib.util
import json
import os
import sys
import time
import types
from concurrent.futures import ProcessPoolExecutor

import numpy as np

sys.dont_write_bytecode = True
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
REF = "/root/reference"
OUT = os.path.join(ROOT, "tests", "golden", "big")
V1_FILE = os.path.join(REF, "DistributedSamplerViaLocallyShuffle.py")
V2_FILE = os.path.join(REF, "DistributedSamplerViaLocallyShuffleV2.py")
HEAD = 4096


def _load(ver):
    import torch.utils.data as tud
    tud.Sampler.__init__ = lambda self, data_source=None: None
    path = V1_FILE if ver == 1 else V2_FILE
    spec = importlib.util.spec_from_file_location("ref_v%d" % ver, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    mod.gc = types.SimpleNamespace(collect=lambda: 0)
    return mod


class Dataset:
    """The reference's `dataset` protocol: `.files` + `.reset()` (V1:101)."""

    def __init__(self, files):
        self.files = list(files)

    def reset(self):
        pass


def make_reader(lengths):
    def reader(path, get_data=False):
        n = lengths[path]
        if not get_data:
            return n
        return {"off": np.arange(n, dtype=np.int32)}, n
    return reader


def names(F):
    return ["f%06d" % i for i in range(F)]


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a, dtype="<i8").tobytes()).hexdigest()


def sampler(ver, lens, R, rank, B, bs):
    mod = _load(ver)
    files = names(len(lens))
    lengths = dict(zip(files, (int(x) for x in lens)))
    return mod.DistributedSamplerViaLocallyShuffle(
        Dataset(files), make_reader(lengths), num_replicas=R, rank=rank, shuffle=True,
        shuffle_buffer=B, total_size=1, batch_size=bs, files_len=dict(lengths))


def v1_epoch_stream(s):
    """Raw V1 ids of one epoch (after set_epoch): every `indices` list of V1:157-172."""
    it = iter(s)
    parts = []

    def local(frame, event, arg):
        if event == "line" and "indices" in frame.f_locals:
            parts.append(frame.f_locals["indices"])
            frame.f_trace_lines = False     # a None return alone keeps line events coming
            frame.f_trace = None
            return None
        return local

    def glob(frame, event, arg):
        if frame.f_code.co_filename == V1_FILE and frame.f_code.co_name == "__next__":
            return local
        return None

    while True:
        sys.settrace(glob)
        try:
            next(it)
        except StopIteration:
            break
        finally:
            sys.settrace(None)
    return np.fromiter((x for p in parts for x in p), dtype=np.int64)


def v2_epoch_stream(s, limit=None):
    """Raw V2 ids of one epoch: get_index() (V2:96-116) until both pools are empty."""
    iter(s)
    out = []
    while len(s.batch_ids) or len(s.batch_ids2):
        out.extend(s.get_index())
        if limit is not None and len(out) >= limit:
            break
    a = np.asarray(out, dtype=np.int64)
    return a if limit is None else a[:limit]


def stream_record(a, B=None, windows=False, full=False):
    rec = {"count": int(len(a)), "sha256": sha(a), "sorted_sha256": sha(np.sort(a))}
    if not full:
        rec["head"] = a[:HEAD].tolist()
        rec["tail"] = a[-HEAD:].tolist() if len(a) > HEAD else []
    if windows:
        rec["window_sha256"] = [sha(a[w:w + B]) for w in range(0, len(a), B)]
    return rec


def run_stream(ver, lens, R, B, bs, ranks, epochs, limit=None, windows=False, full=False):
    recs, full_streams = [], {}
    for r in ranks:
        s = sampler(ver, lens, R, r, B, bs)
        rr = {"rank": r, "num_samples": s.num_samples, "epochs": []}
        for e in epochs:
            s.set_epoch(e)
            old = s.start_num
            a = v1_epoch_stream(s) if ver == 1 else v2_epoch_stream(s, limit)
            er = {"epoch": e, "old_start": int(old), "start_num": int(s.start_num),
                  "blocks_sha256": sha(s.blocks)}
            er.update(stream_record(a, B, windows, full))
            if full:
                full_streams["r%d_e%d" % (r, e)] = a
            rr["epochs"].append(er)
        recs.append(rr)
    return recs, full_streams


def lens_rec(lens):
    lens = np.asarray(lens, dtype=np.int64)
    if len(lens) <= 200:
        return {"lengths": lens.tolist()}
    return {"F": int(len(lens)), "lengths_sha256": sha(lens)}


def write(name, fx, arrays=None):
    os.makedirs(OUT, exist_ok=True)
    with open(os.path.join(OUT, name + ".json"), "w") as f:
        json.dump(fx, f, separators=(",", ":"))
    if arrays:
        np.savez_compressed(os.path.join(OUT, name + ".npz"),
                            **{k: v.astype(np.int32) for k, v in arrays.items()})


# ---- jobs ----------------------------------------------------------------------------------

def c1_lens():
    return np.random.default_rng(2024).integers(8000, 12001, 64).astype(np.int64)


def zipf_lens():
    return np.clip(np.random.default_rng(77).zipf(1.5, 60) * 50, 1, 2000).astype(np.int64)


def job_c1(ver):
    lens = c1_lens()
    R, B, bs = 2, 4096, 1024
    recs, _ = run_stream(ver, lens, R, B, bs, range(R), [0, 1, 2], windows=(ver == 1))
    write("c1_v%d" % ver, {"kind": "stream", "version": ver, "R": R, "B": B, "bs": bs,
                           **lens_rec(lens), "ranks": recs})


def job_zipf(ver):
    lens = zipf_lens()
    R, B, bs = 7, 400, 64
    recs, full = run_stream(ver, lens, R, B, bs, range(R), [0, 1, 2], full=True)
    write("zipf_v%d" % ver, {"kind": "stream", "version": ver, "R": R, "B": B, "bs": bs,
                             **lens_rec(lens), "ranks": recs, "full_npz": True}, full)


def b65536_lens():
    B, R = 1 << 16, 2
    ns = int(3.5 * B)
    N, F = ns * R - 1, 70
    lens = np.full(F, N // F, dtype=np.int64)
    lens[-1] += N - lens.sum()
    return lens


def job_b65536(rank, epoch):
    lens = b65536_lens()
    R, B = 2, 1 << 16
    recs, _ = run_stream(2, lens, R, B, 1024, [rank], [epoch])
    write("v2_b65536_r%d_e%d" % (rank, epoch),
          {"kind": "stream", "version": 2, "R": R, "B": B, "bs": 1024, **lens_rec(lens),
           "ranks": recs})


def c5_lens():
    return np.full(10_000, 10_000, dtype=np.int64)


def job_v1_c5(rank):
    R, B = 8, 1 << 20
    recs, _ = run_stream(1, c5_lens(), R, B, 1 << 16, [rank], [0, 1], windows=True)
    write("v1_c5_r%d" % rank, {"kind": "stream", "version": 1, "R": R, "B": B, "bs": 1 << 16,
                               "uniform": [10_000, 10_000], "ranks": recs})


def job_v2_c5_prefix(rank):
    R, B, n = 8, 1 << 20, 20480
    recs, _ = run_stream(2, c5_lens(), R, B, 1024, [rank], [0], limit=n)
    write("v2_c5_prefix_r%d" % rank, {"kind": "prefix", "version": 2, "R": R, "B": B,
                                      "bs": 1024, "prefix": n, "uniform": [10_000, 10_000],
                                      "ranks": recs})


def job_assign(cfg):
    import workloads as W
    lens, N, R, B, _ = W.shape(cfg)
    out = {"kind": "assignment", "config": cfg, "R": R, "B": B, "N": N, **lens_rec(lens),
           "epochs": [0, 1, 1, 9], "versions": {}}
    for ver in (1, 2):
        s = sampler(ver, lens, R, 0, B, 1)
        idx = {p: i for i, p in enumerate(s.dataset.files)}
        hist = []
        for e in out["epochs"]:
            s.set_epoch(e)
            old_blocks = list(s.blocks)
            iter(s)
            order = np.array([idx[p] for p in s.files], dtype=np.int64)
            blocks = np.asarray(s.blocks, dtype=np.int64)
            hist.append({"epoch": e, "num_samples": s.num_samples,
                         "order_sha256": sha(order), "order_head": order[:32].tolist(),
                         "blocks_sha256": sha(blocks), "blocks_head": blocks[:32].tolist(),
                         "start_sha256": sha(blocks * s.num_samples),
                         "prev_blocks_sha256": sha(old_blocks)})
        out["versions"]["v%d" % ver] = hist
    write("assign_%s" % cfg, out)


def _v2_blocks(cfg, epochs):
    """blocks of each epoch as the reference's V2 sets them (V2:142-148), from rank 0's sampler."""
    import workloads as W
    lens, N, R, B, _ = W.shape(cfg)
    s = sampler(2, lens, R, 0, B, 1)
    out = {}
    for e in epochs:
        s.set_epoch(e)
        iter(s)
        out[e] = list(s.blocks)
    return out, N, R, B


def bench_shape_ranks(cfg):
    """(ranks, epochs) recorded at a true BASELINE shape: rank 0 plus
    the ranks whose block wraps at N (block R-1; C3 has pad 512) and, at C4, two ranks whose
    ids all lie above 2^31 (old start ns*rank and new start ns*block both past 2^31)."""
    if cfg == "c2":
        return [0, 7], [0]
    epochs = [0, 1] if cfg == "c3" else [0]
    blocks, N, R, B = _v2_blocks(cfg, epochs)
    ranks = {0} | {blocks[e].index(R - 1) for e in epochs}
    if cfg == "c4":
        ns = -(-N // R)
        hi = [r for r in range(R) if r * ns > 2 ** 31 and blocks[0][r] * ns > 2 ** 31]
        ranks |= {hi[0], hi[len(hi) // 2]}
    return sorted(ranks), epochs


def _v1_blocks(cfg, epochs):
    """blocks of each epoch as the reference's V1 sets them (cumulative shuffles, V1:118-121)."""
    import workloads as W
    lens, N, R, B, _ = W.shape(cfg)
    s = sampler(1, lens, R, 0, B, 1)
    out = {}
    for e in epochs:
        s.set_epoch(e)
        iter(s)
        out[e] = list(s.blocks)
    return out, N, R, B


def bench_shape_ranks_v1(cfg):
    """V1 ranks recorded at a true shape: rank 0, the ranks whose block is the last one (it wraps
    at N when N % R != 0), at C4 also a rank whose whole block lies above 2^31."""
    if cfg == "c2":
        return [0, 7], [0]
    epochs = [0, 1] if cfg == "c3" else [0]
    blocks, N, R, B = _v1_blocks(cfg, epochs)
    ranks = {0} | {blocks[e].index(R - 1) for e in epochs}
    if cfg == "c4":
        ns = -(-N // R)
        hi = [r for r in range(R) if blocks[0][r] * ns > 2 ** 31]
        ranks |= {hi[len(hi) // 2]}
    return sorted(ranks), epochs


def job_bench_shape_v1(cfg, rank):
    """Whole V1 rank streams at the true C2 / C3 / C4 shape (B = 4096): every `indices` of the
    reference's __next__ (V1:157-172) over the init_iter history of `epochs`."""
    import workloads as W
    lens, N, R, B, _ = W.shape(cfg)
    _, epochs = bench_shape_ranks_v1(cfg)
    recs, _ = run_stream(1, lens, R, B, 1 << 16, [rank], epochs, windows=True)
    write("v1_%s_r%d" % (cfg, rank), {"kind": "stream", "version": 1, "R": R, "B": B, "bs": 1 << 16,
                                      "config": cfg, **lens_rec(lens), "ranks": recs})


def job_bench_shape(cfg, rank):
    """Whole V2 rank streams at the true C2 / C3 / C4 shape (B = 4096), straight from the
    reference's get_index (V2:96-116) over the init_iter history of `epochs`."""
    import workloads as W
    lens, N, R, B, _ = W.shape(cfg)
    _, epochs = bench_shape_ranks(cfg)
    recs, _ = run_stream(2, lens, R, B, 1024, [rank], epochs)
    write("v2_%s_r%d" % (cfg, rank), {"kind": "stream", "version": 2, "R": R, "B": B, "bs": 1024,
                                      "config": cfg, **lens_rec(lens), "ranks": recs})


JOBS = {
    "c1_v1": (job_c1, 1), "c1_v2": (job_c1, 2),
    "zipf_v1": (job_zipf, 1), "zipf_v2": (job_zipf, 2),
    "b65536_r0_e5": (job_b65536, 0, 5), "b65536_r1_e5": (job_b65536, 1, 5),
    "b65536_r1_ebig": (job_b65536, 1, 2 ** 32 - 2),
    "v1_c5_r0": (job_v1_c5, 0), "v1_c5_r5": (job_v1_c5, 5),
    "v2_c5_prefix_r0": (job_v2_c5_prefix, 0), "v2_c5_prefix_r3": (job_v2_c5_prefix, 3),
    "assign_c3": (job_assign, "c3"), "assign_c4": (job_assign, "c4"),
}


def bench_shape_jobs():
    jobs = {}
    for cfg in ("c2", "c3", "c4"):
        for r in bench_shape_ranks(cfg)[0]:
            jobs["v2_%s_r%d" % (cfg, r)] = (job_bench_shape, cfg, r)
    return jobs


def bench_shape_jobs_v1():
    jobs = {}
    for cfg in ("c2", "c3", "c4"):
        for r in bench_shape_ranks_v1(cfg)[0]:
            jobs["v1_%s_r%d" % (cfg, r)] = (job_bench_shape_v1, cfg, r)
    return jobs


def run_job(name):
    t = time.time()
    if name in JOBS:
        fn, *args = JOBS[name]
    elif name.startswith("v1_") and name[3:5] in ("c2", "c3", "c4"):
        fn, *args = bench_shape_jobs_v1()[name]
    else:
        fn, *args = bench_shape_jobs()[name]
    fn(*args)
    return name, time.time() - t


def main(argv):
    if argv == ["bench_shapes"]:
        argv = sorted(bench_shape_jobs())
    elif argv == ["bench_shapes_v1"]:
        argv = sorted(bench_shape_jobs_v1())
    todo = argv or list(JOBS) + sorted(bench_shape_jobs())
    # the longest jobs first
    order = sorted(todo, key=lambda n: ("_c2_" not in n, "c5_prefix" not in n, "b65536" not in n, n))
    with ProcessPoolExecutor(6) as ex:
        for name, dt in ex.map(run_job, order):
            print("wrote %-18s %7.1f s" % (name, dt), flush=True)


if __name__ == "__main__":
    main(sys.argv[1:])
