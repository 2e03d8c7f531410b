#!/usr/bin/env python
"""Benchmark of the MI355X partial-shuffle sampler's hot path (BASELINE.json metric).

Default workload (BASELINE.json configs[1]): V2 two-pool sampler, 10,000 files
x 10,000 samples = 100M samples, 8 logical ranks, shuffle_buffer 4096 -- per GPU.  One step =
one epoch: set_epoch + init_iter (host CPython-MT file/block history, epoch upload) +
generation of every id of the GPU's logical ranks into HBM.  With --gpus N (torchrun, one
process per GPU) GPU g owns logical ranks [8g, 8g+8) of an 8N-rank sampler over N x 100M samples
(weak scaling, no data-path collective); after the timed loop the ranks all-gather
(count, coverage digest) over RCCL and rank 0 checks exact coverage.
Other workloads (--workload): c2v1 (V1 on C2's files), c5 (B = 2^20 pools beyond LDS, weak),
c3 (1B samples / 100K files / R = 1024 sharded over the N GPUs: strong scaling, the total work
of BASELINE configs[2] is fixed), c4 (configs[3]: Zipf file sizes, 2.59B samples, R = 4096,
strong).

Prints ONE JSON line (rank 0).  `value` is the whole-job throughput (all GPUs' ids / the
slowest rank's time), `per_gpu` = value / N is the metric's per-GPU figure.  Also reported:
the dominant kernel's HBM roofline (live HIP-event timing on the launch stream), the CPU
baseline (the reference algorithm restated, on this box's host cores, bounded samples;
cpu_baseline), set_epoch -> first batch latency at 1B samples through the drop-in sampler
class, and the sampler's full per-epoch data path (generate + map + pinned D2H).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import workloads as W  # noqa: E402
from partiallyshuffledistributedsampler_amd.distributed import (  # noqa: E402
    coverage_ok, expected_digest_gpu, gather_pairs, shard)
from partiallyshuffledistributedsampler_amd.engine import IndexEngine, as_u64, digest  # noqa: E402

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
BYTES_PER_ID = 8               # one int64 id written per emitted index
METRIC = "shuffled indices/sec per GPU (G idx/s) + % HBM roofline; set_epoch latency @1B"

# name: (workloads.py config, scaling) -- weak: per-GPU files and ranks fixed, strong: the
# configuration's total fixed and its logical ranks sharded over the GPUs
WORKLOADS = {
    "c2": ("c2", "weak"),
    "c2v1": ("c2", "weak"),
    "c5": ("c5", "weak"),
    "c3": ("c3", "strong"),
    "c4": ("c4", "strong"),
}


def _pmc_traffic(workload, symbols):
    """(HBM bytes per launch, source) of the first kernel symbol found for this workload in
    profiles/pmc_traffic.json (written by tools/pmc_summary.py from separate rocprofv3 --pmc
    FETCH_SIZE / WRITE_SIZE passes over this same bench at N=1 -- not measured in this run), or
    (None, None)."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(p) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None, None
    for sym in symbols:
        e = d.get(workload, {}).get(sym, {})
        v = e.get("hbm_bytes_per_launch")
        if v is not None:
            src = {"file": "profiles/pmc_traffic.json", "workload": workload, "symbol": sym,
                   "measured": "separate rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) of this bench, "
                               "not this run"}
            for k in ("round", "source", "build", "passes"):
                if k in e:
                    src[k] = e[k]
            if "_meta" in d:
                src["meta"] = d["_meta"]
            return v, src
    return None, None


# ---- CPU baseline --------------------------------------------------------------------------------
def _host():
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"cores": len(os.sched_getaffinity(0)), "cpu_model": model}


def _reference_processes(workload, version, nproc, batches, bs, use_gc):
    """The reference's __next__ loop (oracle/pyref.py via oracle/cpu_ref.py) for logical ranks
    0..nproc-1 of `workload`, one process per rank, all started together; aggregate ids/s =
    all ids / (last end - first start).  Child processes of this one (fork + exec of a fresh
    interpreter that never touches the GPU)."""
    import subprocess
    env = {k: v for k, v in os.environ.items() if not k.startswith("PSS_")}
    env["OMP_NUM_THREADS"] = "1"
    procs = [subprocess.Popen([sys.executable, "-m", "oracle.cpu_ref", workload, str(version),
                               str(r), str(batches), str(bs), "1" if use_gc else "0"],
                              cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                              text=True) for r in range(nproc)]
    res = []
    for p in procs:
        o, e = p.communicate(timeout=300)
        if p.returncode != 0:
            raise RuntimeError("cpu_ref worker failed: %s" % e[-2000:])
        res.append(json.loads(o.strip().splitlines()[-1]))
    ids = sum(r["ids"] for r in res)
    span = max(r["wall_end"] for r in res) - min(r["wall_start"] for r in res)
    return {"idx_per_s": ids / span, "processes": nproc, "ids": ids, "seconds": span,
            "per_process_idx_per_s": float(np.median([r["ids"] / r["seconds"] for r in res])),
            "batches_per_rank": batches, "batch_size": bs, "gc_collect_per_batch": use_gc}


def cpu_baseline():
    """The reference's own per-batch loop on this box's host cores, as the reference runs: one
    single-threaded process per logical rank (BASELINE.md "CPU-baseline plan"; the reference
    is not on the GPU box -- oracle/pyref.py restates its loops and tests/test_oracle_golden.py
    pins them to its recorded streams):
      value   -- C2 (the bench workload): V2 __next__ (get_index draws with list.remove pools,
                 V2:96-116; id -> (file, offset) walk and row gather, V2:181-248; the per-batch
                 gc.collect() of V2:253) in 8 processes, ranks 0..7, a prefix of 64 batches of
                 1024 each -- aggregate G idx/s (extrapolated to the epoch: the rate is flat);
      gc_off  -- the same with gc.collect() stubbed;
      c1_v1   -- C1 (BASELINE configs[0]): V1 __next__ (V1:151-259) in 2 processes, gc on / off;
      c_port  -- the oracle's C port of get_index on whole C2 rank streams, one thread: the
                 reference algorithm without the interpreter (labelled, not the headline);
      c3_v2 / c5_v2 -- Python get_index prefixes at B = 4096 / 2^20, one process, extrapolated;
      c3_v2_set_epoch_to_first_batch_ms -- Python init_iter (100K-file shuffle, 1024 blocks) +
                 the first 1024 get_index draws at C3.
    """
    import gc
    import random
    from oracle import oracle as O
    from oracle.pyref import V2Draws
    host = _host()
    nproc = max(1, min(8, host["cores"], 16))
    lengths, N, R, B, _ = W.shape("c2")
    ns = O.num_samples(N, R)
    on = _reference_processes("c2", 2, nproc, 64, 1024, True)
    off = _reference_processes("c2", 2, nproc, 64, 1024, False)
    out = {"value": on["idx_per_s"] / 1e9, "unit": "G idx/s", "cores": nproc,
           "kind": "python_restatement",
           "port_of": "the reference's Python __next__ loop restated line for line in Python "
                      "(oracle/pyref.py, pinned to the reference's recorded streams), run by the "
                      "CPython interpreter -- not a compiled port",
           "sample": "reference V2 __next__ loop (oracle/pyref.py: get_index + map + gather + "
                     "per-batch gc.collect, V2:96-116,170-254) at C2, %d processes = logical "
                     "ranks 0..%d, 64 batches x 1024 ids each, all concurrent; extrapolated "
                     "(label: extrapolated) the C2 epoch (%d ids) takes %.0f s"
                     % (nproc, nproc - 1, ns * R, ns * R / on["idx_per_s"]),
           "gc_on": on, "gc_off": off, "host": host}
    # C1, Python V1 loop, gc on / off, one process per rank (R = 2)
    l1, N1, R1, B1, _ = W.shape("c1")
    ns1 = O.num_samples(N1, R1)
    c1 = {}
    for use_gc in (True, False):
        r = _reference_processes("c1", 1, min(R1, nproc), 64, 1024, use_gc)
        r["epoch_s_extrapolated"] = ns1 * R1 / r["idx_per_s"]
        c1["gc_on" if use_gc else "gc_off"] = r
    out["c1_v1"] = c1
    # the C port of the reference algorithm, one thread, whole rank streams (bounded)
    total, t0, r = 0, time.perf_counter(), 0
    while r < R and time.perf_counter() - t0 < 6.0:
        hr = O.RefHistory(2, len(lengths), R, r, N)
        hr.init_iter(0)
        total += len(O.v2_exact_stream(0, hr.old_start, hr.start, ns, B, N))
        r += 1
    dt = time.perf_counter() - t0
    out["c_port"] = {"value": total / dt / 1e9, "unit": "G idx/s", "cores": 1,
                     "sample": "oracle C port of get_index (CPython MT19937 + list.remove pools, "
                               "V2:96-116), full epoch streams of C2 ranks 0..%d (%d ids, %.1f s)"
                               % (r - 1, total, dt)}
    # C3 / C5 get_index prefixes
    for name, draws in (("c3", 65536), ("c5", 256)):
        ln, Nn, Rn, Bn, _ = W.shape(name)
        nsn = O.num_samples(Nn, Rn)
        d = V2Draws(0, 0, nsn, Bn)
        gc.disable()
        t0 = time.perf_counter()
        for _ in range(draws):
            d.get_index()
        dt = time.perf_counter() - t0
        gc.enable()
        out["%s_v2" % name] = {
            "idx_per_s": draws / dt,
            "epoch_s_extrapolated_one_rank": dt / draws * nsn,
            "sample": "%d get_index draws of one rank (B=%d), extrapolated (label: extrapolated)"
                      % (draws, Bn)}
    # C3 set_epoch -> first batch, Python: init_iter's shuffles (V2:142-152) + 1024 draws
    ln, Nn, Rn, Bn, _ = W.shape("c3")
    nsn = O.num_samples(Nn, Rn)
    files = list(range(len(ln)))
    times = []
    for e in range(3):
        t0 = time.perf_counter()
        random.seed(e)
        fid = list(range(len(files)))
        random.shuffle(fid)
        files = [files[i] for i in fid]
        blocks = list(range(Rn))
        random.seed(e + 1)
        random.shuffle(blocks)
        d = V2Draws(0, nsn * blocks[0], nsn, Bn, epoch=e)
        for _ in range(1024):
            d.get_index()
        times.append((time.perf_counter() - t0) * 1e3)
    out["c3_v2_set_epoch_to_first_batch_ms"] = float(np.median(times))
    return out


def cpu_mode_figure(seconds_budget=8.0):
    """The product's own CPU mode (libpss PSS_DEVICE_CPU, the GPU's schedule on host threads)
    on the c2 workload: G idx/s and the threads it used."""
    lengths, N, R, B, ver = W.shape("c2")
    env = os.environ.get("PSS_CPU_THREADS")
    threads = int(env) if env and int(env) > 0 else len(os.sched_getaffinity(0))
    eng = IndexEngine(lengths, N, R, B, ver, seed=0, device="cpu")
    out = torch.empty((R, eng.num_samples), dtype=torch.int64)
    steps, t0 = 0, time.perf_counter()
    while steps < 3 and time.perf_counter() - t0 < seconds_budget:
        eng.init_iter(steps)
        eng.generate(0, R, out=out)
        steps += 1
    dt = time.perf_counter() - t0
    eng.close()
    return {"value": R * eng.num_samples * steps / dt / 1e9, "unit": "G idx/s",
            "threads": threads, "sample": "%d epochs of c2 (all 8 ranks)" % steps}


# ---- latency and the drop-in data path ---------------------------------------------------------
class _DS:
    def __init__(self, files):
        self.files = files

    def reset(self):
        pass


def _reader_for(fl, width):
    arr = np.arange(width, dtype=np.int64)

    def reader(path, get_data=False):
        n = fl[path]
        return n if not get_data else ({"x": arr[:n]}, n)
    return reader


def latency_dropin(device, reps=5):
    """set_epoch(e); next(iter(sampler)) at 1B samples / 100K files / R = 1024 (C3) through the
    drop-in DistributedSamplerViaLocallyShuffleV2 class with an in-memory reader: host
    init_iter + the epoch's tables + the rank's epoch as (file, offset) pairs (the fused
    hand-off) + pinned D2H + the first batch's grouping and file read.  Also the 128 logical
    ranks one of 8 GPUs owns (ranks=(0, 128)), order="exact" (the reference's own draws: the
    bit-identical stream; warm = consecutive epochs, cold = an epoch that does not follow the
    previous one, its MT draws made in the call), and the engine-level figure."""
    from partiallyshuffledistributedsampler_amd.DistributedSamplerViaLocallyShuffleV2 import \
        DistributedSamplerViaLocallyShuffle as V2
    lengths, N, R, B, _ = W.shape("c3")
    files = ["c3/%06d.npz" % i for i in range(len(lengths))]
    fl = dict(zip(files, lengths.tolist()))
    reader = _reader_for(fl, int(lengths.max()))
    res = {}
    for key, kw in (("set_epoch_to_first_batch_ms", {}),
                    ("set_epoch_to_first_batch_128_ranks_ms", {"ranks": (0, 128)}),
                    ("exact_set_epoch_to_first_batch_ms", {"order": "exact"})):
        s = V2(_DS(files), reader, num_replicas=R, rank=0, shuffle_buffer=B, total_size=1,
               batch_size=1024, files_len=fl, device=device, **kw)
        times = []
        for e in range(reps + 1):
            torch.cuda.synchronize(device)
            t0 = time.perf_counter()
            s.set_epoch(e)
            b = next(iter(s))
            t1 = time.perf_counter()
            assert sum(len(d["x"]) for d in b[0]) == 1024
            if e:
                times.append((t1 - t0) * 1e3)
        res[key] = float(np.median(times))
        if not kw or kw.get("order") == "exact":
            # cold: a resume at an epoch the host prefetcher has not prepared (it computes the
            # coming epochs' file permutations, V2:143-144, on worker threads): the O(F) CPython-MT
            # shuffle of 100K files runs inside set_epoch -> first batch (exact order: also the
            # epoch's MT draws, none made ahead)
            cold = []
            for e in (57, 113, 171, 229, 287):
                torch.cuda.synchronize(device)
                t0 = time.perf_counter()
                s.set_epoch(e)
                b = next(iter(s))
                cold.append((time.perf_counter() - t0) * 1e3)
                assert sum(len(d["x"]) for d in b[0]) == 1024
            res["cold_" + key] = float(np.median(cold))
            res["cold_epochs"] = "57, 113, 171, 229, 287 after 0..%d (prefetcher misses), median" % reps
    # engine only: init_iter + generate + map + D2H of the first batch
    eng = IndexEngine(lengths, N, R, B, 2, seed=0, device=device)
    ns = eng.num_samples
    ids = torch.empty((1, ns), dtype=torch.int64, device=device)
    fpos = torch.empty(ns, dtype=torch.int32, device=device)
    off = torch.empty(ns, dtype=torch.int64, device=device)
    h_f = torch.empty(1024, dtype=torch.int32, pin_memory=True)
    h_o = torch.empty(1024, dtype=torch.int64, pin_memory=True)
    times = []
    for e in range(reps + 1):
        torch.cuda.synchronize(device)
        t0 = time.perf_counter()
        eng.init_iter(e)
        eng.generate(0, 1, out=ids)
        eng.map(ids.view(-1), fpos, off)
        h_f.copy_(fpos[:1024], non_blocking=True)
        h_o.copy_(off[:1024], non_blocking=True)
        torch.cuda.synchronize(device)
        if e:
            times.append((time.perf_counter() - t0) * 1e3)
    eng.close()
    res["engine_set_epoch_to_first_batch_ms"] = float(np.median(times))
    res["config"] = ("V2, 100K files / 1B samples, R=1024, B=4096, batch 1024, in-memory "
                     "reader; through DistributedSamplerViaLocallyShuffleV2 (one rank, and "
                     "ranks=(0, 128): one of 8 GPUs' block)")
    return res


def sampler_data_path(device, reps=5):
    """The drop-in's per-epoch device path at C2 for one rank (12.5M ids): set_epoch + iter ->
    the epoch's tables + the fused hand-off (the rank's (int32 file, int32 offset) pairs in one
    pass) + pinned D2H of every pair; ms until all of it is on the host."""
    from partiallyshuffledistributedsampler_amd.DistributedSamplerViaLocallyShuffleV2 import \
        DistributedSamplerViaLocallyShuffle as V2
    lengths, N, R, B, _ = W.shape("c2")
    files = ["c2/%05d.npz" % i for i in range(len(lengths))]
    fl = dict(zip(files, lengths.tolist()))
    s = V2(_DS(files), _reader_for(fl, int(lengths.max())), num_replicas=R, rank=0,
           shuffle_buffer=B, total_size=1, batch_size=1024, files_len=fl, device=device)
    times = []
    for e in range(reps + 1):
        torch.cuda.synchronize(device)
        t0 = time.perf_counter()
        s.set_epoch(e)
        iter(s)
        s._wait_host(s.num_samples)
        t1 = time.perf_counter()
        if e:
            times.append((t1 - t0) * 1e3)
    ms = float(np.median(times))
    return {"epoch_ms": ms, "ids": s.num_samples, "G_idx_per_s": s.num_samples / ms / 1e6,
            "host_bytes": s.num_samples * 8,
            "host_GBps": s.num_samples * 8 / (ms * 1e-3) / 1e9,
            "config": "C2, one rank (12.5M ids): fused hand-off (pss_generate_mapped) + pinned D2H "
                      "of (int32 file, int32 offset) per id"}


def handoff_figures(device, reps=20, warm=4):
    """The fused hand-off (all 8 logical ranks, 100M positions): pss_generate_mapped -> (int32
    file, int32 offset) per position in HBM, mapped inside the generation kernels -- V1 and V2 at
    C2, V2 at C5 (the grouped replay), and C4's Zipf file sizes (the pairs do not fit 31 bits
    there: the segment map) at C2's size; consecutive epochs after `warm` warm-up epochs (the V2
    lookahead primed and its buffers grown) into preallocated outputs; and the standalone map of
    100M int64 ids.  frac_of_8TBps: 8 B per position against the HBM spec."""
    out = {}
    for key, ver, cfg in (("v1_mapped", 1, "c2"), ("v2_mapped", 2, "c2"), ("c5_v2_mapped", 2, "c5"),
                          ("zipf_v2_mapped", 2, "c4")):
        lengths, N, R, B, _ = W.shape(cfg)
        if cfg == "c4":                 # C4's file sizes, C2's sample count and ranks
            lengths = lengths[np.cumsum(lengths) <= 100_000_000]
            N, R = int(lengths.sum()), 8
        eng = IndexEngine(lengths, N, R, B, ver, seed=0, device=device)
        ns = eng.num_samples
        fp = torch.empty((R, ns), dtype=torch.int32, device=device)
        of = torch.empty_like(fp)
        for e in range(warm):
            eng.init_iter(e)
            eng.generate_mapped(0, R, out=(fp, of))
        torch.cuda.synchronize(device)
        t0 = time.perf_counter()
        for e in range(reps):
            eng.init_iter(warm + e)
            eng.generate_mapped(0, R, out=(fp, of))
        torch.cuda.synchronize(device)
        ms = (time.perf_counter() - t0) / reps * 1e3
        out[key] = {"ms_per_epoch": ms, "G_pos_per_s": R * ns / ms / 1e6,
                    "frac_of_8TBps": R * ns * 8 / (ms * 1e-3) / (HBM_PEAK_GBS * 1e9),
                    "files": len(lengths), "positions": R * ns}
        del fp, of
        if ver == 2 and cfg == "c2":
            ids = eng.generate(0, R)
            fp, off = eng.map(ids.view(-1))
            torch.cuda.synchronize(device)
            t0 = time.perf_counter()
            for _ in range(reps):
                eng.map(ids.view(-1), fp, off)
            torch.cuda.synchronize(device)
            ms = (time.perf_counter() - t0) / reps * 1e3
            out["map_100M_ids_ms"] = ms
            del ids, fp, off
        eng.close()
    out["config"] = ("C2 (V1, V2), C5 (V2, B = 2^20: the grouped replay) and C4's Zipf sizes cut to "
                     "~100M samples (V2), 8 logical ranks, ~12.5M positions each -> (int32 file_pos, "
                     "int32 offset); %d epochs after %d warm-up epochs" % (reps, warm))
    return out


def exact_order_figures(device):
    """order="exact" (the reference's own CPython-MT19937 draws, bit-identical id streams) at
    the bench shapes: C2 (V2 and V1, B = 4096) and C5's pool (B = 2^20), all 8 logical ranks.
    cold: an epoch that does not follow the previous call's, drawn in its own call; steady:
    consecutive epochs after two warm-up epochs, the draws of the coming epochs made ahead on side streams (the
    exact lookahead); ms per epoch (init_iter + generate, synchronised), G idx/s, and the
    pipeline's span on the caller's stream (HIP events around the launch)."""
    res = {}
    for name, cfg, ver, reps in (("c2_v2", "c2", 2, 12), ("c2_v1", "c2", 1, 12), ("c5_v2", "c5", 2, 12),
                                 ("c5_v1", "c5", 1, 12), ("c3_v2", "c3", 2, 6)):
        lengths, N, R, B, _ = W.shape(cfg)
        eng = IndexEngine(lengths, N, R, B, ver, seed=0, device=device, order="exact")
        ns = eng.num_samples
        out = torch.empty((R, ns), dtype=torch.int64, device=device)
        eng.init_iter(0)                 # workspaces
        eng.generate(0, R, out=out)
        torch.cuda.synchronize(device)
        t0 = time.perf_counter()
        eng.init_iter(5)                 # not epoch 0 + 1: its own draws, none made ahead
        eng.generate(0, R, out=out)
        torch.cuda.synchronize(device)
        cold = (time.perf_counter() - t0) * 1e3
        for e in (6, 7):                 # 6 queues the draws of 7, 8, ...
            eng.init_iter(e)
            eng.generate(0, R, out=out)
        torch.cuda.synchronize(device)
        eng.profile(True)
        t0 = time.perf_counter()
        for e in range(reps):
            eng.init_iter(8 + e)
            eng.generate(0, R, out=out)
        # the caller's stream: the draws made ahead for the epochs after these belong to them
        torch.cuda.current_stream(device).synchronize()
        ms = (time.perf_counter() - t0) / reps * 1e3
        torch.cuda.synchronize(device)
        prof = eng.profile_read()
        eng.check()
        eng.close()
        kname = "v2_emit" if ver == 2 else "v1_window"
        k_ms, k_n = prof.get(kname, (0.0, 0))
        res[name] = {"ms_per_epoch": ms, "G_idx_per_s": R * ns / ms / 1e6,
                     "cold_ms_per_epoch": cold,
                     "pipeline_ms_per_epoch": k_ms / max(1, k_n), "ids_per_epoch": R * ns,
                     "shuffle_buffer": B}
        del out
    res["config"] = ("order='exact' (CPython MT19937 draws: the reference's id streams bit for bit); "
                     "c2: 10K files x 10K, R=8, B=4096; c5: the same files, B=2^20; all 8 ranks per epoch; "
                     "c3: 100K files x 10K, R=1024, B=4096, all 1024 ranks (1B ids) per epoch; "
                     "ms_per_epoch: consecutive epochs (draws made ahead), cold: an epoch that does not "
                     "follow the previous call's (its own draws)")
    return res


# ---- main ------------------------------------------------------------------------------------
def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def launch_ranks(n):
    """`python bench.py --gpus N` outside a launcher: start one process per GPU through
    torch.distributed.run (127.0.0.1 rendezvous) as a CHILD of this process, which has not
    touched the GPU (no HIP call before this point; torch.cuda.device_count does not
    initialise it), relay rank 0's output and exit with the launcher's code.  The reference's
    only multi-rank harness loops its ranks in one process (V1:344-355); here every logical-rank
    shard is its own process on its own GPU."""
    import subprocess
    if os.environ.get("PSS_BENCH_SAME_GPU") != "1" and torch.cuda.device_count() < n:
        sys.stderr.write("bench.py: --gpus %d but only %d GPU(s) visible\n" % (n, torch.cuda.device_count()))
        return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.call(cmd, env=env)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="c2", choices=sorted(WORKLOADS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-latency", action="store_true")
    ap.add_argument("--no-exact", action="store_true", help="skip the exact-order figures")
    ap.add_argument("--no-kernel-timing", action="store_true",
                    help="time the steps without the per-launch HIP events (roofline omitted)")
    ap.add_argument("--pipeline", type=int, default=1,
                    help="epochs in flight: 2 alternates two streams and output buffers")
    ap.add_argument("--timing-every", type=int, default=0,
                    help="HIP-event timing of the generation kernel on every n-th timed step "
                         "(default: min(16, steps // 8), i.e. at least 8 timed launches)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        sys.stderr.write("bench.py: --gpus %d but WORLD_SIZE=%d\n" % (args.gpus, world))
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal of the multi-process path on a one-GPU box: every rank on cuda:0, gloo for the
    # (count, digest) exchange.  The real N-GPU run uses RCCL ("nccl") with one GPU per rank.
    rehearse = os.environ.get("PSS_BENCH_SAME_GPU") == "1"
    if rehearse:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    cdev = torch.device("cpu") if rehearse else dev     # device of the collective tensors
    # PSS_BENCH_DIST=1: the process group and its collectives even at one process (an RCCL
    # group of one GPU: the N-GPU code path -- barriers, the max-over-ranks time, the device
    # all-gather of (count, digest) -- executed on a one-GPU box, tests/test_distributed.py)
    distributed = world > 1 or os.environ.get("PSS_BENCH_DIST") == "1"
    if distributed:
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)

    cfg_name, scaling = WORKLOADS[args.workload]
    ver = 1 if args.workload == "c2v1" else W.CONFIGS[cfg_name][5]
    l1, _, R1, B, _ = W.shape(cfg_name)
    if scaling == "weak":        # the configuration per GPU: N x its files and ranks
        lengths = np.tile(l1, world)
        R = R1 * world
    else:                        # the configuration in total, its ranks sharded over the GPUs
        lengths, R = l1, R1
    N = int(lengths.sum())
    eng = IndexEngine(lengths, N, R, B, ver, shuffle=True, seed=0, device=local)
    ns = eng.num_samples
    r_lo, r_hi = shard(R, world, rank)
    RG = r_hi - r_lo
    # --pipeline 2: consecutive epochs alternate between two streams and two output buffers (a
    # data pipeline consuming epoch e while e + 1 is generated), so one epoch's generation may
    # start while the previous one drains; 1: every epoch on one stream into one buffer
    npipe = max(1, args.pipeline)
    outs = [torch.empty((RG, ns), dtype=torch.int64, device=dev) for _ in range(npipe)]
    streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(npipe - 1)]
    out = outs[0]
    stream = streams[0]

    def step(epoch):
        eng.init_iter(epoch)
        eng.generate(r_lo, r_hi, out=outs[epoch % npipe], stream=streams[epoch % npipe])

    for e in range(args.warmup):
        step(e)
    torch.cuda.synchronize(dev)
    eng.check()
    if distributed:
        dist.barrier()
    # live timing of the dominant kernel: two HIP events around the generation kernel on its
    # stream, on every 16th step of the timed region (C2, same box: every 4th step 557-559 G
    # idx/s, every 16th 564-565, none 567; profiles/r05/bench_overheads.txt)
    every = args.timing_every if args.timing_every > 0 else max(1, min(16, args.steps // 8))
    eng.profile(not args.no_kernel_timing, generation_only=True, every=every)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(args.warmup + i)
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    rank_ms = [dt / args.steps * 1e3]
    pg_world = 1
    if distributed:
        dist.barrier()
        pg_world = dist.get_world_size()
        t = torch.tensor([dt], dtype=torch.float64, device=cdev)
        ts = [torch.zeros_like(t) for _ in range(pg_world)]
        dist.all_gather(ts, t)
        rank_ms = [float(x.item()) / args.steps * 1e3 for x in ts]
        dt = max(float(x.item()) for x in ts)          # the slowest rank's time
    prof = eng.profile_read()
    eng.profile(False)
    eng.check()

    # coverage of the last epoch across all GPUs: (count, digest) all-gather over RCCL
    out = outs[(args.warmup + args.steps - 1) % npipe]     # the last epoch's ids
    pairs = gather_pairs(out.numel(), as_u64(digest(out.view(-1))), device=cdev)
    coverage = None
    if rank == 0:
        coverage = coverage_ok(pairs, ns, R, expected_digest_gpu(N, ns, R, dev))

    # the box's achievable write-only rate for the same buffer (after the coverage digest: this
    # overwrites the epoch's ids): torch's fill_ of the output
    # (a plain streaming-store kernel, no compute), HIP events on the same stream.  The HBM
    # roofline's `peak` stays the 8 TB/s spec; this says how much of it writes alone reach here.
    fill_ms = None
    if world == 1 and not args.no_kernel_timing:
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        out.fill_(1)
        ev0.record(stream)
        for i in range(20):
            out.fill_(i)
        ev1.record(stream)
        ev1.synchronize()
        fill_ms = ev0.elapsed_time(ev1) / 20
    ids_total = sum(c for c, _ in pairs) * args.steps
    value = ids_total / dt / 1e9
    kname = "v2_emit" if ver == 2 else "v1_window"
    k_ms, k_n = prof.get(kname, (0.0, 0))
    per_launch_ms = k_ms / max(k_n, 1)
    P1 = min(B, ns)
    if ver == 2 and P1 <= 16384:
        units = RG * (ns - P1)      # ids one v2_emit launch writes (the tail rides along)
        syms = ["k_v2_emit_x"] if eng.emit_path() == "xchg" else ["k_v2_emit"]
    elif ver == 2:
        units = RG * ns             # grouped pools: the emit kernel also drains the tail
        syms = ["k_g_emit"]
    else:
        units = RG * ns
        syms = ["k_v1_os"]           # the one-shot V1 kernel (k_v1_feistel serves the mapped form)
    achieved = units * BYTES_PER_ID / (per_launch_ms * 1e-3) / 1e9 if per_launch_ms > 0 else 0.0
    out_bytes = out.numel() * out.element_size()
    traffic, traffic_src = _pmc_traffic(args.workload, syms) if world == 1 else (None, None)
    desc = W.CONFIGS[cfg_name][0] + (" (V1 variant)" if args.workload == "c2v1" else "")
    line = {
        "metric": METRIC,
        "value": value,
        "unit": "G idx/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "int64",
        "data": "synthetic",
        "value_scope": "aggregate over all n_gpus GPUs (the metric's per-GPU figure is per_gpu)",
        "per_gpu": value / world,
        "aggregate": value,
        "config": {"workload": ("%s; %s" % (desc, "per GPU" if scaling == "weak"
                                            else "sharded over the GPUs")),
                   "name": args.workload, "version": ver, "files": len(lengths), "samples": N,
                   "logical_ranks": R, "ranks_per_gpu": RG, "shuffle_buffer": B,
                   "ids_per_step": ids_total // args.steps,
                   "parallelism": "logical ranks sharded over %d GPU(s)" % world,
                   "epochs_in_flight": npipe},
        "roofline": {"bound": "hbm", "kernel": kname, "symbols": syms, "achieved": achieved,
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                     "traffic": traffic, "traffic_source": traffic_src, "launch_ms": per_launch_ms,
                     "algorithmic_bytes_per_launch": units * BYTES_PER_ID,
                     "write_floor": None if not fill_ms else {
                         "GBps": out_bytes / (fill_ms * 1e-3) / 1e9, "ms": fill_ms,
                         "frac_of_floor": achieved / (out_bytes / (fill_ms * 1e-3) / 1e9),
                         "how": "torch fill_ of the same output buffer (write-only streaming "
                                "kernel), HIP events, mean of 20 on this box"}},
        "kernels_ms_per_launch": {k: v[0] / max(1, v[1]) for k, v in prof.items()},
        "timed_launches": k_n,
        "timing_every": every,
        "coverage_ok": coverage,
        "collective": (dist.get_backend() if distributed else None),
        "process_group_world_size": pg_world,
        "ms_per_step_by_rank": rank_ms,
    }
    eng.close()
    del out, outs
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline()
        line["cpu_mode"] = cpu_mode_figure()
    if rank == 0 and not args.no_latency:
        line["latency"] = latency_dropin(local)
        line["sampler_data_path"] = sampler_data_path(local)
        line["handoff"] = handoff_figures(local)
    if rank == 0 and world == 1 and not args.no_exact:
        line["exact_order"] = exact_order_figures(local)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
