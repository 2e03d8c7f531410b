#!/usr/bin/env python
"""Benchmark of the MI355X partial-shuffle sampler's hot path (BASELINE.json metric).

Workload (BASELINE.json configs[1]): V2 two-pool sampler, 10,000 files x
10,000 samples = 100M samples, 8 logical ranks, shuffle_buffer 4096 -- per GPU.  One step =
one epoch: set_epoch + init_iter (host CPython-MT file/block history, epoch upload) +
generation of every id of the GPU's 8 logical ranks into HBM (the id -> file prefix scan is
run by the first map after an epoch change, not by generation).  With --gpus N
(torchrun, one process per GPU) GPU g owns logical ranks [8g, 8g+8) of an 8N-rank sampler over
N x 100M samples (weak scaling, no data-path collective); after the timed loop the ranks
all-gather (count, coverage digest) over RCCL and rank 0 checks exact coverage.

Prints ONE JSON line (rank 0).  Also reported: the dominant kernel's HBM roofline (live HIP
event timing on the launch stream), the CPU oracle port of the reference algorithm on a
bounded sample (cpu_baseline), and set_epoch -> first batch latency at 1B samples.
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

from partiallyshuffledistributedsampler_amd.distributed import (  # noqa: E402
    coverage_ok, expected_digest_gpu, gather_pairs, shard)
from partiallyshuffledistributedsampler_amd.engine import IndexEngine, as_u64, digest  # noqa: E402

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
BYTES_PER_ID = 8               # one int64 id written per emitted index
METRIC = "shuffled indices/sec per GPU (G idx/s) + % HBM roofline; set_epoch latency @1B"

WORKLOADS = {
    # name: (files per GPU, samples per file, logical ranks per GPU, shuffle_buffer, version)
    "c2": (10_000, 10_000, 8, 4096, 2),
    "c2v1": (10_000, 10_000, 8, 4096, 1),
}


def _pmc_traffic(symbols):
    """HBM bytes per launch of the first kernel symbol found in profiles/pmc_traffic.json
    (written by tools/pmc_summary.py from separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE
    passes over this same bench), or None."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(p) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    for sym in symbols:
        v = d.get(sym, {}).get("hbm_bytes_per_launch")
        if v is not None:
            return v
    return None


def cpu_baseline(seconds_budget=12.0):
    """The oracle's C port of the reference V2 algorithm (CPython MT + list.remove pools,
    V2:96-116) on rank streams of the same workload, single core, bounded sample."""
    from oracle import oracle as O
    F, L, R, B, _ = WORKLOADS["c2"]
    N = F * L
    ns = O.num_samples(N, R)
    h = O.RefHistory(2, F, R, 0, N)
    h.init_iter(0)
    total, t0, r = 0, time.perf_counter(), 0
    while r < R and time.perf_counter() - t0 < seconds_budget:
        hr = O.RefHistory(2, F, R, r, N)
        hr.init_iter(0)
        total += len(O.v2_exact_stream(0, hr.old_start, hr.start, ns, B, N))
        r += 1
    dt = time.perf_counter() - t0
    return {"value": total / dt / 1e9, "unit": "G idx/s", "cores": 1, "kind": "port",
            "sample": "reference V2 algorithm (oracle C port: CPython MT19937 + list.remove "
                      "pools) over the full epoch streams of logical ranks 0..%d of the c2 "
                      "workload (%d ids, %.1f s, 1 thread)" % (r - 1, total, dt)}


def latency_1b(device, reps=5):
    """set_epoch -> first batch at 1B samples / 100K files / R=1024:
    host init_iter + epoch upload + device scan + generation of the rank's whole epoch +
    id->(file, offset) map + pinned D2H of the first batch of 1024."""
    F, L, R, B = 100_000, 10_000, 1024, 4096
    lengths = np.full(F, L, dtype=np.int64)
    eng = IndexEngine(lengths, F * L, R, B, 2, seed=0, device=device)
    ns = eng.num_samples
    ids = torch.empty((1, ns), dtype=torch.int64, device=device)
    fpos = torch.empty(ns, dtype=torch.int32, device=device)
    off = torch.empty(ns, dtype=torch.int64, device=device)
    h_f = torch.empty(1024, dtype=torch.int32, pin_memory=True)
    h_o = torch.empty(1024, dtype=torch.int64, pin_memory=True)
    times, times_gpu = [], []
    for e in range(reps + 1):
        torch.cuda.synchronize(device)
        t0 = time.perf_counter()
        eng.init_iter(e)
        eng.generate(0, 1, out=ids)
        eng.map(ids.view(-1), fpos, off)
        h_f.copy_(fpos[:1024], non_blocking=True)
        h_o.copy_(off[:1024], non_blocking=True)
        torch.cuda.synchronize(device)
        t1 = time.perf_counter()
        # all 128 logical ranks one GPU owns at 8 GPUs
        eng.init_iter(e + 1000)
        big = eng.generate(0, 128)
        torch.cuda.synchronize(device)
        t2 = time.perf_counter()
        del big
        if e:
            times.append((t1 - t0) * 1e3)
            times_gpu.append((t2 - t1) * 1e3)
    eng.close()
    return {"set_epoch_to_first_batch_ms": float(np.median(times)),
            "set_epoch_all_128_ranks_of_one_gpu_ms": float(np.median(times_gpu)),
            "config": "V2, 100K files / 1B samples, R=1024, B=4096 (one sampler rank; and the "
                      "128 logical ranks one of 8 GPUs generates)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="c2", choices=sorted(WORKLOADS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-latency", action="store_true")
    ap.add_argument("--no-kernel-timing", action="store_true",
                    help="time the steps without the per-launch HIP events (roofline omitted)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
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
    if world > 1:
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)

    F1, L, RG, B, ver = WORKLOADS[args.workload]
    F, R = F1 * world, RG * world
    N = F * L
    lengths = np.full(F, L, dtype=np.int64)
    eng = IndexEngine(lengths, N, R, B, ver, shuffle=True, seed=0, device=local)
    ns = eng.num_samples
    r_lo, r_hi = shard(R, world, rank)
    out = torch.empty((RG, ns), dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev)

    def step(epoch):
        eng.init_iter(epoch)
        eng.generate(r_lo, r_hi, out=out, stream=stream)

    for e in range(args.warmup):
        step(e)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    eng.profile(not args.no_kernel_timing)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(args.warmup + i)
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
        t = torch.tensor([dt], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    prof = eng.profile_read()
    eng.profile(False)

    # coverage of the last epoch across all GPUs: (count, digest) all-gather over RCCL
    pairs = gather_pairs(out.numel(), as_u64(digest(out.view(-1))), device=cdev)
    coverage = None
    if rank == 0:
        coverage = coverage_ok(pairs, ns, R, expected_digest_gpu(N, ns, R, dev))

    ids_total = RG * ns * world * args.steps
    value = ids_total / dt / 1e9
    kname = "v2_emit" if ver == 2 else "v1_window"
    k_ms, k_n = prof.get(kname, (0.0, 0))
    per_launch_ms = k_ms / max(k_n, 1)
    if ver == 2:
        P1 = min(B, ns)
        units = RG * (ns - P1)      # ids one v2_emit launch writes
    else:
        units = RG * ns
    achieved = units * BYTES_PER_ID / (per_launch_ms * 1e-3) / 1e9 if per_launch_ms > 0 else 0.0
    if ver == 2:
        syms = ["k_v2_emit_x"] if eng.emit_path() == "xchg" else ["k_v2_emit"]
    else:
        syms = ["k_v1_lds"]
    traffic = _pmc_traffic(syms)
    line = {
        "metric": METRIC,
        "value": value,
        "unit": "G idx/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int64",
        "data": "synthetic",
        "config": {"workload": "%s, %d files x %d samples, %d logical ranks "
                               "per GPU, shuffle_buffer %d (BASELINE configs[1] per GPU%s)"
                               % ("V2 two-pool sampler" if ver == 2 else "V1 windowed sampler",
                                  F1, L, RG, B, "" if ver == 2 else ", V1 variant"),
                   "version": ver, "files": F, "samples": N, "logical_ranks": R,
                   "shuffle_buffer": B, "ids_per_step": RG * ns * world,
                   "parallelism": "logical ranks sharded over %d GPU(s)" % world},
        "roofline": {"bound": "hbm", "kernel": kname, "achieved": achieved,
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                     "traffic": traffic, "launch_ms": per_launch_ms,
                     "algorithmic_bytes_per_launch": units * BYTES_PER_ID},
        "kernels_ms_per_step": {k: v[0] / max(1, args.steps) for k, v in prof.items()},
        "coverage_ok": coverage,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline()
    if rank == 0 and not args.no_latency:
        line["latency"] = latency_1b(local)
    if rank == 0:
        print(json.dumps(line), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
