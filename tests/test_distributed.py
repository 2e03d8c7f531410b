"""Multi-process (gloo, world_size 2, CPU) coverage of the N>1 path: logical-rank sharding,
the (count, digest) all-gather and the coverage check.  Ids come from the oracle's Philox
twin here (the GPU produces the same ids bit for bit, see test_gpu_parity.py)."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from partiallyshuffledistributedsampler_amd.distributed import coverage_ok, gather_pairs, shard


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, version, corrupt, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import oracle as O
    rng = np.random.default_rng(2)
    lengths = rng.integers(100, 900, 50)
    N, R, B, seed, epoch = int(lengths.sum()), 7, 128, 11, 4
    ns = O.num_samples(N, R)
    key = O.epoch_key(seed, epoch)
    lo, hi = shard(R, world, rank)
    cnt, dig = 0, 0
    for r in range(lo, hi):
        h = O.RefHistory(version, len(lengths), R, r, N)
        h.init_iter(epoch)
        if version == 1:
            ids = O.v1_philox_stream(key, r, h.start, ns, B, N)
        else:
            ids = O.v2_philox_stream(key, r, h.old_start, h.start, ns, B, N)
        if corrupt and rank == 1 and r == hi - 1:
            ids = ids.copy()
            ids[0] = ids[1]           # a duplicate + a drop: the digest must notice
        cnt += len(ids)
        dig = (dig + O.digest(ids)) & ((1 << 64) - 1)
    pairs = gather_pairs(cnt, dig)
    pad = ns * R - N
    expect = (O.digest_range(0, N) + O.digest_range(0, pad)) & ((1 << 64) - 1)
    q.put((rank, coverage_ok(pairs, ns, R, expect), len(pairs)))
    dist.destroy_process_group()


@pytest.mark.parametrize("version,corrupt", [(1, False), (2, False), (2, True)])
def test_two_process_coverage(version, corrupt):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, version, corrupt, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert [r[2] for r in res] == [2, 2]
    assert all(r[1] == (not corrupt) for r in res)


def test_shard_is_a_partition():
    for R in (1, 7, 8, 1024, 4096):
        for world in (1, 2, 3, 8):
            blocks = [shard(R, world, g) for g in range(world)]
            assert blocks[0][0] == 0 and blocks[-1][1] == R
            assert all(blocks[i][1] == blocks[i + 1][0] for i in range(world - 1))
            assert max(b - a for a, b in blocks) - min(b - a for a, b in blocks) <= 1
