"""Sharding of logical ranks over GPUs and the coverage check.

Index generation is coordination-free: every process recomputes the O(F + R) prologue and
generates only its own logical ranks.  The single collective is an all-gather of per-rank
(count, digest) pairs -- RCCL over xGMI on the GPU path, any torch.distributed backend here --
after which every process can check exact coverage of [0, N) plus the wrap-around pad.
"""
import torch
import torch.distributed as dist

U64 = (1 << 64) - 1


def shard(num_logical_ranks, world, rank):
    """Contiguous, balanced block [lo, hi) of logical ranks owned by process `rank`."""
    base, extra = divmod(num_logical_ranks, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def _to_signed(x):
    x &= U64
    return x - (1 << 64) if x >= (1 << 63) else x


def gather_pairs(count, digest_u64, device=None, group=None):
    """All-gather (count, digest) of every process -> list of python (int, uint64) tuples."""
    t = torch.tensor([[int(count), _to_signed(int(digest_u64))]], dtype=torch.int64, device=device)
    if not dist.is_available() or not dist.is_initialized():
        parts = [t]
    else:
        parts = [torch.empty_like(t) for _ in range(dist.get_world_size(group))]
        dist.all_gather(parts, t, group=group)
    return [(int(p[0, 0]), int(p[0, 1]) & U64) for p in (q.cpu() for q in parts)]


def coverage_ok(pairs, num_samples, num_logical_ranks, expected_digest):
    """True iff the gathered pairs cover every id exactly as the sampler must: ns*R ids
    whose digest equals digest([0, N)) + digest([0, ns*R - N)) (= expected_digest)."""
    total = sum(c for c, _ in pairs)
    dig = sum(d for _, d in pairs) & U64
    return total == num_samples * num_logical_ranks and dig == (expected_digest & U64)


def expected_digest_gpu(N, num_samples, num_logical_ranks, device):
    """digest([0, N)) + digest([0, pad)) computed by the pss_digest_range kernel."""
    from .engine import as_u64, digest_range
    pad = num_samples * num_logical_ranks - N
    return (as_u64(digest_range(0, N, device)) + as_u64(digest_range(0, pad, device))) & U64
