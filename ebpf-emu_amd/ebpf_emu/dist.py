"""Multi-GPU sharding of a packet batch (one process per GPU, torch.distributed).

Packets are independent and the program is read-only, so a batch shards with no data-path
exchange. A global batch is a sequence of seeded chunks (workloads.py): rank r
of W owns the contiguous chunk range shard_chunks(K, W, r) and generates only those chunks, so
the global result is the same for every W. The single exchange step is the sum of the 8
per-verdict counters (RCCL all-reduce over xGMI on GPUs; gloo in the CPU tests).
"""
from __future__ import annotations


def shard_chunks(n_chunks: int, world: int, rank: int) -> range:
    """Contiguous, balanced (+-1) chunk range of `rank`."""
    lo = n_chunks * rank // world
    hi = n_chunks * (rank + 1) // world
    return range(lo, hi)


def chunk_sizes(total_packets: int, chunk: int) -> list[int]:
    """Packets per chunk of a global batch of `total_packets` (the last chunk may be short)."""
    full, rest = divmod(total_packets, chunk)
    return [chunk] * full + ([rest] if rest else [])


CHUNK = 1 << 20  # packets per seeded chunk of a global batch (BASELINE config 4)


def chunk_seed(k: int) -> int:
    """config_id of chunk k of the config-4 global batch: the one formula bench.py
    --total-packets, tests/golden/make_golden.py (config4.json) and the tests all use."""
    return 3 + 100 * k


def chunk_frames(k: int, size: int):
    """Chunk k of the global batch: `size` seeded 64-byte frames (workloads.frames_fixed)."""
    from . import workloads as W

    return W.frames_fixed(size, 64, config_id=chunk_seed(k))


def reduce_counters(counters, group=None):
    """Sum the per-rank counters (int64 tensor [8], u64 bit patterns) across ranks in place."""
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized():
        dist.all_reduce(counters, op=dist.ReduceOp.SUM, group=group)
    return counters
