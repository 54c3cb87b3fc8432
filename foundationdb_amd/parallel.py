"""Multi-GPU sharding for batched CRC-32C (one process per GPU).

Buffers are independent, so a batch shards with no data-path collective
(SURVEY.md §8e): every rank checksums a contiguous slice of the batch on its
own GPU.  Collectives (RCCL over xGMI with the "nccl" backend, gloo on CPU)
are used only to gather the per-buffer results or the aggregate timing, and
-- for one whole-stream CRC over shards (FileTransfer semantics,
fdbrpc/FileTransfer.cpp:29-37) -- to fold the shard CRCs with crc32c_combine.
"""
import numpy as np
import torch
import torch.distributed as dist

from .crc32c import crc32c_combine


def shard_bounds(count, rank, world):
    """Contiguous, balanced [begin, end) of `count` equal-size buffers."""
    per, extra = divmod(int(count), int(world))
    begin = rank * per + min(rank, extra)
    return begin, begin + per + (1 if rank < extra else 0)


def shard_bounds_by_bytes(lengths, rank, world):
    """Contiguous [begin, end) of a variable-length batch, balanced by bytes."""
    lengths = np.asarray(lengths, dtype=np.uint64)
    if lengths.size == 0:
        return 0, 0
    csum = np.cumsum(lengths, dtype=np.float64)
    total = float(csum[-1])
    cut = lambda r: int(np.searchsorted(csum, total * r / world, side="right")) if r < world else lengths.size  # noqa: E731
    b = 0 if rank == 0 else cut(rank)
    return b, max(b, cut(rank + 1))


def gather_checksums(local, counts, group=None):
    """All-gather per-rank checksum vectors (uint32 tensors of lengths `counts`)
    into the full batch order on every rank."""
    world = dist.get_world_size(group)
    m = max(counts)
    buf = torch.zeros(m, dtype=torch.int64, device=local.device)
    buf[: local.numel()] = local.to(torch.int64)
    parts = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf, group=group)
    return torch.cat([p[:c] for p, c in zip(parts, counts)]).to(torch.int64)


def fold_stream(shard_crcs, shard_lengths, seed=0):
    """crc32c_append(seed, A0 || A1 || ...) from crc_k = crc32c_append(0, A_k)."""
    crc = seed
    for c, n in zip(shard_crcs, shard_lengths):
        crc = crc32c_combine(crc, int(c), int(n))
    return crc
