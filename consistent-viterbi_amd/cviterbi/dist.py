"""Batch sharding across GPUs and the gather of decoded paths.

The unconstrained decode is independent per sequence, so the batch is split into
contiguous shards of ceil(B/world) sequences, one per rank (one process per GPU); the
HMM is replicated.  The only collective is the gather of paths, scores and statuses to
rank 0 -- RCCL over xGMI with the "nccl" backend on the GPU node, gloo in CPU tests.
"""
from __future__ import annotations

import numpy as np


def shard_range(total: int, world: int, rank: int):
    """Contiguous shard [s0, s1) of `total` sequences for `rank` (last shards may be short)."""
    per = (total + world - 1) // world
    return min(rank * per, total), min((rank + 1) * per, total), per


def shard_offsets(offsets, s0, s1):
    """Rebase the CSR offsets of sequences [s0, s1) to start at 0."""
    offsets = np.asarray(offsets, np.int64)
    return offsets[s0:s1 + 1] - offsets[s0]


def gather_to_root(tensors, per_sizes, dist, device=None):
    """Gather each rank's tensors to rank 0, padded to the per-rank capacity `per_sizes`
    (one entry per tensor).  Returns, on rank 0, lists of per-rank tensors trimmed by
    the caller; None elsewhere."""
    import torch

    world = dist.get_world_size()
    rank = dist.get_rank()
    out = []
    for x, cap in zip(tensors, per_sizes):
        if x.numel() != cap:
            y = torch.zeros(cap, dtype=x.dtype, device=x.device)
            y[: x.numel()] = x
            x = y
        lst = [torch.empty(cap, dtype=x.dtype, device=x.device) for _ in range(world)] if rank == 0 else None
        dist.gather(x, lst, dst=0)
        out.append(lst)
    return out if rank == 0 else None


def assemble(parts, lengths):
    """Concatenate per-rank gathered buffers, keeping the first lengths[r] entries of each."""
    import torch

    return torch.cat([p[:n] for p, n in zip(parts, lengths)])
