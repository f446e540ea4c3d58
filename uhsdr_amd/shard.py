"""Channel sharding across the GPUs of a node.

Channels are independent radios: no term of the chain couples two channels, so a batch
splits into contiguous channel ranges, one per rank (one process per GPU), with no
collective on the data path.  The only communication is the optional gather of the f32
audio to rank 0 (torch.distributed.gather: grouped RCCL send/recv over xGMI on the GPU
box, gloo on CPU in the tests).
"""
from __future__ import annotations


def channel_range(per_rank: int, rank: int) -> tuple[int, int]:
    """Weak scaling: every rank owns `per_rank` channels; rank r owns [r*per_rank, (r+1)*per_rank)."""
    return rank * per_rank, (rank + 1) * per_rank


def split_range(total: int, world: int, rank: int) -> tuple[int, int]:
    """Strong scaling: `total` channels split into `world` contiguous ranges (the first
    total % world ranks get one more)."""
    base, extra = divmod(total, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def gather_to_root(local, dist, world: int, rank: int):
    """Rank 0 receives every rank's [C_r, N] block (equal C_r) and returns them concatenated
    along channels in rank order; other ranks return None."""
    import torch
    if world == 1:
        return local
    parts = [torch.empty_like(local) for _ in range(world)] if rank == 0 else None
    dist.gather(local, gather_list=parts, dst=0)
    return torch.cat(parts, dim=0) if rank == 0 else None
