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


class GatherPipeline:
    """Per-launch outputs gathered to rank 0 while the next launch computes.

    `depth` output buffers are used round robin.  Step s computes into buffer s % depth and
    issues its gather asynchronously (``dist.gather(..., async_op=True)``); before buffer k is
    reused, the gather that last read it is waited for.  With RCCL the collective runs on the
    process group's own stream, ordered after the compute stream at issue time, and
    ``Work.wait()`` orders the compute stream after it, so the whole pipeline stays on the
    device queues (no host sync); with gloo (CPU tests) ``wait()`` blocks the caller.

    Rank 0 hands every completed step to ``sink(step, parts)`` (parts: one tensor per rank,
    in rank order) in step order, right before the receive buffers are reused or at drain().
    Backend-agnostic: only ``dist.gather`` and ``Work.wait`` are used.

    With one rank there is nothing to gather and the collective is skipped, unless `always` is
    set: then the one-rank group still runs every ``dist.gather`` (device buffers, ``async_op``,
    ``Work.wait``, the backend's own stream), which exercises the RCCL leg on a one-GPU box.
    """

    def __init__(self, dist, world: int, rank: int, make_buffer, depth: int = 2, sink=None, always: bool = False):
        if depth < 1:
            raise ValueError("depth >= 1")
        self.dist, self.world, self.rank, self.depth, self.sink = dist, world, rank, depth, sink
        self.collective = world > 1 or always
        self.bufs = [make_buffer() for _ in range(depth)]
        self.recv = [[make_buffer() for _ in range(world)] if rank == 0 else None for _ in range(depth)]
        self.work = [None] * depth
        self.issued = 0          # steps issued
        self.retired = 0         # steps whose gather has been waited for

    def _retire(self, k: int) -> None:
        w = self.work[k]
        if w is None:
            return
        w.wait()
        self.work[k] = None
        if self.rank == 0 and self.sink is not None:
            self.sink(self.retired, self.recv[k])
        self.retired += 1

    def step(self, compute) -> None:
        """compute(out) fills this step's output buffer (enqueue only)."""
        k = self.issued % self.depth
        self._retire(k)                       # the gather of step issued - depth read buffer k
        compute(self.bufs[k])
        if not self.collective:
            if self.sink is not None:
                self.sink(self.issued, [self.bufs[k]])
            self.retired += 1
        else:
            self.work[k] = self.dist.gather(self.bufs[k], gather_list=self.recv[k], dst=0, async_op=True)
        self.issued += 1

    def drain(self) -> None:
        """Wait for every gather in flight, oldest first."""
        for i in range(self.issued - self.depth, self.issued):
            if i >= 0:
                self._retire(i % self.depth)


def timed_loop(step, sync, steps: int, warmup: int, dist=None, world: int = 1, reduce_device="cpu") -> float:
    """The bench contract's timed region, shared by bench.py and the multi-rank tests: `warmup`
    untimed steps, then exactly `steps` steps bracketed by a barrier + sync() on both sides; returns
    the MAX over ranks of the elapsed seconds (all_reduce on a tensor on `reduce_device`: the GPU
    for RCCL, the CPU for gloo).  step(s) enqueues step s; sync() waits for the device."""
    import time

    import torch
    for s in range(warmup):
        step(s)
    sync()
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for s in range(steps):
        step(s)
    sync()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device=reduce_device)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_timed(pipe: "GatherPipeline", compute, sync, steps: int, warmup: int, dist, reduce_device="cpu") -> float:
    """timed_loop for the gather leg: every step's output gathered to rank 0 through `pipe`
    (overlapped with the next step), drained before each clock read; max-over-ranks seconds."""
    import time

    import torch
    for _ in range(warmup):
        pipe.step(compute)
    pipe.drain()
    sync()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        pipe.step(compute)
    pipe.drain()
    sync()
    dist.barrier()
    t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=reduce_device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
