"""N > 1 path on CPU: world_size-2 gloo ranks, each owning a contiguous channel range (the
sharding bench.py uses on the GPU box), gathering their audio to rank 0.  The per-rank chain
here is the CPU oracle (the checker; the GPU path is the same code with the HIP chain and
RCCL): rank 0's gathered result must equal one process running all channels, bit for bit."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
import uhsdr_amd as U
from uhsdr_amd import shard, synth

PER_RANK, FRAMES = 6, 256


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = shard.channel_range(PER_RANK, rank)
    plan = U.build_plan(U.default_config())
    iq = synth.ssb_iq(np.arange(lo, hi), 0, FRAMES)
    orx = oracle.OracleRx(plan, hi - lo)
    res = {}

    def step(k):
        res["a1"], _ = orx.process(iq)
    # bench.py's timed region (barrier + sync brackets, max-over-ranks seconds): rank 1 sleeps,
    # so the reduced time must cover its sleep on every rank
    import time
    el = shard.timed_loop(step, lambda: time.sleep(0.2 if rank == 1 else 0.0), 1, 0, dist, world, "cpu")
    assert el >= 0.2
    full = shard.gather_to_root(torch.from_numpy(res["a1"]), dist, world, rank)
    if rank == 0:
        np.save(out_path, full.numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_shard_and_gather(tmp_path):
    world = 2
    out = str(tmp_path / "gathered.npy")
    mp.start_processes(_rank_main, args=(world, _free_port(), out), nprocs=world, start_method="spawn")
    got = np.load(out)
    plan = U.build_plan(U.default_config())
    iq = synth.ssb_iq(np.arange(world * PER_RANK), 0, FRAMES)
    ref, _ = oracle.OracleRx(plan, world * PER_RANK).process(iq)
    assert got.shape == ref.shape
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


STEPS = 5


def _pipe_main(rank, world, port, out_path):
    """shard.GatherPipeline (bench.py's N > 1 gather leg) over gloo: every step's blocks
    arrive at rank 0 in step order and rank order, and no buffer is overwritten while its
    gather is in flight (each step writes distinct data into a reused double buffer)."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = shard.channel_range(PER_RANK, rank)
    plan = U.build_plan(U.default_config())
    orx = oracle.OracleRx(plan, hi - lo)
    got = {}

    def sink(step, parts):
        got[step] = torch.cat([p.clone() for p in parts], dim=0).numpy()

    pipe = shard.GatherPipeline(dist, world, rank, lambda: torch.empty((hi - lo, FRAMES), dtype=torch.float32),
                                depth=2, sink=sink)
    for s in range(STEPS):
        def compute(out, s=s):
            a1, _ = orx.process(synth.ssb_iq(np.arange(lo, hi), s * FRAMES, FRAMES))
            out.copy_(torch.from_numpy(a1))
        pipe.step(compute)
    pipe.drain()
    if rank == 0:
        assert sorted(got) == list(range(STEPS)), sorted(got)
        np.save(out_path, np.concatenate([got[s] for s in range(STEPS)], axis=1))
    dist.barrier()
    dist.destroy_process_group()


def test_gather_pipeline_overlapped_order(tmp_path):
    world = 2
    out = str(tmp_path / "piped.npy")
    mp.start_processes(_pipe_main, args=(world, _free_port(), out), nprocs=world, start_method="spawn")
    got = np.load(out)
    plan = U.build_plan(U.default_config())
    iq = synth.ssb_iq(np.arange(world * PER_RANK), 0, STEPS * FRAMES)
    ref, _ = oracle.OracleRx(plan, world * PER_RANK).process(iq)
    assert got.shape == ref.shape
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


def test_gather_pipeline_single_rank():
    seen = []
    pipe = shard.GatherPipeline(None, 1, 0, lambda: torch.zeros(2), sink=lambda s, p: seen.append((s, p[0].clone())))
    for s in range(3):
        pipe.step(lambda out, s=s: out.fill_(s))
    pipe.drain()
    assert [s for s, _ in seen] == [0, 1, 2] and [float(p[0]) for _, p in seen] == [0.0, 1.0, 2.0]


@pytest.mark.parametrize("total,world", [(10, 3), (4096, 8), (7, 8)])
def test_split_range_covers(total, world):
    ranges = [shard.split_range(total, world, r) for r in range(world)]
    assert ranges[0][0] == 0 and ranges[-1][1] == total
    for (a, b), (c, d) in zip(ranges, ranges[1:]):
        assert b == c and b - a >= d - c
