"""The N > 1 path with the product chain: two ranks (one process each, as bench.py --gpus 2
launches them) share the box's one GPU, each running the HIP chain (libuhsdr_amd.so) on its
own contiguous channel shard; bench.py's shard.timed_loop brackets the steps and
shard.GatherPipeline gathers every step's audio to rank 0 while the next step computes.
Rank 0's gathered stream must equal the CPU oracle over all channels, bit for bit.

The process group is gloo (a single GPU cannot host two RCCL ranks), so the gathered buffers
are host copies; the sharding, ordering and buffer reuse are the code bench.py runs over RCCL."""
import os
import socket

import numpy as np
import pytest

import oracle
import uhsdr_amd as U
from uhsdr_amd import shard, synth

pytestmark = pytest.mark.gpu

PER_RANK, FRAMES, STEPS = 130, 256, 4


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, out_path):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    lo, hi = shard.channel_range(PER_RANK, rank)
    chain = U.RxChain(U.default_config(), channels=hi - lo, frames=FRAMES)
    inputs = [torch.from_numpy(synth.ssb_iq(np.arange(lo, hi), s * FRAMES, FRAMES)).cuda() for s in range(STEPS)]
    dev_out = torch.empty((hi - lo, FRAMES), dtype=torch.float32, device="cuda")
    got = {}

    def sink(step, parts):
        got[step] = torch.cat([p.clone() for p in parts], dim=0).numpy()

    pipe = shard.GatherPipeline(dist, world, rank, lambda: torch.empty((hi - lo, FRAMES), dtype=torch.float32),
                                depth=2, sink=sink)
    state = {"s": 0}

    def compute(out):
        chain.process(inputs[state["s"]], dev_out, None)
        out.copy_(dev_out.cpu())
        state["s"] += 1

    el = shard.gather_timed(pipe, compute, torch.cuda.synchronize, STEPS, 0, dist, "cpu")
    chain.close()
    if rank == 0:
        assert el > 0
        assert sorted(got) == list(range(STEPS)), sorted(got)
        np.save(out_path, np.concatenate([got[s] for s in range(STEPS)], axis=1))
    dist.barrier()
    dist.destroy_process_group()


def test_two_ranks_hip_chain_sharded_and_gathered(cuda, tmp_path):
    import torch.multiprocessing as mp
    world = 2
    out = str(tmp_path / "gathered.npy")
    mp.start_processes(_rank_main, args=(world, _free_port(), out), nprocs=world, start_method="spawn")
    got = np.load(out)
    plan = U.build_plan(U.default_config())
    iq = synth.ssb_iq(np.arange(world * PER_RANK), 0, STEPS * FRAMES)
    ref, _ = oracle.OracleRx(plan, world * PER_RANK).process(iq, threads=8)
    assert got.shape == ref.shape
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
