"""bench.py's own N > 1 entry.

1. `python bench.py --gpus 2 ...` with no WORLD_SIZE in the environment must start two ranks
   itself (torch.distributed.run children) and print one JSON line with n_gpus == 2.  The
   box has one GPU, so the ranks share it through the gloo test hook (--dist-backend gloo).
2. bench.gather_run -- the code of the bench's gather leg -- run by two spawned ranks: rank 0's
   gathered audio must equal the CPU oracle over both shards, bit for bit.  The inputs are the
   bench's device-generated blocks (synth.ssb_iq_torch), copied to the host for the oracle.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import oracle
import uhsdr_amd as U
from uhsdr_amd import shard, synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu

PER_RANK, FRAMES, STEPS = 130, 256, 5


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _bench_env():
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    return env


def _last_json(out: str):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


def test_bench_gpus2_launches_two_ranks(cuda):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "4", "--warmup", "1",
           "--no-northstar", "--no-cpu", "--dist-backend", "gloo"]
    r = subprocess.run(cmd, env=_bench_env(), cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    d = _last_json(r.stdout)
    assert d["n_gpus"] == 2
    assert d["steps"] == 4 and d["outputs_finite"]
    assert np.isfinite(d["value"]) and d["value"] > 0
    assert d["with_gather"]["backend"] == "gloo" and d["with_gather"]["value"] > 0
    # whole-job value counts both ranks' samples over the max-rank time
    per_call = 2 * d["config"]["channels_per_gpu"] * d["config"]["frames_per_call"]
    assert abs(d["value"] - per_call / d["ms_per_step"] / 1e3) / d["value"] < 0.01


def test_bench_world_mismatch_fails():
    env = _bench_env()
    env.update(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--no-cpu"],
                       env=env, cwd=ROOT, capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "WORLD_SIZE" in r.stderr


def _gather_main(rank, world, port, out_path):
    import torch
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    import bench
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    got = {}

    def sink(step, parts):
        got[step] = torch.cat([p.clone() for p in parts], dim=0).numpy()

    el = bench.gather_run(U, synth, shard, torch, dist, dev, world, rank, PER_RANK, FRAMES, STEPS, 0,
                          backend="gloo", pool=STEPS, sink=sink)
    if rank == 0:
        assert el > 0
        assert sorted(got) == list(range(STEPS)), sorted(got)
        np.save(out_path, np.concatenate([got[s] for s in range(STEPS)], axis=1))
    dist.barrier()
    dist.destroy_process_group()


def test_bench_gather_run_bit_exact(cuda, tmp_path):
    import torch
    import torch.multiprocessing as mp
    world = 2
    out = str(tmp_path / "gathered.npy")
    mp.start_processes(_gather_main, args=(world, _free_port(), out), nprocs=world, start_method="spawn")
    got = np.load(out)
    C = world * PER_RANK
    # the bench's input blocks, generated on the device exactly as gather_run makes them
    iq = np.concatenate([np.concatenate([synth.ssb_iq_torch(r * PER_RANK, PER_RANK, k * FRAMES, FRAMES, cuda)
                                         .cpu().numpy() for r in range(world)], axis=0)
                         for k in range(STEPS)], axis=1)
    assert iq.shape == (C, STEPS * FRAMES, 2)
    ref, _ = oracle.OracleRx(U.build_plan(U.default_config()), C).process(iq, threads=8)
    assert got.shape == ref.shape
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


def _nccl_world1_main(rank, world, port, out_path):
    """bench.gather_run over a one-rank RCCL group with the collective forced on: device output
    buffers, dist.gather(async_op=True) on the process group's stream, Work.wait() ordering the
    compute stream -- the path the driver's N > 1 bench takes, on the one GPU of the box."""
    import torch
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    import bench
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    got = {}

    def sink(step, parts):
        assert len(parts) == 1 and parts[0].is_cuda
        got[step] = parts[0].clone().cpu().numpy()

    el = bench.gather_run(U, synth, shard, torch, dist, dev, world, rank, PER_RANK, FRAMES, STEPS, 0,
                          backend="nccl", pool=STEPS, sink=sink, always_collective=True)
    assert el > 0
    assert sorted(got) == list(range(STEPS)), sorted(got)
    np.save(out_path, np.concatenate([got[s] for s in range(STEPS)], axis=1))
    dist.barrier()
    dist.destroy_process_group()


def test_bench_gather_run_nccl_world1_bit_exact(cuda, tmp_path):
    """the RCCL gather leg executed on hardware (one rank, collective forced)."""
    import torch.multiprocessing as mp
    out = str(tmp_path / "gathered_nccl.npy")
    mp.start_processes(_nccl_world1_main, args=(1, _free_port(), out), nprocs=1, start_method="spawn")
    got = np.load(out)
    iq = np.concatenate([synth.ssb_iq_torch(0, PER_RANK, k * FRAMES, FRAMES, cuda).cpu().numpy()
                         for k in range(STEPS)], axis=1)
    ref, _ = oracle.OracleRx(U.build_plan(U.default_config()), PER_RANK).process(iq, threads=8)
    assert got.shape == ref.shape
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
