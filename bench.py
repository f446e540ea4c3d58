#!/usr/bin/env python3
"""Throughput of the batched UHSDR SSB-RX chain on MI355X (BASELINE.json metric).

    python bench.py [--gpus N --steps K --warmup W] [--workload c2|northstar]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

A step = one uhsdr_rx_process() call: every channel of this rank advances by one block of
`frames` 48 kHz I/Q frames through the full reference RX chain (audio_driver.c:2603-2942:
I/Q convert, Fs/4 shift, 89-tap Hilbert pair, USB sum, 43-tap /4 decimator, 10-stage
lattice, WDSP AGC, biquads, interpolator, 6-stage anti-alias lattice, treble shelf, line-out
scale), with inputs resident in HBM.  Ranks own disjoint channel ranges (weak scaling, no
collective on the data path).  value = complex input samples of all ranks / max-rank time.

Also reported: per-kernel device time from HIP events recorded on the library's stream over
the timed region, the HBM roofline of the dominant kernel (algorithmic bytes per launch /
mean launch time vs 8 TB/s), and the CPU oracle's throughput on the host (baseline only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E peak (MI355X_MICROARCH.md, chip table)
WORKLOADS = {
    # BASELINE.json configs[1]: 4096 channels x 256-sample blocks, SSB-RX chain f32, 1 GPU
    "c2": dict(channels=4096, frames=256, desc="C2: 4096 ch x 256-frame blocks, SSB-USB P48 chain, f32"),
    # north_star target regime: >= 1M concurrent 64-sample I/Q blocks per GPU
    "northstar": dict(channels=1048576, frames=64, desc="1048576 ch x 64-frame blocks, SSB-USB P48 chain, f32"),
}


NS_STEPS = 100   # north-star leg: timed calls (~80 ms of device time; 20 left the first-call ramp in the mean)
AGC_Q = 6   # AGC look-ahead ring: the last 6 calls of AGC inputs (uhsdr_rx.hip, rx_back_agc)


def algorithmic_bytes(plan, C: int, N: int, write_dst: bool):
    """Bytes each kernel must move per launch, from the live state sizes.

    Per channel and launch: the I/Q frames in (8 B/frame), f32 audio out (4 B/frame, +8 B for
    int32 codec frames), every persistent state word read once and written once, except the
    AGC look-ahead ring, of which a launch reads and rewrites only the Nd decimated samples it
    advances.  The decimated hand-off between the two kernels (adec) counts for the kernels
    but not for the chain: it is an artefact of the split, not of the algorithm.
    """
    M = plan.decimation_rate
    Nd = N // M
    if plan.use_decimated_iq:
        fir_hist = 2 * (plan.dec_taps - 1) + 2 * (plan.hilbert_taps - 1)
    else:
        fir_hist = 2 * (plan.hilbert_taps - 1) + (plan.dec_taps - 1)
    if plan.iq_auto_correction:
        fir_hist += 3
    # lattice pre/aa, biquad_1/2 state, interpolator history, 5 AGC floats, 5 call maxima,
    # the leaving sample, 3 AGC ints
    back_state = (plan.pre_stages + plan.aa_stages + 16 + 4 + max(plan.interp_phase - 1, 0)
                  + 5 + (AGC_Q - 1) + 1 + 3)
    ring = 2 * 4 * Nd if plan.agc.mode != 5 else 0
    out_b = 4 + (8 if write_dst else 0)
    front = C * (8 * N + 4 * Nd + 2 * 4 * fir_hist)
    back = C * (4 * Nd + out_b * N + 2 * 4 * back_state + ring)
    chain = C * ((8 + out_b) * N + 2 * 4 * (fir_hist + back_state) + ring)
    s_live = 4 * (fir_hist + back_state + (AGC_Q * (BLK // M) if plan.agc.mode != 5 else 0))
    # rx_chain (one kernel per call, the hand-off in LDS) moves exactly the chain's bytes
    return {"rx_front": front, "rx_back": back, "rx_chain": chain, "chain": chain,
            "s_live_bytes": s_live}


BLK = 32


def pmc_traffic(workload: str):
    """HBM bytes per launch per kernel from the committed rocprofv3 PMC summary of this
    workload (profiles/pmc_<workload>.json, tools/pmc_summary.py: FETCH_SIZE x 2 per the gfx950
    correction of MI355X_MICROARCH.md §HBM, + WRITE_SIZE), or None."""
    f = os.path.join(ROOT, "profiles", f"pmc_{workload}.json")
    try:
        d = json.load(open(f))
    except (OSError, ValueError):
        return None
    out = {}
    for k, v in d.items():
        if "hbm_read_bytes_corrected" in v and "hbm_write_bytes" in v:
            out[k] = v["hbm_read_bytes_corrected"] + v["hbm_write_bytes"]
    return out or None


def host_cpus():
    """CPUs this process may run on (its affinity mask), and the host CPU model."""
    try:
        cpus = len(os.sched_getaffinity(0))
    except AttributeError:
        cpus = os.cpu_count() or 1
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return cpus, model


def cpu_baseline(plan, frames: int, budget_s: float = 10.0):
    """The bit-exact CPU restatement (oracle/uhsdr_oracle.c) on the host cores (SURVEY.md
    §8(d) d4): one persistent worker thread per CPU, pinned (sched affinity), channels split
    evenly, no thread creation inside the timed loop.  Threads = the CPUs of this process's
    affinity mask, capped by OMP_NUM_THREADS when the box sets it (the GPU box's per-GPU CPU
    share)."""
    import oracle
    from uhsdr_amd import synth
    cpus, model = host_cpus()
    cap = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    threads = max(1, min(cpus, cap) if cap > 0 else cpus)
    C = 16 * threads
    blocks = np.stack([synth.ssb_iq(np.arange(C), k * frames, frames) for k in range(4)])
    oracle.rx_bench(plan, blocks, threads, 0.5)                 # warm-up (pages, caches, clocks)
    done, el = oracle.rx_bench(plan, blocks, threads, budget_s)
    samples = done * frames
    return {"value": round(samples / el / 1e6, 3), "unit": "Msamples/s", "cores": threads, "kind": "port",
            "sample": f"{C} channels x {frames}-frame calls, {done // C} calls per channel on average "
                      f"({samples} samples, {el:.1f} s) through oracle/uhsdr_oracle.c (bit-exact to the "
                      f"reference build); {threads} persistent worker threads pinned one per CPU "
                      f"(affinity mask has {cpus} CPUs), channels split evenly; host CPU: {model}"}


SCHEDULES = {"auto": None, "pipe": 1, "fused": 2, "chain": 3}   # uhsdr_rx_set_schedule
DEVICE_HANDOFF = 3       # --handoff: uhsdr_rx_set_pipelined's mode (event 1, device 2, persistent 3)
SCHEDULE_NAMES = {1: "split_pipe", 2: "split_fused", 3: "chain"}


def timed_run(U, synth, shard, torch, dist, dev, world, rank, C, N, steps, warmup, pool, want_dst, pipelined=False,
              precision=0, schedule=None, front_block=0, reduce_dev=None, board=0, ensure_dist=None):
    """W untimed + K timed steps of one RxChain on this rank; returns (max-rank seconds,
    per-kernel (total ms, launches) from HIP events on the library's stream, plan, finite, schedule,
    device hand-off give-ups after the timed loop (uhsdr_rx_handoff_timeouts; 0 required))."""
    cfg = U.default_config(board=board)
    stream = torch.cuda.current_stream(dev)
    chain = U.RxChain(cfg, channels=C, frames=N, stream=stream.cuda_stream, schedule=schedule)
    chain.set_precision(precision)
    if front_block:
        chain.set_front_block(front_block)
    sched = SCHEDULE_NAMES.get(chain.schedule, str(chain.schedule))
    if pipelined:
        # call k+1's rx_front overlaps call k's rx_back; 2: the device hand-off (rx_back polls the
        # arrival counters the front waves of its channel group bump, then reads the hand-off with
        # sc1 loads, instead of waiting on a cross-stream event)
        chain.set_pipelined(DEVICE_HANDOFF)
    if ensure_dist is not None:
        ensure_dist()                                  # the process group after the side stream
    plan = chain.plan
    # inputs resident in HBM before timing: a pool of consecutive blocks, cycled
    c0 = shard.channel_range(C, rank)[0]          # weak scaling: rank r owns channels [r*C, (r+1)*C)
    inputs = [synth.ssb_iq_torch(c0, C, k * N, N, dev) for k in range(pool)]
    audio = torch.empty((C, N), dtype=torch.float32, device=dev)
    dst = torch.empty((C, N, 2), dtype=torch.int32, device=dev) if want_dst else None
    torch.cuda.synchronize(dev)
    # throughput: K calls with nothing but the calls themselves inside the timed region
    # (shard.timed_loop: warm-up, barrier + sync brackets, max over ranks)
    # every buffer set validated once (RxChain.bind), so a step is one ctypes call
    ptrs = [chain.bind(x, audio, dst) for x in inputs]
    elapsed = shard.timed_loop(lambda s: chain.process_ptr(ptrs[s % pool]),
                               lambda: torch.cuda.synchronize(dev), steps, warmup, dist, world,
                               dev if reduce_dev is None else reduce_dev)
    # the device hand-off's failure contract (include/uhsdr.h): a poll that gave up poisons its call
    # and sets the handle's failure word; the timed calls count only if none did
    timeouts = chain.handoff_timeouts()
    # per-kernel breakdown in a separate pass: HIP events on the library's own stream bracket
    # every kernel of every call (the records cost host time, so they never share a clock with
    # the throughput loop above)
    tsteps = max(10, min(steps, 200))
    if pipelined:
        # serial for the event pass: with call k+1's rx_front overlapping call k's rx_back the
        # events of each kernel would include the other's time
        chain.set_pipelined(False)
    chain.enable_timing(True, every=1)
    for s in range(tsteps):
        chain.process(inputs[s % pool], audio, dst)
    torch.cuda.synchronize(dev)
    ktimes = chain.kernel_times()
    chain.enable_timing(False)
    ok = bool(torch.isfinite(audio).all().item())
    chain.close()
    del inputs
    return elapsed, ktimes, plan, ok, sched, timeouts


def gather_run(U, synth, shard, torch, dist, dev, world, rank, C, N, steps, warmup, backend="nccl", pool=4, sink=None,
               always_collective=False):
    """The same chain with every launch's f32 audio gathered to rank 0
    through shard.GatherPipeline: double-buffered outputs, the gather of launch k (RCCL
    grouped send/recv over xGMI, rank 0 receiving from every peer on its own link) in flight
    while launch k+1 computes.  Step s processes the rank's block s % pool of consecutive
    48 kHz blocks.  With the gloo test hook the device audio is copied to host buffers and
    those are gathered.  `sink(step, parts)` (rank 0) sees every step's per-rank blocks in
    step order.  `always_collective`: issue the gather even on a one-rank group (the RCCL leg's
    readiness test on a one-GPU box).  Returns max-rank seconds for `steps` steps."""
    cfg = U.default_config()
    comp = torch.cuda.current_stream(dev)
    chain = U.RxChain(cfg, channels=C, frames=N, stream=comp.cuda_stream)
    c0 = shard.channel_range(C, rank)[0]
    xs = [synth.ssb_iq_torch(c0, C, k * N, N, dev) for k in range(pool)]
    host = backend != "nccl"
    dev_out = torch.empty((C, N), dtype=torch.float32, device=dev) if host else None
    pipe = shard.GatherPipeline(dist, world, rank,
                                lambda: torch.empty((C, N), dtype=torch.float32, device="cpu" if host else dev),
                                sink=sink, always=always_collective)
    st = {"s": 0}

    def compute(out):
        x = xs[st["s"] % pool]
        st["s"] += 1
        if host:
            chain.process(x, dev_out, None)
            out.copy_(dev_out.cpu())
        else:
            chain.process(x, out, None)
    t = shard.gather_timed(pipe, compute, lambda: torch.cuda.synchronize(dev), steps, warmup, dist,
                           "cpu" if host else dev)
    chain.close()
    return t


def roofline_of(ab, ktimes, traffic):
    kms = {k: v[0] / max(v[1], 1) for k, v in ktimes.items()}       # mean ms per launch
    dominant = max(kms, key=kms.get)
    achieved = ab[dominant] / (kms[dominant] * 1e-3) / 1e9
    roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": int(traffic[dominant]) if traffic and dominant in traffic else None,
            "kernel": dominant, "alg_bytes_per_launch": ab[dominant],
            "mean_launch_ms": round(kms[dominant], 5)}
    return roof, kms


def launch_ranks(n: int) -> int:
    """`bench.py --gpus N` with no WORLD_SIZE in the environment: run N ranks of this same
    command line as children of torch.distributed.run (one process per GPU, RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_* in their environment) and return its exit code.  Called before
    anything in this process imports torch.cuda state or touches HIP, and the children are
    started as child processes (never an exec of this one)."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--workload", default="c2", choices=sorted(WORKLOADS))
    ap.add_argument("--channels", type=int, default=0, help="override channels per GPU")
    ap.add_argument("--frames", type=int, default=0, help="override frames per call")
    ap.add_argument("--dst", action="store_true", help="also write int32 codec frames")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--no-northstar", action="store_true", help="skip the 1M-channel north-star leg")
    ap.add_argument("--no-gather", action="store_true", help="skip the RCCL gather leg (N > 1)")
    ap.add_argument("--cpu-budget", type=float, default=10.0)
    ap.add_argument("--serial", action="store_true",
                    help="run rx_front and rx_back of a call back to back on one stream instead of the "
                         "default pipelined mode (uhsdr_rx_set_pipelined: call k+1's rx_front overlaps "
                         "call k's rx_back); the 1M-channel north-star leg always runs serial (both "
                         "kernels fill the chip there)")
    ap.add_argument("--pipelined", action="store_true",
                    help="pipelined mode even on the north-star workload (default on for the others)")
    ap.add_argument("--handoff", default="persistent", choices=["event", "device", "persistent"],
                    help="pipelined mode's front -> back hand-off: the persistent back end (uhsdr_rx_set_"
                         "pipelined 3, the default: one rx_back launch runs call after call, taking each "
                         "call the host grants), rx_back per call polling the arrival counters its channel "
                         "group's front waves bump (2: no cross-stream wait per call), or a cross-stream "
                         "event per call (1; for profilers that serialise dispatches)")
    ap.add_argument("--precision", default="exact", choices=["exact", "fma"],
                    help="FIR MACs: exact (bit-identical to the reference) or fma (1e-5 normwise)")
    ap.add_argument("--pool", type=int, default=8, help="distinct input blocks cycled through")
    ap.add_argument("--board", default="ovi40", choices=["ovi40", "mchf"],
                    help="the board's output stage (uhsdr_rx_config.board); the headline is OVI40's")
    ap.add_argument("--schedule", default="auto", choices=sorted(SCHEDULES),
                    help="kernel schedule of a call (uhsdr_rx_set_schedule); auto: the library's choice "
                         "(rx_front + rx_back_fused from 131072 channels on, else rx_front + the back-end wave "
                         "pipeline; rx_chain only when asked for)")
    ap.add_argument("--front-block", type=int, default=0, choices=[0, 8, 16],
                    help="FIR outputs per lane of rx_front (uhsdr_rx_set_front_block; 0: the library default)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="process group of an N > 1 run: nccl (= RCCL over xGMI, one GPU per rank) or gloo "
                         "(test hook: ranks may share one GPU, the gather leg moves host copies)")
    args = ap.parse_args()
    global DEVICE_HANDOFF
    DEVICE_HANDOFF = {"event": 1, "device": 2, "persistent": 3}[args.handoff]

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))

    import torch
    import torch.distributed as dist
    import uhsdr_amd as U
    from uhsdr_amd import shard, synth

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE is {world}", file=sys.stderr)
        sys.exit(2)
    if args.dist_backend == "nccl":
        dev = torch.device("cuda", local)
    else:
        # gloo test hook: ranks may outnumber the GPUs of the box and share them
        dev = torch.device("cuda", local % max(1, torch.cuda.device_count()))
    torch.cuda.set_device(dev)

    def ensure_dist():
        # after the C2 handle has made its side stream (timed_run): the persistent back end waits in
        # its launch for fronts enqueued later on the handle's stream, so the side stream must not share
        # a hardware queue with it; made before RCCL's streams, it takes a queue of its own
        if world > 1 and not dist.is_initialized():
            if args.dist_backend == "nccl":
                dist.init_process_group("nccl", device_id=dev)
            else:
                dist.init_process_group("gloo")

    reduce_dev = dev if args.dist_backend == "nccl" else "cpu"

    prec = U.PRECISION_FMA if args.precision == "fma" else U.PRECISION_EXACT
    wl = WORKLOADS[args.workload]
    C = args.channels or wl["channels"]
    N = args.frames or wl["frames"]
    pipelined = args.pipelined or (not args.serial and args.workload != "northstar")
    elapsed, ktimes, plan, ok, sched, timeouts = timed_run(U, synth, shard, torch, dist, dev, world, rank, C, N, args.steps,
                                                 args.warmup, max(1, args.pool), args.dst, pipelined, prec,
                                                 SCHEDULES[args.schedule], args.front_block, reduce_dev,
                                                 U.BOARD_MCHF if args.board == "mchf" else U.BOARD_OVI40,
                                                 ensure_dist=ensure_dist)
    ensure_dist()

    gather = None
    if world > 1 and not args.no_gather:
        gs = max(10, args.steps // 4)
        gt = gather_run(U, synth, shard, torch, dist, dev, world, rank, C, N, gs, 5, args.dist_backend)
        gather = {"value": round(world * C * N * gs / gt / 1e6, 2), "unit": "Msamples/s", "steps": gs,
                  "ms_per_step": round(gt / gs * 1e3, 5),
                  "backend": args.dist_backend,
                  "how": ("every launch's f32 audio gathered to rank 0 (torch.distributed.gather = grouped RCCL "
                          "send/recv over xGMI) on a comm stream, overlapped with the next launch (double-buffered)"
                          if args.dist_backend == "nccl" else
                          "gloo test hook: every launch's audio copied to host and gathered to rank 0 over gloo")}

    def north_star_leg(precision):
        nw = WORKLOADS["northstar"]
        n_el, n_kt, n_plan, n_ok, n_sched, n_tmo = timed_run(U, synth, shard, torch, dist, dev, 1, 0, nw["channels"],
                                                      nw["frames"], NS_STEPS, 10, 3, False, False, precision)
        n_ab = algorithmic_bytes(n_plan, nw["channels"], nw["frames"], False)
        n_roof, n_kms = roofline_of(n_ab, n_kt, pmc_traffic("northstar" if precision == U.PRECISION_EXACT
                                                            else "northstar_fma"))
        n_dev = sum(n_kms.values())
        return {"workload": nw["desc"], "value": round(nw["channels"] * nw["frames"] * NS_STEPS / n_el / 1e6, 2),
                "unit": "Msamples/s", "steps": NS_STEPS, "ms_per_step": round(n_el / NS_STEPS * 1e3, 5), "roofline": n_roof,
                "kernel_ms": {k: round(v, 5) for k, v in n_kms.items()},
                # the chain's algorithmic bytes over the wall clock of a step (everything between
                # the kernels included), and over the sum of the kernels' own event times
                "chain_hbm_frac": round(n_ab["chain"] / n_el * NS_STEPS / 1e9 / HBM_PEAK_GBS, 4),
                "chain_hbm_frac_kernel_events": round(n_ab["chain"] / (n_dev * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                "alg_bytes_per_sample": round(n_ab["chain"] / (nw["channels"] * nw["frames"]), 2),
                "schedule": n_sched, "outputs_finite": n_ok, "handoff_timeouts": n_tmo}

    ns = None
    if world == 1 and not args.no_northstar and args.workload != "northstar" and not (args.channels or args.frames):
        ns = north_star_leg(prec)
        ns["precision"] = args.precision
        if prec == U.PRECISION_EXACT:
            # the same workload with fused FIR MACs (uhsdr_rx_set_precision FMA): within 1e-5
            # normwise of the reference on this path (tests/test_gpu_fma.py), not bit-identical
            ns["fma"] = north_star_leg(U.PRECISION_FMA)
            ns["fma"]["precision"] = "fma"

    if rank != 0:
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return

    total_samples = world * C * N * args.steps
    value = total_samples / elapsed / 1e6
    ab = algorithmic_bytes(plan, C, N, args.dst)
    roofline, kms = roofline_of(ab, ktimes, pmc_traffic(args.workload) if not (args.channels or args.frames) else None)
    chain_dev_ms = sum(kms.values())
    chain_gbs = ab["chain"] / (chain_dev_ms * 1e-3) / 1e9
    out = {
        "metric": "Msamples/s through full SSB-RX chain (node); % of HBM-roofline per GPU",
        "value": round(value, 2), "unit": "Msamples/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 5),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic (two-tone SSB + noise at +12 kHz, per-channel random tones)",
        "config": {"workload": wl["desc"] if not (args.channels or args.frames) else
                   f"{C} ch x {N}-frame blocks, SSB-USB P48 chain, f32",
                   "channels_per_gpu": C, "frames_per_call": N, "filter_path": int(plan.filter_path),
                   "parallelism": f"channel-sharded x{world}, no data-path collective",
                   "outputs": "f32 audio" + (" + int32 codec frames" if args.dst else ""),
                   "pipelined": pipelined, "handoff": args.handoff if pipelined else None,
                   "precision": args.precision, "schedule": sched,
                   **({"board": "mchf"} if args.board == "mchf" else {})},
        "roofline": roofline,
        "chain": {"device_ms_per_step": round(chain_dev_ms, 5),
                  "kernel_ms": {k: round(v, 5) for k, v in kms.items()},
                  "alg_bytes_per_sample": round(ab["chain"] / (C * N), 2),
                  "s_live_bytes_per_channel": ab["s_live_bytes"],
                  "hbm_frac": round(ab["chain"] / (elapsed / args.steps) / 1e9 / HBM_PEAK_GBS, 4),
                  "hbm_frac_kernel_events": round(chain_gbs / HBM_PEAK_GBS, 4),
                  "note": "C2 (4096 channels) is latency-bound: one lane per channel for the recursive "
                          "stages leaves most of the 256 CUs idle; see DESIGN.md and north_star"
                          + ("; pipelined: rx_front of the next call overlaps rx_back in the timed loop; the "
                             "kernel event times come from a separate serial pass" if pipelined else "")},
        "outputs_finite": ok,
        "handoff_timeouts": timeouts,
    }
    if ns:
        out["north_star"] = ns
    if gather:
        out["with_gather"] = gather
    if not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline(plan, N, args.cpu_budget)
    print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if timeouts or (ns and (ns["handoff_timeouts"] or ns.get("fma", {}).get("handoff_timeouts"))):
        print("bench.py: a device hand-off poll gave up during the timed loop (handoff_timeouts != 0): "
              "the measurement is invalid", file=sys.stderr)
        sys.exit(3)


if __name__ == "__main__":
    main()
