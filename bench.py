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
import time

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


def algorithmic_bytes(plan, C: int, N: int, write_dst: bool):
    """Bytes each kernel must move per launch, from the live state sizes."""
    M = plan.decimation_rate
    Nd = N // M
    if plan.use_decimated_iq:
        fir_hist = 2 * (plan.dec_taps - 1) + 2 * (plan.hilbert_taps - 1)
    else:
        fir_hist = 2 * (plan.hilbert_taps - 1) + (plan.dec_taps - 1)
    if plan.iq_auto_correction:
        fir_hist += 3
    back_state = (plan.pre_stages + plan.aa_stages + 16 + 4 + max(plan.interp_phase - 1, 0)
                  + plan.agc.attack_buffsize + 9)
    out_b = 4 + (8 if write_dst else 0)
    front = C * (8 * N + 4 * Nd + 2 * 4 * fir_hist)
    back = C * (4 * Nd + out_b * N + 2 * 4 * back_state)
    chain = C * ((8 + out_b) * N + 2 * 4 * (fir_hist + back_state))   # adec round trip excluded
    return {"rx_front": front, "rx_back": back, "chain": chain,
            "s_live_bytes": 4 * (fir_hist + back_state)}


def cpu_baseline(plan, frames: int, budget_s: float = 10.0):
    import oracle
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    threads = max(1, min(threads, 64))
    from uhsdr_amd import synth
    C = 32 * threads
    o = oracle.OracleRx(plan, C)
    blocks = [synth.ssb_iq(np.arange(C), k * frames, frames) for k in range(4)]
    o.process(blocks[0], threads=threads)          # warm-up
    done, t0 = 0, time.perf_counter()
    while True:
        o.process(blocks[done % 4], threads=threads)
        done += 1
        el = time.perf_counter() - t0
        if el >= budget_s or done >= 100000:
            break
    samples = C * frames * done
    import platform
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        model = platform.processor()
    return {"value": round(samples / el / 1e6, 3), "unit": "Msamples/s", "cores": threads, "kind": "port",
            "sample": f"{C} channels x {done} blocks of {frames} frames ({samples} samples, {el:.1f} s) "
                      f"through oracle/uhsdr_oracle.c (bit-exact to the reference build), "
                      f"{threads} threads, channels split evenly; host CPU: {model}"}


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
    ap.add_argument("--cpu-budget", type=float, default=10.0)
    ap.add_argument("--pool", type=int, default=8, help="distinct input blocks cycled through")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    import uhsdr_amd as U
    from uhsdr_amd import synth

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    wl = WORKLOADS[args.workload]
    C = args.channels or wl["channels"]
    N = args.frames or wl["frames"]
    cfg = U.default_config()
    stream = torch.cuda.current_stream(dev)
    chain = U.RxChain(cfg, channels=C, frames=N, stream=stream.cuda_stream)
    plan = chain.plan

    # inputs resident in HBM before timing: a pool of consecutive blocks, cycled
    pool = max(1, args.pool)
    inputs = [synth.ssb_iq_torch(rank * C, C, k * N, N, dev) for k in range(pool)]
    audio = torch.empty((C, N), dtype=torch.float32, device=dev)
    dst = torch.empty((C, N, 2), dtype=torch.int32, device=dev) if args.dst else None
    torch.cuda.synchronize(dev)

    for s in range(args.warmup):
        chain.process(inputs[s % pool], audio, dst)
    torch.cuda.synchronize(dev)

    chain.enable_timing(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for s in range(args.steps):
        chain.process(inputs[s % pool], audio, dst)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ktimes = chain.kernel_times()
    chain.enable_timing(False)

    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())

    ok = bool(torch.isfinite(audio).all().item())
    if rank != 0:
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return

    total_samples = world * C * N * args.steps
    value = total_samples / elapsed / 1e6
    ab = algorithmic_bytes(plan, C, N, args.dst)
    kms = {k: v[0] / max(v[1], 1) for k, v in ktimes.items()}       # mean ms per launch
    dominant = max(kms, key=kms.get)
    achieved = ab[dominant] / (kms[dominant] * 1e-3) / 1e9
    chain_dev_ms = sum(kms.values())
    roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                "kernel": dominant, "alg_bytes_per_launch": ab[dominant],
                "mean_launch_ms": round(kms[dominant], 5)}
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
                   "outputs": "f32 audio" + (" + int32 codec frames" if args.dst else "")},
        "roofline": roofline,
        "chain": {"device_ms_per_step": round(chain_dev_ms, 5),
                  "kernel_ms": {k: round(v, 5) for k, v in kms.items()},
                  "alg_bytes_per_sample": round(ab["chain"] / (C * N), 2),
                  "s_live_bytes_per_channel": ab["s_live_bytes"],
                  "hbm_frac": round(chain_gbs / HBM_PEAK_GBS, 4),
                  "fp32_ops_note": "see DESIGN.md: the chain is VALU-bound at this size"},
        "outputs_finite": ok,
    }
    if not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline(plan, N, args.cpu_budget)
    print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
