#!/usr/bin/env python3
"""Spectrum display kernel timing (C3: 32768 channels, 1024-point frames).

    python tools/bench_spectrum.py [--channels C --frames N --fft 1024 --steps K --outputs avg|both|none]

Prints one JSON line: Msamples/s, ms per call and HBM GB/s of the algorithmic bytes
(8 B I/Q in + 4 B per output array per sample + average state read/write once per call)."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--channels", type=int, default=32768)
    ap.add_argument("--frames", type=int, default=4096)
    ap.add_argument("--fft", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--outputs", default="avg", choices=["avg", "both", "none"])
    ap.add_argument("--auto", type=int, default=0)
    a = ap.parse_args()
    import torch
    import uhsdr_amd as U
    from uhsdr_amd import synth
    C, N = a.channels, a.frames
    s = torch.cuda.current_stream()
    spec = U.Spectrum(U.default_spectrum_config(fft_len=a.fft, iq_auto_correction=a.auto), channels=C, frames=N,
                      stream=s.cuda_stream)
    iq = synth.ssb_iq_torch(0, C, 0, N, "cuda")
    avg = torch.empty(spec.out_shape, dtype=torch.float32, device="cuda") if a.outputs != "none" else None
    mag = torch.empty(spec.out_shape, dtype=torch.float32, device="cuda") if a.outputs == "both" else None
    for _ in range(a.warmup):
        spec.process(iq, mag, avg)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(a.steps):
        spec.process(iq, mag, avg)
    e1.record(s)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.steps
    nout = {"avg": 1, "both": 2, "none": 0}[a.outputs]
    L = a.fft
    byts = C * N * (8 + 4 * nout) + C * L * 8 + (C * 3 * 8 if a.auto else 0)
    print(json.dumps({"workload": f"spectrum {C} ch x {N} frames, {L}-point, outputs={a.outputs}, auto={a.auto}",
                      "ms_per_call": round(ms, 4), "msamples_per_s": round(C * N / ms / 1e3, 1),
                      "frames_per_s": round(C * N / L / ms * 1e3, 1),
                      "alg_gbps": round(byts / ms / 1e6, 1), "hbm_frac": round(byts / ms / 1e6 / 8000, 4)}))
    spec.close()


if __name__ == "__main__":
    main()
