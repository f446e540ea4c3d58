#!/usr/bin/env python3
"""Per-GPU throughput of the BASELINE.json configs other than the headline C2 (which bench.py
measures): C3 (SAM P70 + 1024-point spectrum), C4's per-GPU share (FM-RX P1 and SSB-TX),
C5's per-GPU share (CW P4 with the CW decoder front end).

    python tools/bench_configs.py [--steps K] [--only c3,c4fm,c4tx,c5] > profiles/rNN_configs.jsonl

One JSON line per workload: Msamples/s of 48 kHz frames, ms per call, per-kernel device ms
(RX: HIP events on the library stream), algorithmic HBM bytes per frame and the fraction of
the 8 TB/s roofline they imply.  Inputs: 4096 distinct synthetic channels (uhsdr_amd.synth)
tiled over the batch, resident in HBM before timing.  C4 / C5 are 8-GPU configs; a GPU's
share is 1/8 of the channels (weak scaling: no data-path collective, bench.py --gpus N).
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0


def tiled(fn, C, N, distinct=4096):
    import numpy as np
    import torch
    d = min(C, distinct)
    base = fn(np.arange(d), 0, N)
    reps = (C + d - 1) // d
    t = torch.from_numpy(np.ascontiguousarray(base)).cuda()
    return t.repeat((reps,) + (1,) * (t.dim() - 1))[:C].contiguous()


def time_calls(fn, steps, warmup, join=None):
    """ms per call on the current stream; join() (pipelined handles) orders it after the side
    stream before the closing event"""
    import torch
    for _ in range(warmup):
        fn()
    if join:
        join()
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(steps):
        fn()
    if join:
        join()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / steps


FRONT_BLOCK = 0     # --front-block: the RX lines' front outputs per lane (0 = the library's choice)
HANDOFF = "persistent"  # --handoff: the pipelined RX lines' front -> back hand-off (uhsdr_rx_set_pipelined 3 / 2 / 1)


def rx_line(name, cfg, C, N, iq, steps, warmup, cw=False, pipelined=False):
    import torch
    import bench
    import uhsdr_amd as U
    s = torch.cuda.current_stream()
    chain = U.RxChain(cfg, channels=C, frames=N, stream=s.cuda_stream)
    if FRONT_BLOCK:
        chain.set_front_block(FRONT_BLOCK)
    if pipelined:
        chain.set_pipelined({"event": 1, "device": 2, "persistent": 3}[HANDOFF])
    audio = torch.empty((C, N), dtype=torch.float32, device="cuda")
    if cw:
        sig = torch.empty((C, N // 32), dtype=torch.uint8, device="cuda")
        en = torch.empty((C, max(1, chain.cw_blocks_max)), dtype=torch.float32, device="cuda")
        chain.set_cw_outputs(sig, en)
    join = chain.join if pipelined else None
    ms = time_calls(lambda: chain.process(iq, audio, None), steps, warmup, join)
    chain.enable_timing(True)
    time_calls(lambda: chain.process(iq, audio, None), steps, 0, join)
    kt = chain.kernel_times()
    chain.enable_timing(False)
    ab = bench.algorithmic_bytes(chain.plan, C, N, False)
    per = ab["chain"] / (C * N)
    out = {"workload": name, "channels": C, "frames_per_call": N, "pipelined": bool(pipelined), "ms_per_call": round(ms, 4),
           "msamples_per_s": round(C * N / ms / 1e3, 1),
           "kernel_ms": {k: round(v[0] / max(v[1], 1), 4) for k, v in kt.items()},
           "alg_bytes_per_frame": round(per, 2), "hbm_frac": round(C * N * per / ms / 1e6 / HBM_PEAK_GBS, 4),
           "finite": bool(torch.isfinite(audio).all().item()),
           "handoff_timeouts": chain.handoff_timeouts()}      # 0 required (include/uhsdr.h failure contract)
    chain.close()
    if out["handoff_timeouts"]:
        raise RuntimeError(f"{name}: a device hand-off poll gave up: the line is invalid")
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--only", default="c3,c3spec,c3zoom,c4fm,c4tx,c4txfma,c5,c5fir")
    ap.add_argument("--fir-waves", type=int, default=0, help="c5fir: waves per workgroup (EXACT 1, 2, 4; MFMA 1 .. 16; 0 = the default)")
    ap.add_argument("--serial", action="store_true",
                    help="C4 FM-RX / SSB-TX handles in their serial mode (default: pipelined, measured faster there; "
                         "C3 SAM and C5 CW run serial, where the pipelined mode measured slower / the same)")
    ap.add_argument("--front-block", type=int, default=0, choices=[0, 8, 16], help="RX lines: front outputs per lane")
    ap.add_argument("--handoff", default="persistent", choices=["event", "device", "persistent"],
                    help="pipelined RX lines: the persistent back end (uhsdr_rx_set_pipelined 3; other back ends "
                         "fall back to 2), the device hand-off (2) or a cross-stream event (1)")
    a = ap.parse_args()
    global FRONT_BLOCK, HANDOFF
    FRONT_BLOCK = a.front_block
    HANDOFF = a.handoff
    import torch
    import uhsdr_amd as U
    from uhsdr_amd import synth
    want = set(a.only.split(","))
    lines = []
    if "c3" in want:
        C, N = 32768, 1024
        cfg = U.default_config(filter_path=70, dmod_mode=U.DEMOD_SAM)
        lines.append(rx_line("C3 SAM P70 RX (PLL 2500/0.65/250, fade on)", cfg, C, N,
                             tiled(synth.am_iq, C, N), a.steps, a.warmup))
    if "c3pipe" in want:                                 # C3 in the pipelined mode (A/B; not a default line)
        C, N = 32768, 1024
        cfg = U.default_config(filter_path=70, dmod_mode=U.DEMOD_SAM)
        lines.append(rx_line("C3 SAM P70 RX (PLL 2500/0.65/250, fade on)", cfg, C, N,
                             tiled(synth.am_iq, C, N), a.steps, a.warmup, pipelined=True))
    if "c3spec" in want:
        C, N, L = 32768, 1024, 1024
        s = torch.cuda.current_stream()
        spec = U.Spectrum(U.default_spectrum_config(fft_len=L), channels=C, frames=N, stream=s.cuda_stream)
        iq = tiled(synth.am_iq, C, N)
        avg = torch.empty(spec.out_shape, dtype=torch.float32, device="cuda")
        ms = time_calls(lambda: spec.process(iq, None, avg), a.steps, a.warmup)
        byts = C * N * (8 + 4) + C * L * 8
        lines.append({"workload": "C3 spectrum 1024-point (Hann, CFFT, magnitude, IIR average)", "channels": C,
                      "frames_per_call": N, "ms_per_call": round(ms, 4), "msamples_per_s": round(C * N / ms / 1e3, 1),
                      "alg_bytes_per_frame": round(byts / (C * N), 2),
                      "hbm_frac": round(byts / ms / 1e6 / HBM_PEAK_GBS, 4),
                      "finite": bool(torch.isfinite(avg).all().item())})
        spec.close()
    if "c3zoom" in want:
        # zoom producer (spectrum_zoom) 8x + 256-point display: 8 B in per frame, the ring
        # scratch written and read once (8 / D B each way), zoom state (2 x (16 + 3) + 2 + 3
        # floats) and the display state per call
        C, N, L, m = 32768, 2048, 256, 3
        D = 1 << m
        s = torch.cuda.current_stream()
        spec = U.Spectrum(U.default_spectrum_config(fft_len=L, magnify=m), channels=C, frames=N, stream=s.cuda_stream)
        iq = tiled(synth.ssb_iq, C, N)
        avg = torch.empty(spec.out_shape, dtype=torch.float32, device="cuda")
        ms = time_calls(lambda: spec.process(iq, None, avg), a.steps, a.warmup)
        byts = C * N * (8 + 2 * 8 / D) + C * (2 * 4 * (2 * 19 + 5) + 2 * 4 * L) + C * (N // D // L) * L * 4
        lines.append({"workload": f"C3-size zoom spectrum {D}x, {L}-point (FreqShift, zoom biquad, decimate, CFFT)",
                      "channels": C, "frames_per_call": N, "ms_per_call": round(ms, 4),
                      "msamples_per_s": round(C * N / ms / 1e3, 1), "alg_bytes_per_frame": round(byts / (C * N), 2),
                      "hbm_frac": round(byts / ms / 1e6 / HBM_PEAK_GBS, 4),
                      "finite": bool(torch.isfinite(avg).all().item())})
        spec.close()
    if "c4fm" in want:
        C, N = 262144 // 8, 256
        cfg = U.default_config(filter_path=1, dmod_mode=U.DEMOD_FM, fm_sql_threshold=12)
        lines.append(rx_line("C4 per-GPU share: FM-RX P1 (squelch 12)", cfg, C, N,
                             tiled(synth.fm_iq, C, N), a.steps, a.warmup, pipelined=not a.serial))
    for key in ("c4tx", "c4txfma"):
        if key not in want:
            continue
        fma = key == "c4txfma"
        C, N = 262144 // 8, 256
        s = torch.cuda.current_stream()
        tx = U.TxChain(channels=C, frames=N, stream=s.cuda_stream)
        if not a.serial:
            tx.set_pipelined(True)
        if fma:
            tx.set_precision(U.PRECISION_FMA)
        audio = tiled(synth.tx_audio, C, N)
        iq = torch.empty((C, N, 2), dtype=torch.int32, device="cuda")
        a0 = torch.empty((C, N), dtype=torch.float32, device="cuda")
        ms = time_calls(lambda: tx.process(audio, iq, a0), a.steps, a.warmup, None if a.serial else tx.join)
        # 8 B audio frame in, 8 B I/Q frame out, state (Hilbert 200, lattice 10, biquads 12, ALC,
        # 320-sample delay line) read + written once per call, the f32 hand-off between kernels
        state = 4 * (200 + 10 + 12 + 1 + 320)
        per = 16 + 2 * state / N
        lines.append({"workload": "C4 per-GPU share: SSB-TX (IIR_TX_SOPRANO + biquads + ALC + 201-tap Hilbert + Fs/4)",
                      "precision": "fma (Hilbert pair, 1e-5 normwise)" if fma else "exact", "channels": C, "frames_per_call": N, "pipelined": not a.serial, "ms_per_call": round(ms, 4),
                      "msamples_per_s": round(C * N / ms / 1e3, 1), "alg_bytes_per_frame": round(per, 2),
                      "hbm_frac": round(C * N * per / ms / 1e6 / HBM_PEAK_GBS, 4),
                      "finite": bool(torch.isfinite(a0).all().item()) and bool((iq != 0).any().item())})
        tx.close()
    if "c5" in want:
        C, N = 1048576 // 8, 256
        cfg = U.default_config(filter_path=4, dmod_mode=U.DEMOD_CW)
        lines.append(rx_line("C5 per-GPU share: CW P4 (199-tap Hilbert @12k, 300 Hz lattice) + CW decoder Goertzel",
                             cfg, C, N, tiled(synth.cw_iq, C, N), a.steps, a.warmup, cw=True))
    if "c5fir" in want:
        import numpy as np
        C, N = 1048576 // 8, 256
        taps = np.load(os.path.join(ROOT, "tests", "golden", "fir513_kaiser.npy"))
        T = len(taps)
        x = torch.randn((min(C, 4096), N), device="cuda").mul_(1000.0).repeat((C + 4095) // 4096, 1)[:C].contiguous()
        y = torch.empty_like(x)
        s = torch.cuda.current_stream()
        for mode, name in ((U.fir.EXACT, "exact, bit-identical to arm_fir_f32"),
                           (U.fir.MFMA, "MFMA v_mfma_f32_16x16x4_f32, FIR as GEMM, fused MACs")):
            fir = U.FirBatch(taps, C, N, mode, stream=s.cuda_stream)
            if a.fir_waves:
                fir.set_waves(a.fir_waves)
            # at least 200 warm-up calls: in a process that runs only this line, the chip's clock dips
            # during the first ~50 MFMA launches (2.26 -> 1.91 -> 2.31 GHz, profiles/r05_fir_clock.txt)
            # and a 5-call warm-up timed the dip (0.314 vs 0.285 ms, profiles/r06_c5fir_alone.txt)
            ms = time_calls(lambda: fir.process(x, y), a.steps, max(a.warmup, 200))
            waves = fir.waves
            fir.close()
            per = 8 + 2 * 4 * (T - 1) / N                 # 4 B in + 4 B out, carried samples in + out
            K = (T + 15 + 3) & ~3
            line = {"workload": f"C5 per-GPU share: batched 513-tap FIR at 12 ksps ({name})", "channels": C,
                    "frames_per_call": N, "waves_per_workgroup": waves, "ms_per_call": round(ms, 4), "msamples_per_s": round(C * N / ms / 1e3, 1),
                    "alg_bytes_per_frame": round(per, 2), "hbm_frac": round(C * N * per / ms / 1e6 / HBM_PEAK_GBS, 4),
                    "alg_tflops": round(C * N * 2 * T / ms / 1e9, 1),
                    "finite": bool(torch.isfinite(y).all().item())}
            if mode == U.fir.MFMA:
                line["mfma_tflops_issued"] = round(C * N * 2 * K / ms / 1e9, 1)
                line["mfma_f32_peak_tflops"] = 157.3
            lines.append(line)
    bad = []
    for ln in lines:
        ln["data"] = "synthetic: 4096 distinct channels tiled"
        print(json.dumps(ln), flush=True)
        if not ln.get("finite", False):
            bad.append(ln["workload"])
    if bad:
        # every line's outputs must be finite (and the TX I/Q not all zero): a fast wrong kernel
        # is not a measurement
        sys.exit(f"non-finite outputs: {bad}")


if __name__ == "__main__":
    main()
