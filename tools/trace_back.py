#!/usr/bin/env python3
"""Per-role timing of the pipelined back end (rx_back) from a UHSDR_TRACE build
(make variant VTAG=trace VFLAGS=-DUHSDR_TRACE): shader-clock cycles each role spends on its
call per pipeline step, and waiting at the step's barrier.  Usage:
    UHSDR_LIB=uhsdr_amd/lib/variants/libuhsdr_amd_trace.so python tools/trace_back.py [C] [N]"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import uhsdr_amd as U
    from uhsdr_amd import synth
    Cn = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    opts = sys.argv[3:]
    sam = "sam" in opts                                        # C3's SAM P70 chain (demod role first)
    mchf = "mchf" in opts                                      # the mcHF board's output stage
    want_dst = "dst" in opts                                   # int32 codec frames too
    cfg = (U.default_config(filter_path=70, dmod_mode=U.DEMOD_SAM) if sam else
           U.default_config(board=U.BOARD_MCHF) if mchf else U.default_config())
    chain = U.RxChain(cfg, channels=Cn, frames=N, schedule=U.SCHEDULE_SPLIT_PIPE)
    pipe = "device" in opts                                   # the device hand-off: the last launch
    if pipe:                                                   # starts skewed (BackSched) and drains
        chain.set_pipelined(2)
    if sam:
        x = torch.from_numpy(synth.am_iq(np.arange(Cn), 0, N)).cuda()
    else:
        x = synth.ssb_iq_torch(0, Cn, 0, N, "cuda")
    audio = torch.empty((Cn, N), dtype=torch.float32, device="cuda")
    audio0 = torch.empty((Cn, N), dtype=torch.float32, device="cuda")
    dst = torch.empty((Cn, N, 2), dtype=torch.int32, device="cuda") if want_dst else None
    for _ in range(30 if pipe else 5):
        if mchf:
            chain.process_stereo(x, audio, audio0, dst)
        else:
            chain.process(x, audio, dst)
    chain.synchronize()
    lib = U.load()
    buf = np.zeros((64, 10, 40, 3), np.uint64)
    lib.uhsdr_trace_read.argtypes = [C.c_void_p]
    assert lib.uhsdr_trace_read(buf.ctypes.data_as(C.c_void_p)) == 0
    calls = N // 32
    roles = (6 if sam else 5) + 4                              # + the four tail waves
    its = calls + roles - 5
    if pipe:
        its = calls                                            # a skewed launch: n steps, no fill
    ent = buf[:, :roles, 39, :2].astype(np.int64)
    t = buf[:, :roles, :its, :].astype(np.int64)
    t0 = t[:, :, 0, 0].min(axis=1)[:, None, None]
    work = (t[:, :, :, 1] - t[:, :, :, 0])
    wait = (t[:, :, :, 2] - t[:, :, :, 1])
    names = (["demod"] if sam else []) + ["pre", "agc", "audio", "aa", "output", "tail0", "tail1", "tail2", "tail3"]
    print(f"C={Cn} N={N}: per-step cycles (median over workgroups), work / barrier wait")
    for it in range(its):
        row = " ".join(f"{names[r]:>6} {int(np.median(work[:, r, it])):6d}/{int(np.median(wait[:, r, it])):6d}" for r in range(roles))
        print(f"step {it:2d}: {row}")
    total = int(np.median(t[:, 0, its - 1, 2] - t[:, 0, 0, 0]))
    print(f"total cycles (median WG): {total}")
    e0 = ent[:, :, 0].min(axis=1)
    print("entry -> first step start, per role (median cycles):",
          [int(np.median(t[:, r, 0, 0] - e0)) for r in range(roles)])
    print("wave start after the workgroup's first, per role (median cycles):",
          [int(np.median(ent[:, r, 0] - e0)) for r in range(roles)])
    sk = buf[:, :roles, 39, 2].astype(np.int64)
    print("own entry -> skew word consumed, per role (median cycles):",
          [int(np.median(sk[:, r] - ent[:, r, 0])) for r in range(roles)])
    print("last barrier -> exit, per role (median cycles):",
          [int(np.median(ent[:, r, 1] - t[:, r, its - 1, 2])) for r in range(roles)])
    print("entry -> last exit (median WG):", int(np.median(ent[:, :, 1].max(axis=1) - e0)))
    rt = buf[:, :roles, 38, :2].astype(np.int64)               # s_memrealtime (100 MHz) at entry / exit
    if rt.any():
        cyc = ent[:, :, 1] - ent[:, :, 0]
        ns = (rt[:, :, 1] - rt[:, :, 0]) * 10.0
        print(f"shader clock (median over waves): {np.median(cyc / np.maximum(ns, 1)):.3f} GHz; "
              f"wave life median {np.median(ns) / 1e3:.2f} us")


if __name__ == "__main__":
    main()
