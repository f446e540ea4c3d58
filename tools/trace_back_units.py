#!/usr/bin/env python3
"""Per-unit timeline of the rx_back wave pipeline (SPLIT_PIPE, serial) from a UHSDR_STREAM_TRACE
build (make variant VTAG=strace VFLAGS="-DUHSDR_STREAM_TRACE -Itools/isa"):
    UHSDR_LIB=uhsdr_amd/lib/variants/libuhsdr_amd_strace.so python tools/trace_back_units.py [C] [N]
For every role: when it reached unit u (event u), when its wait for unit u ended (14 + u), and
its end (30); s_memrealtime (100 MHz).  Printed: medians over the channel groups, in us from the
launch's first stamp; 'wait' = time the role spent polling before the unit, 'work' = until the next."""
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
    chain = U.RxChain(U.default_config(), channels=Cn, frames=N, schedule=U.SCHEDULE_SPLIT_PIPE)
    x = synth.ssb_iq_torch(0, Cn, 0, N, "cuda")
    audio = torch.empty((Cn, N), dtype=torch.float32, device="cuda")
    for _ in range(6):
        chain.process(x, audio)
        torch.cuda.synchronize()
    lib = U.load()
    buf = np.zeros((256, 8, 32), np.uint64)
    lib.uhsdr_strace_read.argtypes = [C.c_void_p]
    assert lib.uhsdr_strace_read(buf.ctypes.data_as(C.c_void_p)) == 0
    groups = (Cn + 63) // 64
    t = buf[:groups, :5].astype(np.int64)
    t0 = t[t > 0].min()
    us = (t - t0) / 100.0
    units = min(14, (N // 32) * int(os.environ.get("UNITS", "2")))
    names = ["pre", "agc", "audio", "aa", "output"]
    print(f"C={Cn} N={N}, rx_back (SPLIT_PIPE): per unit, median over {groups} groups (us)")
    for r in range(5):
        st = np.median(us[:, r, :units], axis=0)
        wt = np.median(us[:, r, 14:14 + units] - us[:, r, :units], axis=0)
        print(f"{names[r]:>6} start " + " ".join(f"{v:6.2f}" for v in st) + f"  end {np.median(us[:, r, 30]):6.2f}")
        print(f"{'':>6} wait  " + " ".join(f"{v:6.2f}" for v in wt))
    print(f"launch span (median): {np.median(us[:, :, 30].max(axis=1)):.2f} us")


if __name__ == "__main__":
    main()
