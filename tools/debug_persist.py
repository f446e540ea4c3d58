"""The persistent back end's control words after each call (uhsdr_rx_debug_persist), C2-like shape
with a few hundred channels: process calls one at a time with pauses, print the words.
Usage: UHSDR_LIB=... python tools/debug_persist.py [C] [calls] [pause_ms]"""
import ctypes as C
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    import torch
    import uhsdr_amd as U
    from uhsdr_amd import synth
    Cn = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    calls = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    pause = float(sys.argv[3]) / 1e3 if len(sys.argv) > 3 else 0.05
    N = 256
    lib = U.load()
    lib.uhsdr_rx_debug_persist.argtypes = [C.c_void_p, C.POINTER(C.c_uint32)]
    chain = U.RxChain(U.default_config(), channels=Cn, frames=N)
    chain.set_pipelined(3)
    xs = [synth.ssb_iq_torch(0, Cn, k * N, N, torch.device("cuda")) for k in range(calls)]
    audio = torch.empty((calls, Cn, N), dtype=torch.float32, device="cuda")
    w = (C.c_uint32 * 7)()
    names = ["grant", "epoch", "exit", "decided", "consumed", "plive", "plast"]

    def show(tag):
        lib.uhsdr_rx_debug_persist(chain.handle, w)
        print(tag, {n: (int(v) if n != "decided" else (int(v) >> 1, int(v) & 1)) for n, v in zip(names, w)}, flush=True)

    torch.cuda.synchronize()
    for k in range(calls):
        chain.process(xs[k], audio[k], None)
        show(f"after process {k}")
        time.sleep(pause)
        show(f"  +{pause * 1e3:.0f} ms")
    chain.synchronize()
    show("after synchronize")
    print("timeouts", chain.handoff_timeouts(), "finite", bool(torch.isfinite(audio).all()))
    chain.close()


if __name__ == "__main__":
    main()
