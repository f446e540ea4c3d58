#!/usr/bin/env python3
"""Timeline of one rx_stream launch (the STREAM schedule) from a UHSDR_STREAM_TRACE build:
    make variant VTAG=strace VFLAGS="-DUHSDR_STREAM_TRACE -Itools/isa"
    UHSDR_LIB=uhsdr_amd/lib/variants/libuhsdr_amd_strace.so python tools/trace_stream.py [C] [N]
s_memrealtime (100 MHz, chip-wide) stamps: each front wave's publish of every 32-frame call, the
back end's pre-role poll returning per call, every role's pipeline-step starts and ends.  Printed
in us from the launch's first stamp, medians over the channel groups (front: the group's last wave)."""
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
    chain = U.RxChain(U.default_config(), channels=Cn, frames=N, schedule=U.SCHEDULE_STREAM)
    x = synth.ssb_iq_torch(0, Cn, 0, N, "cuda")
    audio = torch.empty((Cn, N), dtype=torch.float32, device="cuda")
    for _ in range(6):
        chain.process(x, audio)
        torch.cuda.synchronize()
    assert chain.stream_timeouts() == 0
    lib = U.load()
    buf = np.zeros((256, 8, 32), np.uint64)
    lib.uhsdr_strace_read.argtypes = [C.c_void_p]
    assert lib.uhsdr_strace_read(buf.ctypes.data_as(C.c_void_p)) == 0
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    groups = (Cn + 63) // 64
    SWPG = 16                                                     # front waves per group (uhsdr_rx.hip)
    F = min((cus - groups) // groups, SWPG)
    wpw = (SWPG + F - 1) // F
    nfront = F * groups
    S = N // 32
    t = buf.astype(np.int64)
    live = t[: nfront + groups]
    t0 = live[live > 0].min()
    us = lambda v: (v - t0) / 100.0                              # noqa: E731
    # front: group of each front workgroup (the kernel's mapping)
    pub = np.zeros((groups, S))
    fend = np.zeros(groups)
    for b in range(nfront):
        if groups % 8 == 0 and nfront % 8 == 0:
            x_, q = b & 7, b >> 3
            g = x_ + 8 * (q % (groups // 8))
        else:
            g = b // F
        for w in range(wpw):
            if t[b, w, 0] == 0:
                continue
            pub[g] = np.maximum(pub[g], [us(t[b, w, 1 + s]) for s in range(S)])
            fend[g] = max(fend[g], us(t[b, w, 30]))
    print(f"C={Cn} N={N}: {nfront} front + {groups} back workgroups ({F} front WGs x {wpw} waves per group)")
    # front step 3 in detail (events 20-26 of every front wave)
    fw = []
    for b in range(nfront):
        for w in range(wpw):
            if t[b, w, 20] > 0:
                fw.append(t[b, w, 20:27] - t[b, w, 20])
    if fw:
        fw = np.array(fw) / 100.0
        lbl = ["convert+prefetch", "wave_sync", "Hilbert FIR", "comb+window+sync", "decimator", "lazy publish", "store+end"]
        d = np.median(np.diff(fw, axis=1), axis=0)
        print("front step 3, median us per part: " + ", ".join(f"{lbl[i + 1]} {d[i]:.2f}" for i in range(len(d))))
    print("front publish of call s (group's last wave), median / max over groups:")
    print("  " + " ".join(f"{np.median(pub[:, s]):6.2f}/{pub[:, s].max():6.2f}" for s in range(S)), f" end {np.median(fend):.2f}")
    bk = t[nfront: nfront + groups]
    print("pre-role poll return per call (median):")
    print("  " + " ".join(f"{np.median(us(bk[:, 0, 16 + s])):6.2f}" for s in range(S)))
    names = ["pre", "agc", "audio", "aa", "output"]
    steps = S + 4
    for r in range(5):
        print(f"{names[r]:>6} step starts: " + " ".join(f"{np.median(us(bk[:, r, i])):6.2f}" for i in range(min(steps, 16)))
              + f"  end {np.median(us(bk[:, r, 30])):6.2f}")
    print(f"launch span (median group end): {np.median(us(bk[:, :5, 30].max(axis=1))):.2f} us; "
          f"max {us(bk[:, :5, 30].max()):.2f} us")


if __name__ == "__main__":
    main()
