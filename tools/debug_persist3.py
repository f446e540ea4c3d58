"""Per-call timing inside one persistent back-end launch (UHSDR_PDEBUG build): group 0's pre role
stamps s_memrealtime (100 MHz) at sub-call 4, n-4, n-1 and after the decision of every call.
Usage: UHSDR_LIB=<pdebug build> python tools/debug_persist3.py [calls] [warmup]"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    import torch
    import uhsdr_amd as U
    from uhsdr_amd import synth
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 60
    warm = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    Cn, N = 4096, 256
    dev = torch.device("cuda")
    lib = U.load()
    chain = U.RxChain(U.default_config(), channels=Cn, frames=N, stream=torch.cuda.current_stream(dev).cuda_stream)
    chain.set_pipelined(3)
    xs = [synth.ssb_iq_torch(0, Cn, k * N, N, dev) for k in range(8)]
    audio = torch.empty((Cn, N), dtype=torch.float32, device=dev)
    ptrs = [chain.bind(x, audio, None) for x in xs]
    for k in range(warm):
        chain.process_ptr(ptrs[k % 8])
    torch.cuda.synchronize()
    for k in range(calls):
        chain.process_ptr(ptrs[k % 8])
    torch.cuda.synchronize()
    buf = np.zeros(64 * 8 + 64 * 4 * 2 + 1024 * 8, np.uint64)
    lib.uhsdr_pdbg_read.argtypes = [C.c_void_p]
    assert lib.uhsdr_pdbg_read(buf.ctypes.data_as(C.c_void_p)) == 0
    t = buf[64 * 8 + 64 * 4 * 2:].reshape(1024, 8).astype(np.int64)
    first = warm + 1               # (call 0 of the handle runs the event path; the warm-up launch closes)
    rows = []
    for k in range(warm + 1, warm + calls):
        if t[k, 3] == 0 or t[k - 1, 3] == 0:
            continue
        us = lambda a, b: (t[k, b] - t[k, a]) * 10 / 1e3
        rows.append((k, (t[k, 3] - t[k - 1, 3]) * 10 / 1e3, us(1, 4), us(4, 5), us(5, 2), us(2, 3), us(6, 7)))
    print("call, decision-to-decision, g0: n-4 -> n-3 (grant consumed), -> n-2, -> n-1, decision; g1: decision wait (us)")
    for r in rows[:40]:
        print(f"{r[0]:4d} {r[1]:7.2f} | {r[2]:6.2f} {r[3]:6.2f} {r[4]:6.2f} {r[5]:6.2f} | {r[6]:6.2f}")
    d = np.array([r[1] for r in rows])
    if len(d):
        print(f"median {np.median(d):.2f} us, first 10 mean {d[:10].mean():.2f}, last 10 mean {d[-10:].mean():.2f}")
    chain.close()


if __name__ == "__main__":
    main()
