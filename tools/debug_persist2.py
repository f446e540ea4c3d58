"""Persistent back end against the device hand-off on the same inputs, per call: the first call whose
audio differs, and the launches the persistent run took (uhsdr_rx_debug_persist).
Usage: UHSDR_LIB=... python tools/debug_persist2.py [C] [N] [calls] [pause_ms]"""
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
    Cn = int(sys.argv[1]) if len(sys.argv) > 1 else 130
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 512
    calls = int(sys.argv[3]) if len(sys.argv) > 3 else 15
    pause = float(sys.argv[4]) / 1e3 if len(sys.argv) > 4 else 0.0
    opts = sys.argv[5:]
    cfg = U.default_config(filter_path=48, dmod_mode=U.DEMOD_USB) if "usb" in opts else U.default_config()
    lib = U.load()
    lib.uhsdr_rx_debug_persist.argtypes = [C.c_void_p, C.POINTER(C.c_uint32)]
    iq = synth.ssb_iq(np.arange(Cn), 0, calls * N)
    xs = [torch.from_numpy(np.ascontiguousarray(iq[:, k * N:(k + 1) * N])).cuda() for k in range(calls)]
    outs = {}
    for mode in ((3,) if "only3" in opts else (2, 3)):
        chain = U.RxChain(cfg, channels=Cn, frames=N)
        chain.set_pipelined(mode)
        audio = torch.empty((calls, Cn, N), dtype=torch.float32, device="cuda")
        dst = torch.empty((calls, Cn, N, 2), dtype=torch.int32, device="cuda") if "dst" in opts else None
        torch.cuda.synchronize()
        for k in range(calls):
            try:
                chain.process(xs[k], audio[k], dst[k] if dst is not None else None)
                if "join" in opts:
                    chain.join()
            except U.UhsdrError as e:
                print("call", k, "raised", e.status, flush=True)
            if mode == 3 and "trace" in opts:
                w = (C.c_uint32 * 8)()
                lib.uhsdr_rx_debug_persist(chain.handle, w)
                print("  after call", k, list(w), flush=True)
            if pause:
                time.sleep(pause)
        try:
            chain.synchronize()
        except U.UhsdrError as e:
            print("synchronize raised", e.status, flush=True)
        if mode == 3:
            w = (C.c_uint32 * 8)()
            lib.uhsdr_rx_debug_persist(chain.handle, w)
            print("persist words", list(w), flush=True)
            if hasattr(lib, "uhsdr_pdbg_read"):
                buf = np.zeros(64 * 8 + 64 * 4 * 2, np.uint64)
                lib.uhsdr_pdbg_read.argtypes = [C.c_void_p]
                lib.uhsdr_pdbg_read(buf.ctypes.data_as(C.c_void_p))
                b2 = buf[64 * 8:].reshape(64, 4, 2)
                buf = buf[:64 * 8].reshape(64, 8)
                for k in range(calls):
                    print(f"followers call {k}:", [(hex(int(b2[k, g, 0])), int(b2[k, g, 1])) for g in range(4)], flush=True)
                for k in range(calls if "quiet" not in opts else 0):
                    r = buf[k]
                    print(f"dev call {int(r[0])}: adec {int(r[1]):#x} cnt {int(r[2]):#x} target {int(r[3])} "
                          f"arrived {int(r[4])} dst {int(r[5]):#x} fast {int(r[6])} gave_up {int(r[7])}", flush=True)
        outs[mode] = audio.cpu().numpy()
        print("mode", mode, "timeouts", chain.handoff_timeouts(), "nan calls",
              [k for k in range(calls) if not np.isfinite(outs[mode][k]).all()], flush=True)
        chain.close()
    if 2 not in outs:
        return
    d = np.abs(outs[2].astype(np.float64) - outs[3])
    bad_calls = [k for k in range(calls) if d[k].max() > 0]
    print("summary", sys.argv[1:], "first bad call", bad_calls[0] if bad_calls else None, flush=True)
    if "quiet" in opts:
        return
    for k in range(calls):
        bad = np.argwhere(d[k] > 0)
        first = tuple(bad[0]) if len(bad) else None
        print(f"call {k}: max diff {d[k].max():.3e}, differing {len(bad)}, first (ch, frame) {first}")


if __name__ == "__main__":
    main()
