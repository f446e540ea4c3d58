"""Host-side submission cost of one RxChain call at the C2 shape (4096 x 256), per schedule / mode
and per Python entry (process(): shape and contiguity checks every call; process_ptr(): a buffer
set validated once by bind()).  30 calls are enqueued without synchronising (the GPU queue does
not fill: host us/call), then the GPU drains them (host+drain us/call = the wall clock of 30
calls from an idle device, the driver's short-run regime)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import uhsdr_amd as U  # noqa: E402
from uhsdr_amd import synth  # noqa: E402

C, N = 4096, 256
dev = torch.device("cuda:0")
MODES = [("serial", U.SCHEDULE_SPLIT_PIPE, False), ("pipelined", U.SCHEDULE_SPLIT_PIPE, True),
         ("device hand-off", U.SCHEDULE_SPLIT_PIPE, 2), ("persistent", U.SCHEDULE_SPLIT_PIPE, 3)]
for name, sched, pipe in MODES:
    stream = torch.cuda.current_stream(dev)
    ch = U.RxChain(U.default_config(), channels=C, frames=N, stream=stream.cuda_stream, schedule=sched)
    ch.set_pipelined(pipe)
    x = synth.ssb_iq_torch(0, C, 0, N, dev)
    a = torch.empty((C, N), dtype=torch.float32, device=dev)
    ptrs = ch.bind(x, a, None)
    for _ in range(50):
        ch.process(x, a, None)
    torch.cuda.synchronize()
    for entry in ("process", "process_ptr"):
        call = (lambda: ch.process(x, a, None)) if entry == "process" else (lambda: ch.process_ptr(ptrs))
        for rep in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(30):
                call()
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            print(f"{name:9s} {entry:11s} host {1e6 * (t1 - t0) / 30:6.1f} us/call, host+drain {1e6 * (t2 - t0) / 30:6.1f} us/call",
                  flush=True)
    ch.close()
