"""Host-side submission cost of one RxChain.process call (C2 shape), serial and pipelined:
30 calls timed without synchronising (the GPU queue does not fill), then the GPU time of the
same 30 calls after a sync."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import uhsdr_amd as U  # noqa: E402
from uhsdr_amd import synth  # noqa: E402

C, N = 4096, 256
dev = torch.device("cuda:0")
for pipe in (False, True):
    stream = torch.cuda.current_stream(dev)
    ch = U.RxChain(U.default_config(), channels=C, frames=N, stream=stream.cuda_stream)
    ch.set_pipelined(pipe)
    x = synth.ssb_iq_torch(0, C, 0, N, dev)
    a = torch.empty((C, N), dtype=torch.float32, device=dev)
    for _ in range(50):
        ch.process(x, a, None)
    torch.cuda.synchronize()
    for rep in range(3):
        t0 = time.perf_counter()
        for _ in range(30):
            ch.process(x, a, None)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"pipelined={pipe} host {1e6 * (t1 - t0) / 30:.1f} us/call, host+drain {1e6 * (t2 - t0) / 30:.1f} us/call")
    ch.close()
