"""Host-side cost of one uhsdr_rx_process call (C2 shape): enqueue rate with the GPU far ahead
vs the device rate, for serial / pipelined and per-kernel timing on / off."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import uhsdr_amd as U
from uhsdr_amd import synth

C, N = int(sys.argv[1]) if len(sys.argv) > 1 else 4096, 256
dev = torch.device("cuda", 0)
x = [synth.ssb_iq_torch(0, C, k * N, N, dev) for k in range(8)]
audio = torch.empty((C, N), dtype=torch.float32, device=dev)
for pipe in (False, True):
    for timing in (False, True):
        chain = U.RxChain(U.default_config(), channels=C, frames=N, stream=torch.cuda.current_stream(dev).cuda_stream)
        chain.set_pipelined(pipe)
        for s in range(50):
            chain.process(x[s % 8], audio, None)
        torch.cuda.synchronize()
        chain.enable_timing(timing)
        K = 2000
        t0 = time.perf_counter()
        for s in range(K):
            chain.process(x[s % 8], audio, None)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        kt = chain.kernel_times() if timing else {}
        chain.enable_timing(False)
        print(f"pipe={pipe} timing={timing}: host enqueue {1e6*(t1-t0)/K:.1f} us/call, wall {1e6*(t2-t0)/K:.1f} us/call "
              + " ".join(f"{k}={1e3*v[0]/max(v[1],1):.1f}us" for k, v in kt.items()), flush=True)
        chain.close()
# raw ctypes cost
lib = U._abi.lib() if hasattr(U._abi, "lib") else None
t0 = time.perf_counter()
for s in range(20000):
    x[0].data_ptr(); audio.is_contiguous()
print(f"python tensor attr overhead ~{1e6*(time.perf_counter()-t0)/20000:.2f} us", flush=True)
