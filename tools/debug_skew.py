#!/usr/bin/env python3
"""Debug aid for the skewed device hand-off: the C2 shape, 12 calls back to back (device hand-off),
every channel against the oracle; prints per-call / per-group counts of differing samples."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import oracle  # noqa: E402
import uhsdr_amd as U  # noqa: E402
from uhsdr_amd import synth  # noqa: E402

C, N, calls = int(sys.argv[1]) if len(sys.argv) > 1 else 4096, 256, 12
dev = torch.device("cuda:0")
cfg = U.default_config()
chain = U.RxChain(cfg, channels=C, frames=N)
chain.set_pipelined(2)
xs = [synth.ssb_iq_torch(0, C, k * N, N, dev) for k in range(calls)]
audio = torch.empty((calls, C, N), dtype=torch.float32, device=dev)
torch.cuda.synchronize()
for k in range(calls):
    chain.process(xs[k], audio[k], None)
chain.synchronize()
print("timeouts", chain.handoff_timeouts())
iq = np.concatenate([x.cpu().numpy() for x in xs], axis=1)
ref, _ = oracle.OracleRx(U.build_plan(cfg), C).process(np.ascontiguousarray(iq), threads=16)
got = audio.permute(1, 0, 2).reshape(C, calls * N).cpu().numpy()
bad = got.view(np.uint32) != ref.view(np.uint32)
print("bad total", int(bad.sum()), "nan", int(np.isnan(got).sum()))
for k in range(calls):
    b = bad[:, k * N:(k + 1) * N]
    if b.any():
        groups = sorted(set((np.nonzero(b.any(axis=1))[0] // 64).tolist()))
        subs = sorted(set((np.nonzero(b.any(axis=0))[0] // 32).tolist()))
        print(f"call {k}: {int(b.sum())} bad, groups {groups[:20]}, subcalls {subs}")
