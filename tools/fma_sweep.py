"""Normwise FMA error of every path x demodulator x stereo the library accepts FMA for
(tests/test_gpu_fma.py's accepted_fma_cases), against the CPU oracle: one JSON line per case.
The evidence behind uhsdr_rx_set_precision's FMA acceptance list.

  python tools/fma_sweep.py > gpurun_out/fma_sweep.jsonl
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]

import oracle  # noqa: E402
import uhsdr_amd as U  # noqa: E402
from test_gpu_fma import accepted_fma_cases, fma_case_error  # noqa: E402


def main():
    import torch
    torch.cuda.init()
    for kw in accepted_fma_cases(refused_too=True):
        if not U.plan_fma_ok(U.build_plan(U.default_config(**kw))):
            print(json.dumps(dict(kw, refused=True)), flush=True)
            continue
        try:
            err = fma_case_error(kw)
            line = dict(kw, err=max(err.values()), **{f"err_{k}": v for k, v in err.items()})
        except Exception as e:          # noqa: BLE001
            line = dict(kw, error=str(e)[:200])
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
