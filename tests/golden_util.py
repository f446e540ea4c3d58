"""Shared helpers for the golden-fixture tests (tests/golden/rx_*.npz, see make_golden.py)."""
import glob
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def golden_files():
    return sorted(glob.glob(os.path.join(GOLDEN, "rx_*.npz")))


def golden_file(name):
    return os.path.join(GOLDEN, f"rx_{name}.npz")


def load(path):
    d = np.load(path)
    return {
        "name": os.path.basename(path)[3:-4],
        "iq": d["iq"], "a1": d["a1"], "dst": d["dst"],
        "args": json.loads(str(d["args"])), "setup": json.loads(str(d["setup"])), "agc": json.loads(str(d["agc"])),
    }


def bits(x):
    return np.ascontiguousarray(x, dtype=np.float32).view(np.uint32)


def assert_bitexact(got, ref, what=""):
    g, r = bits(got), bits(ref)
    if not np.array_equal(g, r):
        bad = np.argwhere(g != r)
        i = tuple(bad[0])
        rel = np.abs(got.astype(np.float64) - ref) .max() / max(np.abs(ref).max(), 1e-30)
        raise AssertionError(f"{what}: {len(bad)} of {g.size} samples differ; first at {i}: "
                             f"{got[i]!r} vs {ref[i]!r}; normwise {rel:.3e}")
