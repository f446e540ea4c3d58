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
    g = {
        "name": os.path.basename(path)[3:-4],
        "iq": d["iq"], "a1": d["a1"], "dst": d["dst"],
        "args": json.loads(str(d["args"])), "setup": json.loads(str(d["setup"])), "agc": json.loads(str(d["agc"])),
    }
    if "a0" in d.files:
        g["a0"] = d["a0"]
    return g


def beep_of(args):
    """(first call, calls) of the fixture's key beep (uhsdr_ref beep=b0:K), or None."""
    b = args.get("beep")
    if not b:
        return None
    b0, k = (int(x) for x in str(b).split(":"))
    return b0, k


def drive(g, frames, process, key_beep=None):
    """Feed the fixture's I/Q to `process(iq_block)` in blocks of `frames`, issuing the
    fixture's key beep (AudioManagement_KeyBeep) right before the block that starts at its first
    call.  Returns the concatenated results of process (tuples concatenated per element)."""
    iq = g["iq"]
    n = iq.shape[1]
    b = beep_of(g["args"])
    if b is not None:
        assert (b[0] * 32) % frames == 0, f"beep start call {b[0]} not on a {frames}-frame boundary"
    outs = []
    for off in range(0, n, frames):
        if b is not None and off == b[0] * 32:
            key_beep(b[1])
        outs.append(process(np.ascontiguousarray(iq[:, off:off + frames])))
    if isinstance(outs[0], tuple):
        return tuple(np.concatenate([o[i] for o in outs], axis=1) for i in range(len(outs[0])))
    return np.concatenate(outs, axis=1)


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
