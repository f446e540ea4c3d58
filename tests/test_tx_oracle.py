"""SSB and FM transmit (TxProcessor_Run, drivers/audio/tx_processor.c:891-1078): the product's TX setup
layer (uhsdr_tx_plan_build) and the CPU oracle's TX chain against the reference firmware's own
fixtures (tests/golden/tx_*.npz: codec mic frames in, IQ DAC frames out), bit for bit."""
import glob
import json
import os

import numpy as np
import pytest

import oracle
import uhsdr_amd as U

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def tx_files():
    return sorted(glob.glob(os.path.join(GOLDEN, "tx_*.npz")))


def load_tx(path):
    d = np.load(path)
    return {"name": os.path.basename(path)[:-4], "audio": d["audio"], "a0": d["a0"], "iq": d["iq"],
            "setup": json.loads(str(d["setup"])), "args": json.loads(str(d["args"]))}


def tx_events(args):
    """uhsdr_ref's run-time TX controls -> {call: [(what, value)]}: tune=t0:K:M (TUNE mode M on calls
    t0 .. t0+K-1), burst=t0:K (FM tone burst)"""
    ev = {}
    if "tune" in args:
        t0, k, m = (int(x) for x in str(args["tune"]).split(":"))
        ev.setdefault(t0, []).append(("tune", m))
        ev.setdefault(t0 + k, []).append(("tune", 0))
    if "burst" in args:
        b0, k = (int(x) for x in str(args["burst"]).split(":"))
        ev.setdefault(b0, []).append(("burst", 1))
        ev.setdefault(b0 + k, []).append(("burst", 0))
    return ev


def drive_tx(chain, process, audio, frames, args):
    """Feed audio [C][n][2] in calls of `frames`, applying the run-time events between calls
    (chain: set_tune / set_tone_burst); process(block) -> (iq, a0)."""
    ev = tx_events(args)
    cpl = frames // 32
    assert all(c % cpl == 0 for c in ev), "events must fall on call boundaries"
    iqs, a0s = [], []
    for off in range(0, audio.shape[1], frames):
        for what, v in ev.get(off // 32, []):
            (chain.set_tune if what == "tune" else chain.set_tone_burst)(v)
        iq, a0 = process(np.ascontiguousarray(audio[:, off:off + frames]))
        iqs.append(iq)
        a0s.append(a0)
    return np.concatenate(iqs, axis=1), np.concatenate(a0s, axis=1)


def fb(arr, n):
    return np.frombuffer(bytes(arr), dtype=np.uint32)[:n]


@pytest.mark.parametrize("path", tx_files(), ids=lambda p: os.path.basename(p)[:-4])
def test_tx_plan_matches_reference_setup(path):
    g = load_tx(path)
    s = g["setup"]
    p = U.build_tx_plan(U.tx_config_from_ref_args(g["args"]))
    np.testing.assert_array_equal(fb(p.lat_k, p.lat_stages), np.array(s["tx_k"], np.uint32))
    np.testing.assert_array_equal(fb(p.lat_v, p.lat_stages + 1), np.array(s["tx_v"], np.uint32))
    np.testing.assert_array_equal(fb(p.biquad, 15), np.array(s["tx_biquad"], np.uint32))
    hi, hq = np.array(s["tx_hilbert_i"], np.uint32), np.array(s["tx_hilbert_q"], np.uint32)
    if p.lsb:
        hi, hq = hq, hi
    np.testing.assert_array_equal(fb(p.hilbert_i, 201), hi)
    np.testing.assert_array_equal(fb(p.hilbert_q, 201), hq)
    assert np.array([p.alc_decay], np.float32).view(np.uint32)[0] == s["tx_alc"][0]


@pytest.mark.parametrize("path", tx_files(), ids=lambda p: os.path.basename(p)[:-4])
def test_tx_oracle_matches_reference(path):
    g = load_tx(path)
    plan = U.build_tx_plan(U.tx_config_from_ref_args(g["args"]))
    o = oracle.OracleTx(plan, g["audio"].shape[0])
    iq, a0 = drive_tx(o, o.process, g["audio"], 256, g["args"])
    np.testing.assert_array_equal(a0.view(np.uint32), g["a0"].view(np.uint32))
    np.testing.assert_array_equal(iq, g["iq"])
