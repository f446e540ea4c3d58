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
    iq, a0 = oracle.OracleTx(plan, g["audio"].shape[0]).process(g["audio"])
    np.testing.assert_array_equal(a0.view(np.uint32), g["a0"].view(np.uint32))
    np.testing.assert_array_equal(iq, g["iq"])
