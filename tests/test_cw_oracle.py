"""CW decoder front end on the CPU: the oracle's restatement (cw_front in
oracle/uhsdr_oracle.c) against the reference firmware's own CwDecode_RxProcessor / CW_Decode_exe
(tests/golden/cw_*.npz: Goertzel energy of every block, recorded by a pass-through around the
reference AudioFilter_GoertzelEnergy, and ads.CW_signal after every call), and the product's
Goertzel setup (uhsdr_rx_plan_build) against AudioFilter_CalcGoertzel's dumped values."""
import glob
import json
import os

import numpy as np
import pytest

import oracle
import uhsdr_amd as U
from golden_util import GOLDEN, assert_bitexact


def cw_files():
    return sorted(glob.glob(os.path.join(GOLDEN, "cw_*.npz")))


def load_cw(path):
    d = np.load(path)
    return {"iq": d["iq"], "signal": d["signal"], "energy": d["energy"], "args": json.loads(str(d["args"])),
            "setup": json.loads(str(d["setup"]))}


def cw_blocks(plan, n):
    ndc = 32 // plan.decimation_rate
    cpb = -(-plan.cw_blocksize // ndc)
    return (n // 32) // cpb


@pytest.mark.parametrize("path", cw_files(), ids=lambda p: os.path.basename(p)[3:-4])
def test_oracle_cw_matches_reference(path):
    g = load_cw(path)
    plan = U.build_plan(U.config_from_ref_args(g["args"]))
    assert plan.cw_enabled
    n = g["iq"].shape[1]
    _, _, sig, en = oracle.rx_process_cw(oracle.OracleRx(plan, g["iq"].shape[0]), g["iq"], cw_blocks(plan, n))
    assert en.shape == g["energy"].shape
    assert_bitexact(en, g["energy"], "Goertzel energy")
    np.testing.assert_array_equal(sig, g["signal"])


@pytest.mark.parametrize("path", cw_files(), ids=lambda p: os.path.basename(p)[3:-4])
def test_plan_goertzel_matches_reference(path):
    g = load_cw(path)
    p = U.build_plan(U.config_from_ref_args(g["args"]))
    mine = np.array([p.cw_r, p.cw_cos, p.cw_sin], np.float32).view(np.uint32)
    np.testing.assert_array_equal(mine, np.array(g["setup"]["cw_goertzel"], np.uint32))
    assert p.cw_blocksize == g["args"].get("cwblock", 88)


def test_cw_enabled_only_at_12k_in_cw_am_sam():
    on = lambda **k: U.build_plan(U.default_config(**k)).cw_enabled  # noqa: E731
    assert on(dmod_mode=U.DEMOD_CW, filter_path=4)
    assert on(dmod_mode=U.DEMOD_SAM, filter_path=70)
    assert not on(dmod_mode=U.DEMOD_USB, filter_path=48)
    assert not on(dmod_mode=U.DEMOD_FM, filter_path=1)
    p83 = U.build_plan(U.default_config(dmod_mode=U.DEMOD_AM, filter_path=83))
    assert p83.cw_enabled == (p83.decimated_freq == 12000)
