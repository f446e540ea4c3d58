"""Status side outputs of the RX chain: the ADC clip indicators (audio_driver.c:2660-2676) and the
twin-peaks I/Q fault detector (AudioDriver_RxHandleTwinpeaks, :2173-2248).

Fixtures tests/golden/st_*.npz come from the reference firmware compiled for x86
(tests/golden/make_golden.py, uhsdr_ref out_clip= / out_tp= / uiperiod=): per 32-frame call the
clip flags (read and cleared after every call) and ts.twinpeaks_tested, with the UI's codec
restart acknowledgement every `uiperiod` calls, over >1000-call settling periods and four restart
cycles.  The input is synth.status_iq, regenerated here and checked against the stored crc32.

CPU: the oracle restatement against the fixtures, call by call.  GPU: the device through the C
ABI in launches of `uiperiod` calls -- the clip flags OR-ed over a launch, the twin-peaks state
after it, the restart acknowledged between launches -- and the audio at both ends of the run.
"""
import glob
import json
import os
import zlib

import numpy as np
import pytest

import oracle
import uhsdr_amd as U
from golden_util import assert_bitexact
from uhsdr_amd import synth

HERE = os.path.dirname(os.path.abspath(__file__))
FILES = sorted(glob.glob(os.path.join(HERE, "golden", "st_*.npz")))
NAMES = [os.path.basename(f)[3:-4] for f in FILES]


def load_case(path):
    g = dict(np.load(path, allow_pickle=False))
    args = json.loads(str(g["args"]))
    n = int(g["frames"])
    iq = synth.status_iq(np.arange(g["tp"].shape[0]), 0, n)
    assert zlib.crc32(np.ascontiguousarray(iq).tobytes()) == int(g["iq_crc32"]), "synth.status_iq drifted"
    return g, args, iq


def test_status_fixtures_present():
    assert len(FILES) >= 3
    g = np.load(FILES[0], allow_pickle=False)
    # the fixtures exercise every outcome: DONE, codec restart, UNCORRECTABLE, and every clip bit
    outcomes = set()
    bits = 0
    for f in FILES:
        g = np.load(f, allow_pickle=False)
        outcomes |= set(np.unique(g["tp"]).tolist())
        bits |= int(np.bitwise_or.reduce(g["clip"].ravel()))
    assert {U.TWINPEAKS_SAMPLING, U.TWINPEAKS_DONE, U.TWINPEAKS_WAIT, U.TWINPEAKS_UNCORRECTABLE,
            U.TWINPEAKS_CODEC_RESTART} <= outcomes
    assert bits == U.ADC_CLIP | U.ADC_HALF_CLIP | U.ADC_QUARTER_CLIP


@pytest.mark.parametrize("path", FILES, ids=NAMES)
def test_oracle_status_matches_reference(path):
    g, args, iq = load_case(path)
    cfg = U.config_from_ref_args(args)
    P = int(args.get("uiperiod", 1))
    C, calls = g["tp"].shape
    o = oracle.OracleRx(U.build_plan(cfg), C)
    tp = np.empty((C, calls), np.int32)
    clip = np.empty((C, calls), np.int32)
    a1 = np.empty((C, iq.shape[1]), np.float32)
    for k in range(calls):
        a1[:, 32 * k:32 * k + 32], _ = o.process(np.ascontiguousarray(iq[:, 32 * k:32 * k + 32]))
        clip[:, k], tp[:, k] = o.status(rearm=(k + 1) % P == 0)
    np.testing.assert_array_equal(clip, g["clip"])
    np.testing.assert_array_equal(tp, g["tp"])
    assert_bitexact(a1[:, :2048], g["a1_head"], "a1 head")
    assert_bitexact(a1[:, -2048:], g["a1_tail"], "a1 tail")


@pytest.mark.gpu
@pytest.mark.parametrize("path", FILES, ids=NAMES)
def test_device_status_matches_reference(cuda, path):
    import torch
    g, args, iq = load_case(path)
    cfg = U.config_from_ref_args(args)
    P = int(args.get("uiperiod", 1))
    C, calls = g["tp"].shape
    N = 32 * P
    chain = U.RxChain(cfg, channels=C, frames=N)
    clip = torch.zeros(C, dtype=torch.int32, device="cuda")
    tpd = torch.empty(C, dtype=torch.int32, device="cuda")
    chain.set_clip_output(clip)
    audio = torch.empty((C, N), dtype=torch.float32, device="cuda")
    dev_iq = torch.from_numpy(iq).cuda()
    a1 = np.empty((C, iq.shape[1]), np.float32)
    for L in range(calls // P):
        chain.process(dev_iq[:, L * N:(L + 1) * N].contiguous(), audio, None)
        chain.twinpeaks_state(tpd)
        torch.cuda.synchronize()
        a1[:, L * N:(L + 1) * N] = audio.cpu().numpy()
        want_clip = np.bitwise_or.reduce(g["clip"][:, L * P:(L + 1) * P].astype(np.int32), axis=1)
        np.testing.assert_array_equal(clip.cpu().numpy(), want_clip, err_msg=f"clip flags, launch {L}")
        np.testing.assert_array_equal(tpd.cpu().numpy(), g["tp"][:, (L + 1) * P - 1], err_msg=f"twinpeaks, launch {L}")
        clip.zero_()
        chain.twinpeaks_rearm()
    chain.close()
    assert_bitexact(a1[:, :2048], g["a1_head"], "a1 head")
    assert_bitexact(a1[:, -2048:], g["a1_tail"], "a1 tail")


@pytest.mark.gpu
def test_device_twinpeaks_reset_and_no_auto_iq(cuda):
    """reset() returns every channel to WAIT; without auto I/Q the detector never runs (the
    reference calls it only from the automatic branch, audio_driver.c:2271-2300), and with no
    clip output set nothing is written."""
    import torch
    C, N = 70, 1024
    iq = synth.status_iq(np.arange(C), 0, N)
    tpd = torch.empty(C, dtype=torch.int32, device="cuda")
    chain = U.RxChain(U.default_config(), channels=C, frames=N)
    chain.process(torch.from_numpy(iq).cuda())
    chain.twinpeaks_state(tpd)
    torch.cuda.synchronize()
    assert (tpd.cpu().numpy() == U.TWINPEAKS_WAIT).all()
    chain.close()
    chain = U.RxChain(U.default_config(iq_auto_correction=1), channels=C, frames=N)
    for _ in range(40):                        # 1280 calls: past the 1000-call settling
        chain.process(torch.from_numpy(iq).cuda())
    chain.twinpeaks_state(tpd)
    torch.cuda.synchronize()
    assert (tpd.cpu().numpy() != U.TWINPEAKS_WAIT).all()
    chain.reset()
    chain.twinpeaks_state(tpd)
    torch.cuda.synchronize()
    assert (tpd.cpu().numpy() == U.TWINPEAKS_WAIT).all()
    chain.close()
