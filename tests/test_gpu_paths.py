"""Parity breadth: every live FilterPathInfo entry (drivers/audio/audio_filter.c:147-922) in every
demodulator its mode mask admits, on the device through the C ABI, bit-exact against the CPU
oracle; and sampled channels of the full 1,048,576 x 64 EXACT batch that bench.py times.

The mode mask bits are FILTER_MODE_CW/SSB/AM/FM/SAM (audio_filter.h:77-85) -> 1/2/4/8/16.
SSB paths run USB and LSB; CW|SSB paths add CW; AM|SAM paths run AM and SAM (both sidebands);
the three FM paths run FM.  65 channels (one full wave + a ragged lane) x 512 frames in 128-frame
calls (four launches carrying state), both back-end kernels.
"""
import json
import os

import numpy as np
import pytest

import oracle
import uhsdr_amd as U
from golden_util import assert_bitexact
from uhsdr_amd import synth

HERE = os.path.dirname(os.path.abspath(__file__))
PATHS = json.load(open(os.path.join(HERE, "golden", "filter_paths.json")))

MODE_CW, MODE_SSB, MODE_AM, MODE_FM, MODE_SAM = 1, 2, 4, 8, 16


def path_cases():
    cases = []
    for p in PATHS:
        m, i = p["mode"], p["index"]
        if m & MODE_SSB:
            cases += [(i, U.DEMOD_USB), (i, U.DEMOD_LSB)]
        if m & MODE_CW:
            cases.append((i, U.DEMOD_CW))
        if m & MODE_AM:
            cases.append((i, U.DEMOD_AM))
        if m & MODE_SAM:
            cases.append((i, U.DEMOD_SAM))
        if m & MODE_FM:
            cases.append((i, U.DEMOD_FM))
    return cases


CASES = path_cases()
NAMES = {U.DEMOD_USB: "usb", U.DEMOD_LSB: "lsb", U.DEMOD_CW: "cw", U.DEMOD_AM: "am", U.DEMOD_SAM: "sam",
         U.DEMOD_FM: "fm"}


def case_config(path, mode):
    kw = dict(filter_path=path, dmod_mode=mode)
    if mode == U.DEMOD_FM:
        kw["fm_sql_threshold"] = 0
    return U.default_config(**kw)


def case_input(mode, C, n):
    ch = np.arange(C)
    if mode in (U.DEMOD_AM, U.DEMOD_SAM):
        return synth.am_iq(ch, 0, n)
    if mode == U.DEMOD_FM:
        return synth.fm_iq(ch, 0, n)
    return synth.ssb_iq(ch, 0, n, lsb=mode == U.DEMOD_LSB)


def test_sweep_covers_every_live_path():
    """86 live paths (index 0 is the 'off' entry), 139 (path, demodulator) pairs, all offered."""
    live = {i for i, _ in CASES}
    assert live == set(range(1, 87))
    assert len(CASES) == 2 * 62 + 32 + 2 * 21 + 3
    for path, mode in CASES:
        assert U.plan_supported(U.build_plan(case_config(path, mode))), (path, mode)


@pytest.mark.gpu
@pytest.mark.parametrize("path,mode", CASES, ids=[f"p{p}_{NAMES[m]}" for p, m in CASES])
def test_device_path_matches_oracle(cuda, back, path, mode):
    import torch
    C, n, N = 65, 512, 128
    cfg = case_config(path, mode)
    iq = case_input(mode, C, n)
    chain = U.RxChain(cfg, channels=C, frames=N)
    audio = torch.empty((C, N), dtype=torch.float32, device="cuda")
    dst = torch.empty((C, N, 2), dtype=torch.int32, device="cuda")
    a1 = np.empty((C, n), np.float32)
    d = np.empty((C, n, 2), np.int32)
    for off in range(0, n, N):
        chain.process(torch.from_numpy(np.ascontiguousarray(iq[:, off:off + N])).cuda(), audio, dst)
        torch.cuda.synchronize()
        a1[:, off:off + N] = audio.cpu().numpy()
        d[:, off:off + N] = dst.cpu().numpy()
    chain.close()
    ref_a1, ref_dst = oracle.OracleRx(U.build_plan(cfg), C).process(iq, threads=8)
    assert_bitexact(a1, ref_a1, f"P{path} {NAMES[mode]}")
    np.testing.assert_array_equal(d, ref_dst)
    assert np.abs(ref_a1).max() > 0 or mode == U.DEMOD_FM


@pytest.mark.gpu
def test_device_north_star_full_batch_sampled_channels(cuda):
    """The bench's north-star workload itself: 1,048,576 channels x 64-frame calls, EXACT, inputs
    generated on the device (synth.ssb_iq_torch, as bench.py does); 7 calls (past the AGC's
    6-call look-ahead ring) on sampled channels against the oracle fed the same input rows."""
    import torch
    cfg = U.default_config()
    C, N, calls = 1048576, 64, 7
    pick = np.array([0, 1, 63, 64, 65535, 262144, 524287, 777777, 1048512, 1048575])
    tp = torch.from_numpy(pick).cuda()
    chain = U.RxChain(cfg, channels=C, frames=N)
    assert chain.precision == U.PRECISION_EXACT
    audio = torch.empty((C, N), dtype=torch.float32, device="cuda")
    ins, outs = [], []
    for k in range(calls):
        x = synth.ssb_iq_torch(0, C, k * N, N, "cuda")
        chain.process(x, audio, None)
        torch.cuda.synchronize()
        ins.append(x[tp].cpu().numpy())
        outs.append(audio[tp].cpu().numpy())
        del x
    chain.close()
    iq = np.concatenate(ins, axis=1)
    got = np.concatenate(outs, axis=1)
    ref, _ = oracle.OracleRx(U.build_plan(cfg), len(pick)).process(iq)
    assert_bitexact(got, ref, "north-star 1M x 64 sampled")
    assert np.abs(got[:, N:]).max() > 100
