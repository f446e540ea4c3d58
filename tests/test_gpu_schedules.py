"""Kernel schedules of a call (uhsdr_rx_set_schedule, include/uhsdr.h): every schedule computes
the same binary32 sequence, so each is held bit-exact against the CPU oracle on the call sizes
where its kernels differ from the others':

  * SPLIT_FUSED runs rx_back_fused (every back-end stage per sample in one wave per 64 channels);
  * CHAIN runs rx_chain (front passes + fused back end per wave, the hand-off in LDS), whose
    front passes and LDS-fed back end only run here and in the 1M-channel check.

Every SSB / CW / DIGI filter path (the families rx_chain covers, audio_filter.c:
147-922) in 16-decimated-sample calls (64 frames at 12 ksps, 32 at 24 ksps), ragged channel
counts, several calls carrying state; plus the schedule API's own rules.
"""
import json
import os

import numpy as np
import pytest

import oracle
import uhsdr_amd as U
from golden_util import assert_bitexact
from uhsdr_amd import _abi, synth

HERE = os.path.dirname(os.path.abspath(__file__))
PATHS = json.load(open(os.path.join(HERE, "golden", "filter_paths.json")))
MODE_CW, MODE_SSB = 1, 2

SSB_PATHS = [p["index"] for p in PATHS if p["mode"] & (MODE_SSB | MODE_CW)]
MODES = {p["index"]: p["mode"] for p in PATHS}


def path_demod(path):
    """CW on the CW paths (and every other CW|SSB one), else LSB / USB alternating"""
    m = MODES[path]
    if m & MODE_CW and (path % 2 == 0 or not m & MODE_SSB):
        return U.DEMOD_CW
    return U.DEMOD_LSB if path % 3 == 0 else U.DEMOD_USB
SCHED = {"pipe": U.SCHEDULE_SPLIT_PIPE, "fused": U.SCHEDULE_SPLIT_FUSED, "chain": U.SCHEDULE_CHAIN}


def short_frames(plan):
    """a launch of 16 decimated samples per channel"""
    return 16 * plan.decimation_rate


def run(cfg, C, frames, calls, schedule, gen=synth.ssb_iq, precision=None):
    import torch
    iq = gen(np.arange(C), 0, frames * calls)
    chain = U.RxChain(cfg, channels=C, frames=frames, schedule=schedule)
    if precision is not None:
        chain.set_precision(precision)
    audio = torch.empty((C, frames), dtype=torch.float32, device="cuda")
    dst = torch.empty((C, frames, 2), dtype=torch.int32, device="cuda")
    a1 = np.empty((C, frames * calls), np.float32)
    d = np.empty((C, frames * calls, 2), np.int32)
    for k in range(calls):
        blk = np.ascontiguousarray(iq[:, k * frames:(k + 1) * frames])
        chain.process(torch.from_numpy(blk).cuda(), audio, dst)
        torch.cuda.synchronize()
        a1[:, k * frames:(k + 1) * frames] = audio.cpu().numpy()
        d[:, k * frames:(k + 1) * frames] = dst.cpu().numpy()
    got = chain.schedule
    chain.close()
    return iq, a1, d, got


def test_every_ssb_cw_path_listed():
    assert len(SSB_PATHS) == 62
    for path in SSB_PATHS:
        plan = U.build_plan(U.default_config(filter_path=path, dmod_mode=path_demod(path)))
        assert plan.decimation_rate in (2, 4)
        assert U.plan_supported(plan)


@pytest.mark.gpu
@pytest.mark.parametrize("sched", ["fused", "chain"])
@pytest.mark.parametrize("path", SSB_PATHS)
def test_short_calls_match_oracle(cuda, path, sched):
    cfg = U.default_config(filter_path=path, dmod_mode=path_demod(path))
    plan = U.build_plan(cfg)
    C, N = 130, short_frames(plan)
    iq, a1, d, got = run(cfg, C, N, 9, SCHED[sched])        # 9 calls: past the AGC's 6-call ring
    assert got == SCHED[sched]
    ref_a1, ref_d = oracle.OracleRx(plan, C).process(iq, threads=8)
    assert_bitexact(a1, ref_a1, f"P{path} {sched} N={N}")
    np.testing.assert_array_equal(d, ref_d)


# launch flags the back ends carry as template arguments or per-lane selects, on short calls
FLAG_CASES = [
    ("agc_off", dict(agc_mode=5)),
    ("agc_hang", dict(agc_mode=1, agc_hang_enable=1)),
    ("iq_auto", dict(iq_auto_correction=1)),
    ("m6k", dict(iq_freq_mode=3)),
    ("eq", dict(bass_gain=-8, treble_gain=6, dsp_active=_abi.DSP_MPEAK_ENABLE | _abi.DSP_MNOTCH_ENABLE)),
]


@pytest.mark.gpu
@pytest.mark.parametrize("sched", ["fused", "chain"])
@pytest.mark.parametrize("name,kw", FLAG_CASES, ids=[c[0] for c in FLAG_CASES])
def test_short_call_flags(cuda, sched, name, kw):
    cfg = U.default_config(**kw)
    plan = U.build_plan(cfg)
    C, N = 97, 64
    iq, a1, d, got = run(cfg, C, N, 8, SCHED[sched])
    assert got == SCHED[sched]
    ref_a1, ref_d = oracle.OracleRx(plan, C).process(iq, threads=8)
    assert_bitexact(a1, ref_a1, f"{name} {sched}")
    np.testing.assert_array_equal(d, ref_d)


@pytest.mark.gpu
def test_short_calls_cw_decoder_outputs(cuda):
    """CW decoder front end outputs (Goertzel energy per block, signal state per call) from the
    fused back end and rx_chain equal the wave pipeline's (itself pinned to the reference,
    tests/test_gpu_cw.py)."""
    import torch
    cfg = U.default_config(filter_path=4, dmod_mode=U.DEMOD_CW)
    C, N, calls = 70, 64, 12
    iq = synth.ssb_iq(np.arange(C), 0, N * calls)
    outs = {}
    for s in ("pipe", "fused", "chain"):
        chain = U.RxChain(cfg, channels=C, frames=N, schedule=SCHED[s])
        sig = torch.zeros((C, N // 32), dtype=torch.uint8, device="cuda")
        en = torch.zeros((C, max(chain.cw_blocks_max, 1)), dtype=torch.float32, device="cuda")
        chain.set_cw_outputs(sig, en)
        audio = torch.empty((C, N), dtype=torch.float32, device="cuda")
        rs, re = [], []
        for k in range(calls):
            chain.process(torch.from_numpy(np.ascontiguousarray(iq[:, k * N:(k + 1) * N])).cuda(), audio, None)
            torch.cuda.synchronize()
            rs.append(sig.cpu().numpy().copy())
            re.append(en[:, :chain.cw_blocks_last].cpu().numpy().copy())
        chain.close()
        outs[s] = (np.concatenate(rs, axis=1), np.concatenate(re, axis=1))
    for s in ("fused", "chain"):
        np.testing.assert_array_equal(outs[s][0], outs["pipe"][0])
        assert_bitexact(outs[s][1], outs["pipe"][1], f"cw energy {s}")
    assert outs["pipe"][1].size > 0


@pytest.mark.gpu
def test_schedule_api(cuda):
    cfg = U.default_config()
    small = U.RxChain(cfg, channels=4096, frames=256)
    assert small.schedule == U.SCHEDULE_SPLIT_PIPE                 # AUTO below 131072 channels
    small.set_schedule(U.SCHEDULE_CHAIN)
    assert small.schedule == U.SCHEDULE_CHAIN
    small.set_schedule(U.SCHEDULE_AUTO)
    assert small.schedule == U.SCHEDULE_SPLIT_PIPE
    with pytest.raises(RuntimeError):
        small.set_schedule(7)
    small.set_front_block(16)
    assert small.schedule == U.SCHEDULE_SPLIT_PIPE
    small.close()
    big = U.RxChain(cfg, channels=131072, frames=64)
    assert big.schedule == U.SCHEDULE_SPLIT_FUSED                  # AUTO from 131072 channels on
    big.close()
    am = U.RxChain(U.default_config(filter_path=70, dmod_mode=U.DEMOD_AM), channels=64, frames=64)
    with pytest.raises(RuntimeError):
        am.set_schedule(U.SCHEDULE_CHAIN)                          # AM / SAM: no rx_chain
    assert am.schedule == U.SCHEDULE_SPLIT_PIPE
    am.close()
    long_calls = U.RxChain(cfg, channels=64, frames=2048)          # two front launches per call
    with pytest.raises(RuntimeError):
        long_calls.set_schedule(U.SCHEDULE_CHAIN)
    long_calls.close()


@pytest.mark.gpu
@pytest.mark.parametrize("sched", ["pipe", "fused", "chain"])
def test_schedule_switch_mid_stream(cuda, sched):
    """Switching schedule between calls (state carried across kernels) stays bit-exact."""
    import torch
    cfg = U.default_config()
    C, N, calls = 200, 64, 10
    iq = synth.ssb_iq(np.arange(C), 0, N * calls)
    chain = U.RxChain(cfg, channels=C, frames=N)
    audio = torch.empty((C, N), dtype=torch.float32, device="cuda")
    got = []
    order = ["pipe", "fused", "chain"]
    for k in range(calls):
        chain.set_schedule(SCHED[sched] if k % 2 == 0 else SCHED[order[k % 3]])
        chain.process(torch.from_numpy(np.ascontiguousarray(iq[:, k * N:(k + 1) * N])).cuda(), audio, None)
        torch.cuda.synchronize()
        got.append(audio.cpu().numpy())
    chain.close()
    ref, _ = oracle.OracleRx(U.build_plan(cfg), C).process(iq, threads=8)
    assert_bitexact(np.concatenate(got, axis=1), ref, f"switch {sched}")
