"""The STREAM schedule (uhsdr_rx_set_schedule, include/uhsdr.h): one rx_stream launch per call, the
front's waves and the rx_back wave pipeline on disjoint CUs, the decimated hand-off published per
32-frame call through progress words (write-through stores, sc1 polls).  Held bit-exact against the
CPU oracle like every other schedule:

  * every wide (Hilbert-first) SSB / CW / DIGI filter path it serves, ragged batches, several calls;
  * the launch flags (AGC off / hang, equaliser, key beep, clip flags, mcHF) and a reset;
  * the C2 shape (4096 x 256) with no synchronisation between calls, and the largest batch;
  * switching to and from it (and out of the pipelined mode) between calls;
  * no bounded hand-off poll ever gives up (uhsdr_rx_stream_timeouts).
"""
import json
import os

import numpy as np
import pytest

import oracle
import uhsdr_amd as U
from golden_util import assert_bitexact
from uhsdr_amd import _abi, synth

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
PATHS = json.load(open(os.path.join(HERE, "golden", "filter_paths.json")))
MODE_CW, MODE_SSB = 1, 2
SSB_PATHS = [p["index"] for p in PATHS if p["mode"] & (MODE_SSB | MODE_CW)]
MODES = {p["index"]: p["mode"] for p in PATHS}


def path_demod(path):
    m = MODES[path]
    if m & MODE_CW and (path % 2 == 0 or not m & MODE_SSB):
        return U.DEMOD_CW
    return U.DEMOD_LSB if path % 3 == 0 else U.DEMOD_USB


def stream_paths():
    """the paths whose plan STREAM serves: Hilbert-first, 12 ksps (rx_stream instances)"""
    out = []
    for path in SSB_PATHS:
        plan = U.build_plan(U.default_config(filter_path=path, dmod_mode=path_demod(path)))
        if not plan.use_decimated_iq and plan.decimation_rate == 4:
            out.append(path)
    return out


def run_stream(cfg, iq, N, sync_each=True, beep_at=None, beep_calls=0, clip=None, precision=None):
    import torch
    C, n, _ = iq.shape
    calls = n // N
    chain = U.RxChain(cfg, channels=C, frames=N)
    chain.set_schedule(U.SCHEDULE_STREAM)
    if precision is not None:
        chain.set_precision(precision)
    assert chain.schedule == U.SCHEDULE_STREAM
    if clip is not None:
        chain.set_clip_output(clip)
    xs = [torch.from_numpy(np.ascontiguousarray(iq[:, k * N:(k + 1) * N])).cuda() for k in range(calls)]
    audio = torch.empty((calls, C, N), dtype=torch.float32, device="cuda")
    dst = torch.empty((calls, C, N, 2), dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    for k in range(calls):
        if beep_at is not None and k == beep_at:
            chain.key_beep(beep_calls)
        chain.process(xs[k], audio[k], dst[k])
        if sync_each:
            torch.cuda.synchronize()
    chain.synchronize()
    assert chain.stream_timeouts() == 0
    chain.close()
    a = audio.permute(1, 0, 2).reshape(C, n).cpu().numpy()
    d = dst.permute(1, 0, 2, 3).reshape(C, n, 2).cpu().numpy()
    return a, d


def test_stream_paths_listed():
    assert stream_paths() == list(range(48, 55))


@pytest.mark.parametrize("N", [64, 256])
@pytest.mark.parametrize("path", list(range(48, 55)))
def test_stream_paths_match_oracle(cuda, path, N):
    cfg = U.default_config(filter_path=path, dmod_mode=path_demod(path))
    plan = U.build_plan(cfg)
    C = 130
    iq = synth.ssb_iq(np.arange(C), 0, 9 * N)
    a1, d = run_stream(cfg, iq, N, sync_each=(N == 64))
    ref_a1, ref_d = oracle.OracleRx(plan, C).process(iq, threads=8)
    assert_bitexact(a1, ref_a1, f"stream P{path} N={N}")
    np.testing.assert_array_equal(d, ref_d)


FLAG_CASES = [
    ("agc_off", dict(agc_mode=5)),
    ("agc_hang", dict(agc_mode=1, agc_hang_enable=1)),
    ("eq", dict(bass_gain=-8, treble_gain=6, dsp_active=_abi.DSP_MPEAK_ENABLE | _abi.DSP_MNOTCH_ENABLE)),
    ("lsb_p12k", dict(dmod_mode=U.DEMOD_LSB, iq_freq_mode=3)),
    ("no_shift", dict(iq_freq_mode=0)),
    ("iq_manual", dict(iq_gain_i=1.02, iq_gain_q=0.97, iq_phase_balance=-0.01)),
    ("iq_phase_pos", dict(iq_phase_balance=0.004)),
    ("mchf", dict(board=U.BOARD_MCHF, spkr_gain=24)),
]


@pytest.mark.parametrize("name,kw", FLAG_CASES, ids=[c[0] for c in FLAG_CASES])
def test_stream_flags_match_oracle(cuda, name, kw):
    cfg = U.default_config(**kw)
    plan = U.build_plan(cfg)
    C, N = 97, 128
    iq = synth.ssb_iq(np.arange(C), 0, 8 * N)
    a1, d = run_stream(cfg, iq, N, sync_each=False)
    ref_a1, ref_d = oracle.OracleRx(plan, C).process(iq, threads=8)
    assert_bitexact(a1, ref_a1, f"stream {name}")
    np.testing.assert_array_equal(d, ref_d)


def test_stream_key_beep_and_clip(cuda):
    import torch
    cfg = U.default_config()
    C, N = 70, 256
    iq = synth.ssb_iq(np.arange(C), 0, 6 * N)
    iq[3, 100] = (2 ** 31 - 1, 0)            # one full-scale frame: ADC clip on channel 3
    clip = torch.zeros((C,), dtype=torch.int32, device="cuda")
    a1, _ = run_stream(cfg, iq, N, sync_each=False, beep_at=2, beep_calls=N // 32 + 3, clip=clip)
    o = oracle.OracleRx(U.build_plan(cfg), C)
    ref = []
    for k in range(6):
        if k == 2:
            o.key_beep(N // 32 + 3)
        ref.append(o.process2(np.ascontiguousarray(iq[:, k * N:(k + 1) * N]))[0])
    assert_bitexact(a1, np.concatenate(ref, axis=1), "stream key beep")
    c = clip.cpu().numpy()
    assert c[3] & U.ADC_CLIP
    assert (c[np.arange(C) != 3] & U.ADC_CLIP == 0).all()


def test_stream_reset_restarts_epoch(cuda):
    """uhsdr_rx_reset zeroes the progress words with the epoch: calls after a reset (the words'
    values from before it would otherwise satisfy the polls early) match a fresh handle's."""
    import torch
    cfg = U.default_config()
    C, N = 150, 256
    iq = synth.ssb_iq(np.arange(C), 0, 4 * N)
    chain = U.RxChain(cfg, channels=C, frames=N, schedule=U.SCHEDULE_STREAM)
    audio = torch.empty((4, C, N), dtype=torch.float32, device="cuda")
    xs = [torch.from_numpy(np.ascontiguousarray(iq[:, k * N:(k + 1) * N])).cuda() for k in range(4)]
    for k in range(4):
        chain.process(xs[k], audio[k], None)        # epochs 1..4
    chain.reset()
    for k in range(4):
        chain.process(xs[k], audio[k], None)        # epochs 1..4 again, after the words were zeroed
    chain.synchronize()
    assert chain.stream_timeouts() == 0
    got = audio.permute(1, 0, 2).reshape(C, 4 * N).cpu().numpy()
    chain.close()
    ref, _ = oracle.OracleRx(U.build_plan(cfg), C).process(iq, threads=8)
    assert_bitexact(got, ref, "stream after reset")


def test_stream_c2_shape_unsynchronised(cuda):
    """The benchmarked shape, 4096 x 256, 10 calls back to back (the progress words reused across
    launches by epoch), the EXACT and FMA instances; every channel against the oracle (FMA: the
    north_star bound, 1e-5 normwise, against the EXACT run)."""
    cfg = U.default_config()
    C, N = 4096, 256
    iq = synth.ssb_iq(np.arange(C), 0, 10 * N)
    a1, d = run_stream(cfg, iq, N, sync_each=False)
    ref_a1, ref_d = oracle.OracleRx(U.build_plan(cfg), C).process(iq, threads=8)
    assert_bitexact(a1, ref_a1, "stream C2")
    np.testing.assert_array_equal(d, ref_d)
    fa, _ = run_stream(cfg, iq, N, sync_each=False, precision=U.PRECISION_FMA)
    err = np.abs(fa - a1).max(axis=1) / np.maximum(np.abs(a1).max(axis=1), 1e-30)
    assert err.max() <= 1e-5, err.max()


def test_stream_largest_batch_and_limits(cuda):
    import torch
    cfg = U.default_config()
    props = torch.cuda.get_device_properties(0)
    groups = props.multi_processor_count // 3                     # 2 front workgroups per group at least
    C = groups * 64
    N = 64
    iq = synth.ssb_iq(np.arange(C), 0, 8 * N)
    a1, _ = run_stream(cfg, iq, N, sync_each=False)
    pick = np.arange(0, C, 37)
    ref, _ = oracle.OracleRx(U.build_plan(cfg), len(pick)).process(np.ascontiguousarray(iq[pick]), threads=8)
    assert_bitexact(a1[pick], ref, f"stream C={C}")
    too_big = U.RxChain(cfg, channels=C + 64, frames=N)
    with pytest.raises(RuntimeError):
        too_big.set_schedule(U.SCHEDULE_STREAM)
    too_big.close()


@pytest.mark.parametrize("kw", [dict(iq_auto_correction=1), dict(iq_freq_mode=2),
                                dict(filter_path=35, dmod_mode=U.DEMOD_LSB),
                                dict(filter_path=70, dmod_mode=U.DEMOD_AM)],
                         ids=["iq_auto", "osc_6k", "narrow", "am"])
def test_stream_unsupported(cuda, kw):
    chain = U.RxChain(U.default_config(**kw), channels=64, frames=64)
    before = chain.schedule
    with pytest.raises(RuntimeError):
        chain.set_schedule(U.SCHEDULE_STREAM)
    assert chain.schedule == before
    chain.close()


def test_stream_switch_and_pipelined(cuda):
    """STREAM between the other schedules and after the pipelined mode, state carried across."""
    import torch
    cfg = U.default_config()
    C, N, calls = 200, 128, 12
    iq = synth.ssb_iq(np.arange(C), 0, N * calls)
    chain = U.RxChain(cfg, channels=C, frames=N)
    audio = torch.empty((calls, C, N), dtype=torch.float32, device="cuda")
    order = [U.SCHEDULE_STREAM, U.SCHEDULE_SPLIT_PIPE, U.SCHEDULE_STREAM, U.SCHEDULE_SPLIT_FUSED,
             U.SCHEDULE_STREAM, U.SCHEDULE_CHAIN]
    for k in range(calls):
        if k == 6:
            chain.set_pipelined(True)          # pipelined SPLIT calls, then STREAM joins the side stream
        chain.set_schedule(order[k % len(order)])
        chain.process(torch.from_numpy(np.ascontiguousarray(iq[:, k * N:(k + 1) * N])).cuda(), audio[k], None)
    chain.synchronize()
    assert chain.stream_timeouts() == 0
    got = audio.permute(1, 0, 2).reshape(C, calls * N).cpu().numpy()
    chain.close()
    ref, _ = oracle.OracleRx(U.build_plan(cfg), C).process(iq, threads=8)
    assert_bitexact(got, ref, "stream switch")
