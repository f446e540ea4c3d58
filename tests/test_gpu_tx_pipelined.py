"""TX pipelined mode (uhsdr_tx_set_pipelined: tx_iq on a side stream, two compressed-audio
hand-off buffers): calls enqueued back to back without a host sync give the same DAC frames and
compressed audio, bit for bit, as the serial mode and the CPU oracle -- across the hand-off
buffers' reuse, mode toggles mid-stream, and TUNE / DIGIQ switches on a DIGIQ handle."""
import numpy as np
import pytest

import oracle
import uhsdr_amd as U
from uhsdr_amd import synth

pytestmark = pytest.mark.gpu


def enqueue(cfg, audio, frames, schedule, tune=None):
    """schedule[k]: pipelined mode for call k; tune[k]: TUNE setting before call k (or None).
    Every call gets its own output buffers; one sync at the end."""
    import torch
    C, n, _ = audio.shape
    chain = U.TxChain(cfg, channels=C, frames=frames)
    d_in = [torch.from_numpy(np.ascontiguousarray(audio[:, k * frames:(k + 1) * frames])).cuda()
            for k in range(n // frames)]
    iqs = [torch.full((C, frames, 2), -7, dtype=torch.int32, device="cuda") for _ in d_in]
    a0s = [torch.zeros((C, frames), dtype=torch.float32, device="cuda") for _ in d_in]
    torch.cuda.synchronize()
    for k, x in enumerate(d_in):
        if schedule[k] != chain.pipelined:
            chain.set_pipelined(schedule[k])
        if tune is not None and tune[k] is not None:
            chain.set_tune(tune[k])
        chain.process(x, iqs[k], a0s[k])
    chain.join()
    torch.cuda.synchronize()
    chain.close()
    return (np.concatenate([t.cpu().numpy() for t in iqs], axis=1),
            np.concatenate([t.cpu().numpy() for t in a0s], axis=1))


CASES = [
    ("usb_p12k", dict(dmod_mode=0, iq_freq_mode=1)),
    ("lsb_m6k", dict(dmod_mode=1, iq_freq_mode=4)),
    ("am_p6k", dict(dmod_mode=U.DEMOD_AM, iq_freq_mode=3)),
    ("usb_off", dict(dmod_mode=0, iq_freq_mode=0)),
]


@pytest.mark.parametrize("name,kw", CASES, ids=[c[0] for c in CASES])
@pytest.mark.parametrize("frames", [64, 256])
def test_pipelined_matches_serial_and_oracle(cuda, name, kw, frames):
    cfg = U.default_tx_config(**kw)
    C, calls = 200, 9
    audio = synth.tx_audio(np.arange(C), 0, calls * frames)
    iq_s, a0_s = enqueue(cfg, audio, frames, [False] * calls)
    iq_p, a0_p = enqueue(cfg, audio, frames, [True] * calls)
    np.testing.assert_array_equal(iq_p, iq_s)
    np.testing.assert_array_equal(a0_p.view(np.uint32), a0_s.view(np.uint32))
    ref_iq, ref_a0 = oracle.OracleTx(U.build_tx_plan(cfg), C).process(audio, threads=8)
    np.testing.assert_array_equal(iq_p, ref_iq)
    np.testing.assert_array_equal(a0_p.view(np.uint32), ref_a0.view(np.uint32))


def test_pipelined_toggled_mid_stream(cuda):
    cfg = U.default_tx_config(dmod_mode=0, iq_freq_mode=1)
    C, frames, calls = 130, 128, 10
    audio = synth.tx_audio(np.arange(C), 0, calls * frames)
    iq_s, a0_s = enqueue(cfg, audio, frames, [False] * calls)
    sched = [True, True, True, False, True, False, False, True, True, True]
    iq_p, a0_p = enqueue(cfg, audio, frames, sched)
    np.testing.assert_array_equal(iq_p, iq_s)
    np.testing.assert_array_equal(a0_p.view(np.uint32), a0_s.view(np.uint32))


def test_pipelined_digiq_with_tune(cuda):
    """a DIGIQ handle runs the pass-through kernel, or the voice chain while TUNE is on: both
    orders of the DAC-frame writes hold in the pipelined mode"""
    cfg = U.default_tx_config(dmod_mode=0, iq_freq_mode=1, audio_source=U._abi.TX_AUDIO_DIGIQ)
    C, frames, calls = 96, 64, 8
    audio = (synth.tx_audio(np.arange(C), 0, calls * frames).astype(np.int64) * 7).astype(np.int32)
    tune = [None, U.TUNE_SINGLE, None, U.TUNE_OFF, None, U.TUNE_TWO, U.TUNE_OFF, None]
    iq_s, a0_s = enqueue(cfg, audio, frames, [False] * calls, tune)
    iq_p, a0_p = enqueue(cfg, audio, frames, [True] * calls, tune)
    np.testing.assert_array_equal(iq_p, iq_s)
    np.testing.assert_array_equal(a0_p.view(np.uint32), a0_s.view(np.uint32))
