"""TX FMA precision (uhsdr_tx_set_precision): the 201-tap Hilbert pair with fused MACs.

Tolerance (north_star): per channel, max |iq_fma - iq_ref| / max |iq_ref| <= 1e-5 over the DAC
frames, for every SSB / AM mode and frequency translation; the compressed audio (a_buffer[0], the
voice chain before the pair) stays bit-identical; FM (no Hilbert pair) is bit-identical; switching
back to EXACT mid-stream gives bit-identical frames again (the pair's history holds its inputs,
which precision does not touch); the pipelined mode gives the serial mode's FMA frames bit for bit.
The reference is the CPU oracle (oracle/uhsdr_oracle.c, bit-exact to the reference build)."""
import numpy as np
import pytest

import oracle
import uhsdr_amd as U
from uhsdr_amd import synth

pytestmark = pytest.mark.gpu

TOL = 1e-5


def run(cfg, audio, frames, precision, pipelined=False, schedule=None):
    """schedule[k]: precision for call k (overrides `precision`); outputs of every call"""
    import torch
    C, n, _ = audio.shape
    chain = U.TxChain(cfg, channels=C, frames=frames)
    if pipelined:
        chain.set_pipelined(True)
    calls = n // frames
    d_in = [torch.from_numpy(np.ascontiguousarray(audio[:, k * frames:(k + 1) * frames])).cuda() for k in range(calls)]
    iqs = [torch.empty((C, frames, 2), dtype=torch.int32, device="cuda") for _ in range(calls)]
    a0s = [torch.zeros((C, frames), dtype=torch.float32, device="cuda") for _ in range(calls)]
    for k in range(calls):
        p = schedule[k] if schedule is not None else precision
        if p != chain.precision:
            chain.set_precision(p)
        chain.process(d_in[k], iqs[k], a0s[k])
    chain.join()
    torch.cuda.synchronize()
    chain.close()
    return (np.concatenate([t.cpu().numpy() for t in iqs], axis=1),
            np.concatenate([t.cpu().numpy() for t in a0s], axis=1))


def normwise(iq, ref):
    """per channel max|diff| / max|ref| (channels with an all-zero reference must match exactly)"""
    d = np.abs(iq.astype(np.int64) - ref.astype(np.int64)).reshape(len(ref), -1).max(axis=1)
    m = np.abs(ref.astype(np.int64)).reshape(len(ref), -1).max(axis=1)
    assert np.all(d[m == 0] == 0)
    return float(np.max(np.where(m > 0, d / np.maximum(m, 1), 0.0)))


# every SSB / AM mode with each I/Q frequency translation (AM needs one: uhsdr_tx_plan_build)
CASES = [(m, n, q) for m, n in [(U.DEMOD_USB, "usb"), (U.DEMOD_LSB, "lsb"), (U.DEMOD_AM, "am")]
         for q in range(5) if not (m == U.DEMOD_AM and q == 0)]


@pytest.mark.parametrize("mode,name,iqmode", CASES, ids=[f"{c[1]}-{c[2]}" for c in CASES])
def test_fma_within_tolerance(cuda, mode, name, iqmode):
    cfg = U.default_tx_config(dmod_mode=mode, iq_freq_mode=iqmode)
    C, frames = 96, 256
    audio = synth.tx_audio(np.arange(C), 0, 4 * frames)
    iq, a0 = run(cfg, audio, frames, U.PRECISION_FMA)
    ref_iq, ref_a0 = oracle.OracleTx(U.build_tx_plan(cfg), C).process(audio, threads=8)
    np.testing.assert_array_equal(a0.view(np.uint32), ref_a0.view(np.uint32))
    err = normwise(iq, ref_iq)
    print(f"tx fma {name} iqmode {iqmode}: max normwise {err:.3e}")
    assert err <= TOL
    assert not np.array_equal(iq, ref_iq), "FMA precision did not reach the kernel"


def test_fma_fm_is_exact(cuda):
    cfg = U.default_tx_config(dmod_mode=U.DEMOD_FM, iq_freq_mode=3, fm_subaudible_tone=7)
    C = 70
    audio = synth.tx_audio(np.arange(C), 0, 512)
    iq, _ = run(cfg, audio, 128, U.PRECISION_FMA)
    ref_iq, _ = oracle.OracleTx(U.build_tx_plan(cfg), C).process(audio, threads=8)
    np.testing.assert_array_equal(iq, ref_iq)


def test_fma_toggle_mid_stream(cuda):
    cfg = U.default_tx_config(dmod_mode=U.DEMOD_USB, iq_freq_mode=1)
    C, frames = 65, 128
    audio = synth.tx_audio(np.arange(C), 0, 6 * frames)
    sched = [U.PRECISION_EXACT, U.PRECISION_FMA, U.PRECISION_FMA, U.PRECISION_EXACT, U.PRECISION_FMA, U.PRECISION_EXACT]
    iq, _ = run(cfg, audio, frames, None, schedule=sched)
    ref_iq, _ = oracle.OracleTx(U.build_tx_plan(cfg), C).process(audio, threads=8)
    for k, p in enumerate(sched):
        s = slice(k * frames, (k + 1) * frames)
        if p == U.PRECISION_EXACT:
            np.testing.assert_array_equal(iq[:, s], ref_iq[:, s])
        else:
            assert normwise(iq[:, s], ref_iq[:, s]) <= TOL


def test_fma_pipelined_matches_serial(cuda):
    cfg = U.default_tx_config(dmod_mode=U.DEMOD_LSB, iq_freq_mode=4)
    C, frames = 200, 256
    audio = synth.tx_audio(np.arange(C), 0, 6 * frames)
    iq_s, a0_s = run(cfg, audio, frames, U.PRECISION_FMA)
    iq_p, a0_p = run(cfg, audio, frames, U.PRECISION_FMA, pipelined=True)
    np.testing.assert_array_equal(iq_p, iq_s)
    np.testing.assert_array_equal(a0_p.view(np.uint32), a0_s.view(np.uint32))


def test_precision_argument_errors(cuda):
    chain = U.TxChain(U.default_tx_config(), channels=4, frames=64)
    try:
        assert chain.precision == U.PRECISION_EXACT
        with pytest.raises(Exception):
            chain.set_precision(7)
        assert chain.precision == U.PRECISION_EXACT
    finally:
        chain.close()
