"""Every configuration tools/bench_configs.py times, checked at the size it is timed at (the
kernels' launch shapes there -- grid, persistent waves walking several channel groups, the
larger-batch kernel choices -- never run at the ragged test sizes of the other files): the
whole batch is fed distinct inputs, and sampled channels (first, wave edges, last) are held
against the CPU oracle fed the same rows.

  * C5 513-tap FIR (uhsdr_fir_*, arm_fir_f32 semantics, CMSIS FilteringFunctions/arm_fir_f32.c:
    482-560): 131072 channels x 256 (the persistent MFMA kernel walks >= 2 channel groups per
    wave there) and 16384; EXACT bit-exact, MFMA within 1e-5 normwise;
  * C4 FM-RX P1 (AudioDriver_DemodFM, audio_driver.c:1544-1737) and SSB-TX (TxProcessor_Run,
    tx_processor.c:891-1078): 32768 channels x 256, bit-exact;
  * C5 CW P4 with the CW decoder front end (audio_driver.c:2539-2557, cw_decoder.c:383-397):
    131072 channels x 256, bit-exact audio and decoder outputs.
"""
import os

import numpy as np
import pytest

import oracle
import uhsdr_amd as U
from golden_util import assert_bitexact
from test_cw_oracle import cw_blocks
from uhsdr_amd import synth

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def picks(C):
    return np.unique(np.array([0, 1, 63, 64, 65, 4095, 4096, C // 2 - 1, C // 2, C - 65, C - 64, C - 2, C - 1]))


def gen_rows(fn, C, start, n, chunk=16384):
    """fn(channels, start, n) for every channel, on the device (built in chunks)"""
    import torch
    out = []
    for c0 in range(0, C, chunk):
        out.append(torch.from_numpy(fn(np.arange(c0, min(C, c0 + chunk)), start, n)).cuda())
    return torch.cat(out, 0).contiguous()


def normwise(got, ref):
    return float(np.max(np.abs(got.astype(np.float64) - ref), axis=-1).max() /
                 max(float(np.abs(ref).max()), 1e-30))


@pytest.mark.parametrize("mode", [U.fir.EXACT, U.fir.MFMA], ids=["exact", "mfma"])
@pytest.mark.parametrize("C", [16384, 131072])
def test_fir_bench_size(cuda, mode, C):
    import torch
    B, calls = 256, 2
    taps = np.load(os.path.join(GOLD, "fir513_kaiser.npy"))
    pk = picks(C)
    tp = torch.from_numpy(pk).cuda()
    g = torch.Generator(device="cuda").manual_seed(513 + C)
    fir = U.FirBatch(taps, C, B, mode)
    y = torch.empty((C, B), dtype=torch.float32, device="cuda")
    xs, ys = [], []
    for k in range(calls):
        x = torch.randn((C, B), generator=g, device="cuda").mul_(1000.0)
        fir.process(x, y)
        torch.cuda.synchronize()
        xs.append(x[tp].cpu().numpy())
        ys.append(y[tp].cpu().numpy())
        assert bool(torch.isfinite(y).all().item())
        del x
    fir.close()
    o = oracle.OracleFir(taps, len(pk))
    ref = np.concatenate([o.process(xk) for xk in xs], axis=1)
    got = np.concatenate(ys, axis=1)
    if mode == U.fir.EXACT:
        np.testing.assert_array_equal(got.view(np.uint32), ref.view(np.uint32))
    else:
        assert normwise(got, ref) < 1e-5


def rx_bench_size(cfg, C, N, calls, gen, cw=False, pipelined=False):
    """`calls` launches over C channels.  Serial: one call at a time, outputs copied back after
    each.  Pipelined (how tools/bench_configs.py / bench.py time it): every call enqueued back to
    back with no host sync or join in between -- rx_front of call k+1 overlapping rx_back of call
    k, the hand-off buffers rotating -- into per-call outputs, one join at the end."""
    import torch
    pk = picks(C)
    tp = torch.from_numpy(pk).cuda()
    chain = U.RxChain(cfg, channels=C, frames=N)
    if pipelined:
        chain.set_pipelined(True)
    nbuf = calls if pipelined else 1
    audio = [torch.empty((C, N), dtype=torch.float32, device="cuda") for _ in range(nbuf)]
    dst = [torch.empty((C, N, 2), dtype=torch.int32, device="cuda") for _ in range(nbuf)]
    if cw:
        sig = torch.zeros((C, N // 32), dtype=torch.uint8, device="cuda")
        en = torch.zeros((C, max(1, chain.cw_blocks_max)), dtype=torch.float32, device="cuda")
        chain.set_cw_outputs(sig, en)
    ins, outs, douts, sigs, ens = [], [], [], [], []
    xs = [gen_rows(gen, C, k * N, N) for k in range(calls)] if pipelined else None
    for k in range(calls):
        x = xs[k] if pipelined else gen_rows(gen, C, k * N, N)
        b = k % nbuf
        chain.process(x, audio[b], dst[b])
        if pipelined:
            continue
        torch.cuda.synchronize()
        assert bool(torch.isfinite(audio[0]).all().item())
        ins.append(x[tp].cpu().numpy())
        outs.append(audio[0][tp].cpu().numpy())
        douts.append(dst[0][tp].cpu().numpy())
        if cw:
            sigs.append(sig[tp].cpu().numpy())
            ens.append(en[tp, :chain.cw_blocks_last].cpu().numpy())
        del x
    if pipelined:
        assert not cw
        chain.join()
        torch.cuda.synchronize()
        for k in range(calls):
            assert bool(torch.isfinite(audio[k]).all().item())
            ins.append(xs[k][tp].cpu().numpy())
            outs.append(audio[k][tp].cpu().numpy())
            douts.append(dst[k][tp].cpu().numpy())
        del xs
    chain.close()
    iq = np.concatenate(ins, axis=1)
    o = oracle.OracleRx(U.build_plan(cfg), len(pk))
    if cw:
        ref_a, ref_d, ref_sig, ref_en = oracle.rx_process_cw(o, iq, cw_blocks(o.plan, iq.shape[1]), threads=8)
        np.testing.assert_array_equal(np.concatenate(sigs, 1), ref_sig)
        assert_bitexact(np.concatenate(ens, 1), ref_en, "CW energy")
    else:
        ref_a, ref_d = o.process(iq, threads=8)
    assert_bitexact(np.concatenate(outs, 1), ref_a, f"{C} x {N}{' pipelined' if pipelined else ''}")
    np.testing.assert_array_equal(np.concatenate(douts, 1), ref_d)
    return ref_a


@pytest.mark.parametrize("pipelined", [False, True], ids=["serial", "pipelined"])
@pytest.mark.parametrize("sql", [12, 0])
def test_fm_rx_bench_size(cuda, sql, pipelined):
    """squelch 12 is the bench's setting.  The receiver starts squelched and decides every 200
    32-frame calls (audio_driver.c:475, :1600-1640), so the output is muted until then; with
    squelch 0 the first decision opens it, and 28 launches (224 calls) compare the demodulated
    audio itself after it."""
    cfg = U.default_config(filter_path=1, dmod_mode=U.DEMOD_FM, fm_sql_threshold=sql)
    ref = rx_bench_size(cfg, 32768, 256, 3 if sql else 28, synth.fm_iq, pipelined=pipelined)
    assert sql or np.abs(ref).max() > 0


@pytest.mark.parametrize("name,kw", [("sam_p70", dict(dmod_mode=U.DEMOD_SAM)), ("am_p70", dict(dmod_mode=U.DEMOD_AM))])
def test_c3_bench_size(cuda, name, kw):
    """C3 as tools/bench_configs.py times it: 32768 channels x 1024-frame calls (two 512-frame
    front launches per call, one channel per wave, padded pair window; the SAM PLL,
    audio_driver.c:1990-2166), 3 calls."""
    cfg = U.default_config(filter_path=70, **kw)
    ref = rx_bench_size(cfg, 32768, 1024, 3, synth.am_iq)
    assert np.abs(ref).max() > 0


def test_cw_bench_size(cuda):
    cfg = U.default_config(filter_path=4, dmod_mode=U.DEMOD_CW)
    ref = rx_bench_size(cfg, 131072, 256, 2, synth.cw_iq, cw=True)
    assert np.abs(ref).max() > 0


@pytest.mark.parametrize("pipelined", [False, True], ids=["serial", "pipelined"])
def test_ssb_tx_bench_size(cuda, pipelined):
    """SSB-TX at the C4 per-GPU share; pipelined is how tools/bench_configs.py times it (tx_voice2
    of call k+1 beside tx_iq of call k)."""
    import torch
    C, N, calls = 32768, 256, 5
    cfg = U.default_tx_config()
    pk = picks(C)
    tp = torch.from_numpy(pk).cuda()
    tx = U.TxChain(cfg, channels=C, frames=N)
    if pipelined:
        tx.set_pipelined(True)
    nbuf = calls if pipelined else 1
    iq = [torch.empty((C, N, 2), dtype=torch.int32, device="cuda") for _ in range(nbuf)]
    a0 = [torch.empty((C, N), dtype=torch.float32, device="cuda") for _ in range(nbuf)]
    xs = [gen_rows(synth.tx_audio, C, k * N, N) for k in range(calls)]
    ins, outs, aouts = [], [], []
    for k in range(calls):
        b = k % nbuf
        tx.process(xs[k], iq[b], a0[b])      # pipelined: no sync or join between calls
        if pipelined:
            continue
        torch.cuda.synchronize()
        outs.append(iq[0][tp].cpu().numpy())
        aouts.append(a0[0][tp].cpu().numpy())
    if pipelined:
        tx.join()
        torch.cuda.synchronize()
        outs = [iq[k][tp].cpu().numpy() for k in range(calls)]
        aouts = [a0[k][tp].cpu().numpy() for k in range(calls)]
    ins = [x[tp].cpu().numpy() for x in xs]
    del xs
    tx.close()
    ref_iq, ref_a0 = oracle.OracleTx(U.build_tx_plan(cfg), len(pk)).process(np.concatenate(ins, 1), threads=8)
    np.testing.assert_array_equal(np.concatenate(aouts, 1).view(np.uint32), ref_a0.view(np.uint32))
    np.testing.assert_array_equal(np.concatenate(outs, 1), ref_iq)
    assert np.abs(ref_iq).max() > 0
