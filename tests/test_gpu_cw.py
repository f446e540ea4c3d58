"""Device CW decoder front end (rx_back's audio wave, through the C ABI) against the reference
firmware's own CW fixtures (tests/golden/cw_*.npz) and the CPU oracle: Goertzel energies and
ads.CW_signal bit for bit, at several call sizes and on ragged batches."""
import numpy as np
import pytest

import oracle
import uhsdr_amd as U
from golden_util import assert_bitexact
from test_cw_oracle import cw_blocks, cw_files, load_cw
from uhsdr_amd import synth

pytestmark = pytest.mark.gpu


def run_cw(cfg, iq, frames):
    import torch
    C, n, _ = iq.shape
    chain = U.RxChain(cfg, channels=C, frames=frames)
    bmax = chain.cw_blocks_max
    d_sig = torch.zeros((C, frames // 32), dtype=torch.uint8, device="cuda")
    d_en = torch.zeros((C, max(bmax, 1)), dtype=torch.float32, device="cuda")
    chain.set_cw_outputs(d_sig, d_en)
    audio = torch.empty((C, frames), dtype=torch.float32, device="cuda")
    sig, en, a1 = [], [], []
    for off in range(0, n, frames):
        x = torch.from_numpy(np.ascontiguousarray(iq[:, off:off + frames])).cuda()
        chain.process(x, audio, None)
        torch.cuda.synchronize()
        sig.append(d_sig.cpu().numpy())
        en.append(d_en[:, :chain.cw_blocks_last].cpu().numpy())
        a1.append(audio.cpu().numpy())
    chain.close()
    return np.concatenate(sig, axis=1), np.concatenate(en, axis=1), np.concatenate(a1, axis=1)


@pytest.mark.parametrize("path", cw_files(), ids=lambda p: p.split("cw_")[-1][:-4])
def test_device_cw_matches_reference_firmware(cuda, back, path):
    g = load_cw(path)
    sig, en, _ = run_cw(U.config_from_ref_args(g["args"]), g["iq"], 256)
    assert_bitexact(en, g["energy"], "Goertzel energy")
    np.testing.assert_array_equal(sig, g["signal"])


@pytest.mark.parametrize("frames", [32, 64, 128, 1024, 2048])
def test_device_cw_call_granularity(cuda, frames):
    g = load_cw([p for p in cw_files() if p.endswith("cw_p4_cw_b90.npz")][0])
    n = g["iq"].shape[1] // frames * frames
    sig, en, _ = run_cw(U.config_from_ref_args(g["args"]), g["iq"][:, :n], frames)
    np.testing.assert_array_equal(sig, g["signal"][:, :n // 32])
    assert_bitexact(en, g["energy"][:, :en.shape[1]], f"energy N={frames}")


@pytest.mark.parametrize("mode,path,channels", [(U.DEMOD_CW, 4, 333), (U.DEMOD_CW, 12, 130), (U.DEMOD_SAM, 70, 65)])
def test_device_cw_matches_oracle_ragged(cuda, back, mode, path, channels):
    cfg = U.default_config(dmod_mode=mode, filter_path=path, cw_decoder_thresh=1200, cw_decoder_blocksize=72)
    n = 4096
    iq = synth.cw_iq(np.arange(channels), 3, n) if mode == U.DEMOD_CW else synth.am_iq(np.arange(channels), 3, n)
    plan = U.build_plan(cfg)
    assert plan.cw_enabled
    a1o, _, sigo, eno = oracle.rx_process_cw(oracle.OracleRx(plan, channels), iq, cw_blocks(plan, n), threads=8)
    sig, en, a1 = run_cw(cfg, iq, 512)
    assert_bitexact(a1, a1o, "audio")
    np.testing.assert_array_equal(sig, sigo)
    assert_bitexact(en, eno, "energy")
