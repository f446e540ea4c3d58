"""Device SSB and FM transmit (uhsdr_tx.hip through the C ABI) against the reference firmware's own
TX fixtures (tests/golden/tx_*.npz) and against the CPU oracle on ragged batches: bit for bit
(IQ DAC frames and the compressed audio)."""
import numpy as np
import pytest

import oracle
import uhsdr_amd as U
from test_tx_oracle import drive_tx, load_tx, tx_files
from uhsdr_amd import synth

pytestmark = pytest.mark.gpu


def run_tx(cfg, audio, frames, args=None):
    import torch
    C, n, _ = audio.shape
    chain = U.TxChain(cfg, channels=C, frames=frames)
    d_iq = torch.empty((C, frames, 2), dtype=torch.int32, device="cuda")
    d_a0 = torch.zeros((C, frames), dtype=torch.float32, device="cuda")   # DIGIQ calls leave a_buffer[0]

    def process(block):
        chain.process(torch.from_numpy(block).cuda(), d_iq, d_a0)
        torch.cuda.synchronize()
        return d_iq.cpu().numpy(), d_a0.cpu().numpy()

    iq, a0 = drive_tx(chain, process, audio, frames, args or {})
    chain.close()
    return iq, a0


@pytest.mark.parametrize("path", tx_files(), ids=lambda p: p.split("/")[-1][:-4])
def test_device_tx_matches_reference_firmware(cuda, path):
    g = load_tx(path)
    iq, a0 = run_tx(U.tx_config_from_ref_args(g["args"]), g["audio"], 256, g["args"])
    np.testing.assert_array_equal(a0.view(np.uint32), g["a0"].view(np.uint32))
    np.testing.assert_array_equal(iq, g["iq"])


@pytest.mark.parametrize("frames", [32, 64, 512, 2048])
@pytest.mark.parametrize("name", ["tx_usb", "tx_fm_m6k_subtone"])
def test_device_tx_call_granularity(cuda, frames, name):
    g = load_tx([p for p in tx_files() if p.endswith(name + ".npz")][0])
    iq, _ = run_tx(U.tx_config_from_ref_args(g["args"]), g["audio"], frames)
    np.testing.assert_array_equal(iq, g["iq"])


@pytest.mark.parametrize("mode,iqmode,channels", [(0, 4, 333), (1, 2, 130), (0, 0, 65), (5, 3, 200), (5, 1, 70)])
def test_device_tx_matches_oracle_ragged(cuda, mode, iqmode, channels):
    cfg = U.default_tx_config(dmod_mode=mode, iq_freq_mode=iqmode, fm_subaudible_tone=7 if mode == 5 else 0,
                              fm_deviation_5k=int(iqmode == 1))
    audio = synth.tx_audio(np.arange(channels), 0, 1024)
    iq, a0 = run_tx(cfg, audio, 256)
    ref_iq, ref_a0 = oracle.OracleTx(U.build_tx_plan(cfg), channels).process(audio, threads=8)
    np.testing.assert_array_equal(a0.view(np.uint32), ref_a0.view(np.uint32))
    np.testing.assert_array_equal(iq, ref_iq)


@pytest.mark.parametrize("mode,iqmode,args,channels", [
    (0, 4, {"tune": "4:16:2"}, 130), (1, 2, {"tune": "0:8:1"}, 65),
    (5, 3, {"tune": "8:8:1", "burst": "20:8"}, 100)])
def test_device_tx_tones_match_oracle_ragged(cuda, mode, iqmode, args, channels):
    """TUNE tones and the FM tone burst switched between 128-frame calls, vs the oracle."""
    cfg = U.default_tx_config(dmod_mode=mode, iq_freq_mode=iqmode, fm_subaudible_tone=7 if mode == 5 else 0,
                              fm_tone_burst_mode=2 if mode == 5 else 0)
    audio = synth.tx_audio(np.arange(channels), 0, 1024)
    iq, a0 = run_tx(cfg, audio, 128, args)
    o = oracle.OracleTx(U.build_tx_plan(cfg), channels)
    ref_iq, ref_a0 = drive_tx(o, lambda b: o.process(b, threads=8), audio, 128, args)
    np.testing.assert_array_equal(a0.view(np.uint32), ref_a0.view(np.uint32))
    np.testing.assert_array_equal(iq, ref_iq)
