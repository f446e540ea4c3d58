"""The firmware ISR entry (uhsdr_i2s_*, AudioDriver_I2SCallback audio_driver.c:2962-3049) on the
device: one transceiver fed the firmware's 32-frame DMA half-buffers.

  * RX: the reference firmware's own codec frames (tests/golden/rx_*.npz, channel 0), bit-exact;
  * TX: the reference firmware's own DAC I/Q frames (tests/golden/tx_*.npz, channel 0), bit-exact;
  * the switch semantics -- silenced input and muted output on the first RX call after TX and
    while the input-mute counter runs, TxProcessor_PrepareRun plus a skipped (state-frozen) TX
    call on the first TX call after RX -- against the batched chains run on the equivalently
    silenced inputs (the firmware code paths these restate are cited in uhsdr_i2s.hip)."""
import numpy as np
import pytest

import uhsdr_amd as U
from golden_util import golden_file, load
from test_tx_oracle import load_tx, tx_files

pytestmark = pytest.mark.gpu
B = 32


def run_rx_blocks(trx, iq):
    out = np.empty_like(iq)
    for k in range(iq.shape[0] // B):
        a = np.zeros((B, 2), np.int32)
        x = np.ascontiguousarray(iq[k * B:(k + 1) * B])
        trx.callback(a, x)
        out[k * B:(k + 1) * B] = a
    return out


@pytest.mark.parametrize("name", ["p48_usb", "p35_usb", "p70_sam", "p1_fm"])
def test_i2s_rx_matches_reference_firmware(cuda, name):
    g = load(golden_file(name))
    trx = U.Transceiver(U.config_from_ref_args(g["args"]), block=B)
    got = run_rx_blocks(trx, g["iq"][0])
    trx.close()
    np.testing.assert_array_equal(got, g["dst"][0])


I2S_TX = ("tx_fm", "tx_fm_m6k_subtone", "tx_usb", "tx_lsb")


@pytest.mark.parametrize("path", [p for p in tx_files() if p.split("/")[-1][:-4] in I2S_TX],
                         ids=lambda p: p.split("/")[-1][:-4])
def test_i2s_tx_matches_reference_firmware(cuda, path):
    g = load_tx(path)
    trx = U.Transceiver(U.default_config(), U.tx_config_from_ref_args(g["args"]), block=B)
    trx.set_txrx_mode(True)
    audio = g["audio"][0]
    got = np.empty((audio.shape[0], 2), np.int32)
    dst = np.empty((B, 2), np.int32)
    for k in range(audio.shape[0] // B):
        a = np.ascontiguousarray(audio[k * B:(k + 1) * B])
        q = np.zeros((B, 2), np.int32)
        trx.callback(a, q, dst)
        got[k * B:(k + 1) * B] = q
        assert not dst.any()
    trx.close()
    np.testing.assert_array_equal(got, g["iq"][0])


def test_i2s_input_mute_and_rx_tx_switching(cuda):
    g = load(golden_file("p48_usb"))
    cfg = U.config_from_ref_args(g["args"])
    iq = g["iq"][0][:32 * B]
    tcfg = U.default_tx_config()
    mic = load_tx(tx_files()[0])["audio"][0][:8 * B]
    trx = U.Transceiver(cfg, tcfg, block=B)

    # RX: 2 counted input mutes, 10 calls; TX: 8 calls (the first silenced); RX again: 22 calls
    trx.set_input_mute(2)
    rx1 = run_rx_blocks(trx, iq[:10 * B].copy())
    trx.set_txrx_mode(True)
    tx_iq = np.empty((8 * B, 2), np.int32)
    for k in range(8):
        a = np.ascontiguousarray(mic[k * B:(k + 1) * B])
        q = np.full((B, 2), 7, np.int32)
        trx.callback(a, q)
        tx_iq[k * B:(k + 1) * B] = q
    trx.set_txrx_mode(False)
    rx2 = run_rx_blocks(trx, iq[10 * B:32 * B].copy())
    trx.close()

    # expected RX: one continuous chain over the input with the muted calls' blocks silenced
    x = iq[:32 * B].copy()
    x[:2 * B] = 0
    x[10 * B:11 * B] = 0
    ref = U.RxChain(cfg, channels=1, frames=32 * B).process_host(x[None])[1][0]
    ref[:2 * B] = 0
    ref[10 * B:11 * B] = 0
    np.testing.assert_array_equal(np.concatenate([rx1, rx2]), ref)

    # expected TX: the first TX call outputs zero and leaves the TX state untouched
    t = U.TxChain(tcfg, channels=1, frames=B)
    import torch
    want = np.zeros((8 * B, 2), np.int32)
    d_iq = torch.empty((1, B, 2), dtype=torch.int32, device="cuda")
    for k in range(1, 8):
        t.process(torch.from_numpy(np.ascontiguousarray(mic[None, k * B:(k + 1) * B])).cuda(), d_iq)
        torch.cuda.synchronize()
        want[k * B:(k + 1) * B] = d_iq.cpu().numpy()[0]
    t.close()
    np.testing.assert_array_equal(tx_iq, want)
