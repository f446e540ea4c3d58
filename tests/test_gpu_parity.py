"""Device parity: the HIP chain in libuhsdr_amd.so, called through its C ABI, against

  * the reference firmware's own outputs (tests/golden/rx_*.npz) -- bit-exact, every config;
  * the CPU oracle at larger batches (many channels, ragged channel counts, several calls
    carrying state) -- bit-exact;
  * the oracle on sampled channels of the full C2 / north-star batch sizes -- bit-exact.

The chain computes in the reference's binary32 operation order (no FP contraction), so the
bar is bit equality (north_star's 1e-5 relative tolerance is implied).
"""
import numpy as np
import pytest

import oracle
import uhsdr_amd as U
from golden_util import assert_bitexact, golden_file, golden_files, load
from uhsdr_amd import synth

pytestmark = pytest.mark.gpu


def run_device(cfg, iq, frames_per_call, want_dst=True):
    import torch
    C, n, _ = iq.shape
    chain = U.RxChain(cfg, channels=C, frames=frames_per_call)
    a_out = np.empty((C, n), np.float32)
    d_out = np.empty((C, n, 2), np.int32)
    audio = torch.empty((C, frames_per_call), dtype=torch.float32, device="cuda")
    dst = torch.empty((C, frames_per_call, 2), dtype=torch.int32, device="cuda") if want_dst else None
    for off in range(0, n, frames_per_call):
        x = torch.from_numpy(np.ascontiguousarray(iq[:, off:off + frames_per_call])).cuda()
        chain.process(x, audio, dst)
        torch.cuda.synchronize()
        a_out[:, off:off + frames_per_call] = audio.cpu().numpy()
        if want_dst:
            d_out[:, off:off + frames_per_call] = dst.cpu().numpy()
    chain.close()
    return a_out, d_out


@pytest.mark.parametrize("path", golden_files(), ids=lambda p: p.split("rx_")[-1][:-4])
def test_device_matches_reference_firmware(cuda, back, path):
    g = load(path)
    cfg = U.config_from_ref_args(g["args"])
    a1, dst = run_device(cfg, g["iq"], 256)
    assert_bitexact(a1, g["a1"], g["name"])
    np.testing.assert_array_equal(dst, g["dst"])


@pytest.mark.parametrize("frames", [32, 64, 128, 1024, 2048])
def test_device_call_granularity(cuda, back, frames):
    g = load(golden_file("p48_usb"))
    cfg = U.config_from_ref_args(g["args"])
    a1, _ = run_device(cfg, g["iq"], frames, want_dst=False)
    assert_bitexact(a1, g["a1"], f"frames={frames}")


@pytest.mark.parametrize("path,channels", [(48, 1000), (35, 333), (55, 130), (4, 65)])
def test_device_matches_oracle_ragged_batches(cuda, back, path, channels):
    mode = U.DEMOD_CW if path == 4 else U.DEMOD_USB
    cfg = U.default_config(filter_path=path, dmod_mode=mode)
    iq = synth.ssb_iq(np.arange(channels), 0, 1024)
    a1, dst = run_device(cfg, iq, 256)
    ref_a1, ref_dst = oracle.OracleRx(U.build_plan(cfg), channels).process(iq, threads=8)
    assert_bitexact(a1, ref_a1, f"P{path} C={channels}")
    np.testing.assert_array_equal(dst, ref_dst)


def test_device_c2_batch_sampled_channels(cuda):
    """C2: 4096 channels x 256-frame calls; every 257th channel checked against the oracle."""
    cfg = U.default_config()
    C = 4096
    iq = synth.ssb_iq(np.arange(C), 0, 1024)
    a1, _ = run_device(cfg, iq, 256, want_dst=False)
    pick = np.arange(0, C, 257)
    ref, _ = oracle.OracleRx(U.build_plan(cfg), len(pick)).process(iq[pick], threads=8)
    assert_bitexact(a1[pick], ref, "C2 sampled")
    assert np.isfinite(a1).all()


@pytest.mark.parametrize("path", [48, 35, 55])
def test_device_north_star_batch_sampled_channels(cuda, path):
    """262144 channels x 64-frame calls (north-star regime, R = 16 front blocks): sampled
    channels vs oracle, for each filter-path family."""
    import torch
    cfg = U.default_config(filter_path=path)
    C, n = 262144, 128
    pick = np.array([0, 1, 63, 64, 4095, 65536, 131071, 262143])
    chain = U.RxChain(cfg, channels=C, frames=64)
    audio = torch.empty((C, 64), dtype=torch.float32, device="cuda")
    got = np.empty((len(pick), n), np.float32)
    for off in range(0, n, 64):
        x = torch.from_numpy(synth.ssb_iq(np.arange(C), off, 64)).cuda()
        chain.process(x, audio, None)
        torch.cuda.synchronize()
        got[:, off:off + 64] = audio[torch.from_numpy(pick).cuda()].cpu().numpy()
    chain.close()
    ref, _ = oracle.OracleRx(U.build_plan(cfg), len(pick)).process(synth.ssb_iq(pick, 0, n))
    assert_bitexact(got, ref, "north-star sampled")


def test_device_reset_restarts_stream(cuda, back):
    import torch
    g = load(golden_file("p48_usb"))
    cfg = U.config_from_ref_args(g["args"])
    chain = U.RxChain(cfg, channels=4, frames=256)
    audio = torch.empty((4, 256), dtype=torch.float32, device="cuda")
    x = torch.from_numpy(np.ascontiguousarray(g["iq"][:, :256])).cuda()
    chain.process(x, audio)
    chain.process(x, audio)
    chain.reset()
    chain.process(x, audio)
    torch.cuda.synchronize()
    assert_bitexact(audio.cpu().numpy(), g["a1"][:, :256], "after reset")


def test_device_host_entry_point(cuda):
    g = load(golden_file("p48_usb"))
    chain = U.RxChain(U.config_from_ref_args(g["args"]), channels=4, frames=2048)
    a1, dst = chain.process_host(g["iq"])
    assert_bitexact(a1, g["a1"], "process_host")
    np.testing.assert_array_equal(dst, g["dst"])


def test_plain_c_host_matches_reference_firmware(cuda, tmp_path):
    """The gcc-built C host (examples/rx_batch.c) through the C ABI: bit-exact vs the
    reference firmware's fixture."""
    import os
    import subprocess
    g = load(golden_file("p48_usb"))
    C, n, _ = g["iq"].shape
    src, out = tmp_path / "iq.bin", tmp_path / "audio.bin"
    np.ascontiguousarray(g["iq"], dtype=np.int32).tofile(src)
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "examples", "build", "rx_batch")
    cfg = U.config_from_ref_args(g["args"])
    r = subprocess.run([exe, str(src), str(out), str(C), str(n), "256", str(cfg.filter_path), str(cfg.dmod_mode)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    got = np.fromfile(out, dtype=np.float32).reshape(C, n)
    assert_bitexact(got, g["a1"], "rx_batch.c")


@pytest.mark.parametrize("path,mode,sb,channels", [(70, U.DEMOD_AM, 0, 300), (70, U.DEMOD_SAM, 0, 257),
                                                   (86, U.DEMOD_SAM, 0, 129), (75, U.DEMOD_SAM, 2, 65),
                                                   (83, U.DEMOD_AM, 0, 100)])
def test_device_am_sam_matches_oracle(cuda, back, path, mode, sb, channels):
    cfg = U.default_config(filter_path=path, dmod_mode=mode, sam_sideband=sb)
    iq = synth.am_iq(np.arange(channels), 0, 1024)
    a1, dst = run_device(cfg, iq, 256)
    ref_a1, ref_dst = oracle.OracleRx(U.build_plan(cfg), channels).process(iq, threads=8)
    assert_bitexact(a1, ref_a1, f"P{path} mode {mode} C={channels}")
    np.testing.assert_array_equal(dst, ref_dst)


def test_device_c3_sam_batch_sampled_channels(cuda):
    """C3: 32768 channels of SAM P70 (PLL 2500 / 0.65 / 250, fade on) x 64-frame calls; sampled
    channels vs the oracle."""
    import torch
    cfg = U.default_config(filter_path=70, dmod_mode=U.DEMOD_SAM)
    C, n = 32768, 256
    pick = np.array([0, 1, 63, 64, 4095, 16384, 32767])
    chain = U.RxChain(cfg, channels=C, frames=64)
    audio = torch.empty((C, 64), dtype=torch.float32, device="cuda")
    got = np.empty((len(pick), n), np.float32)
    for off in range(0, n, 64):
        chain.process(torch.from_numpy(synth.am_iq(np.arange(C), off, 64)).cuda(), audio, None)
        torch.cuda.synchronize()
        got[:, off:off + 64] = audio[torch.from_numpy(pick).cuda()].cpu().numpy()
    chain.close()
    ref, _ = oracle.OracleRx(U.build_plan(cfg), len(pick)).process(synth.am_iq(pick, 0, n))
    assert_bitexact(got, ref, "C3 sampled")


@pytest.mark.parametrize("path,sql,channels", [(1, 12, 200), (1, 0, 77), (3, 2, 65)])
def test_device_fm_matches_oracle(cuda, path, sql, channels):
    """FM-RX (C4 row a10): 8192 frames so the squelch decides inside the run."""
    cfg = U.default_config(filter_path=path, dmod_mode=U.DEMOD_FM, fm_sql_threshold=sql)
    iq = synth.fm_iq(np.arange(channels), 0, 8192)
    a1, dst = run_device(cfg, iq, 512)
    ref_a1, ref_dst = oracle.OracleRx(U.build_plan(cfg), channels).process(iq, threads=8)
    assert_bitexact(a1, ref_a1, f"FM P{path} sql={sql} C={channels}")
    np.testing.assert_array_equal(dst, ref_dst)
