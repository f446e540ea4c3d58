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
from golden_util import assert_bitexact, drive, golden_file, golden_files, load
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


class DeviceStream:
    """One RxChain fed block by block (golden_util.drive), outputs copied back per call."""

    def __init__(self, cfg, channels, frames):
        import torch
        self.torch = torch
        self.chain = U.RxChain(cfg, channels=channels, frames=frames)
        # a_buffer[0] is an output of its own in stereo and on mcHF (the line-out channel)
        self.stereo = bool(self.chain.plan.stereo) or bool(self.chain.plan.single_channel)
        self.audio = torch.empty((channels, frames), dtype=torch.float32, device="cuda")
        self.audio0 = torch.empty((channels, frames), dtype=torch.float32, device="cuda")
        self.dst = torch.empty((channels, frames, 2), dtype=torch.int32, device="cuda")

    def __call__(self, iq_block):
        """(a_buffer[1], a_buffer[0], dst); a_buffer[0] is a copy of [1] in OVI40 mono"""
        self.chain.process_stereo(self.torch.from_numpy(iq_block).cuda(), self.audio, self.audio0, self.dst)
        self.torch.cuda.synchronize()
        a1 = self.audio.cpu().numpy()
        return a1, (self.audio0.cpu().numpy() if self.stereo else a1.copy()), self.dst.cpu().numpy()


@pytest.mark.parametrize("path", golden_files(), ids=lambda p: p.split("rx_")[-1][:-4])
def test_device_matches_reference_firmware(cuda, back, path):
    g = load(path)
    cfg = U.config_from_ref_args(g["args"])
    dev = DeviceStream(cfg, g["iq"].shape[0], 256)
    a1, a0, dst = drive(g, 256, dev, dev.chain.key_beep)
    dev.chain.close()
    assert_bitexact(a1, g["a1"], g["name"])
    if "a0" in g:
        assert_bitexact(a0, g["a0"], g["name"] + " a_buffer[0]")
    np.testing.assert_array_equal(dst, g["dst"])


@pytest.mark.parametrize("frames", [32, 64, 128, 1024, 2048])
def test_device_call_granularity(cuda, back, frames):
    g = load(golden_file("p48_usb"))
    cfg = U.config_from_ref_args(g["args"])
    a1, _ = run_device(cfg, g["iq"], frames, want_dst=False)
    assert_bitexact(a1, g["a1"], f"frames={frames}")


@pytest.mark.parametrize("frames", [512, 1024, 2048])
@pytest.mark.parametrize("name", ["p70_sam", "p70_am", "p35_usb", "p4_cw", "p86_sam"])
def test_device_call_granularity_decimate_first(cuda, back, name, frames):
    """The decimate-first fronts (AM / SAM, narrow SSB / CW) at the call sizes C3 is timed at
    (1024 frames: two 512-frame front launches per call, one channel per wave, through the padded
    pair window) against the reference firmware's own outputs (audio_driver.c:1990-2166,
    :2718-2746)."""
    g = load(golden_file(name))
    cfg = U.config_from_ref_args(g["args"])
    a1, dst = run_device(cfg, g["iq"], frames)
    assert_bitexact(a1, g["a1"], f"{name} frames={frames}")
    np.testing.assert_array_equal(dst, g["dst"])


SEG_CASES = [(mode, iqmode, kw) for mode in (U.DEMOD_AM, U.DEMOD_SAM) for iqmode in (0, 1, 3)
             for kw in ({}, dict(iq_gain_i=1.02, iq_gain_q=0.97, iq_phase_balance=-0.01))]
SEG_CASES += [(U.DEMOD_SAM, 2, {}), (U.DEMOD_AM, 0, dict(iq_auto_correction=1))]


@pytest.mark.parametrize("mode,iqmode,kw", SEG_CASES,
                         ids=[f"{'am' if m == U.DEMOD_AM else 'sam'}-iq{q}-{'imb' if 'iq_gain_i' in k else 'auto' if k else 'plain'}"
                              for m, q, k in SEG_CASES])
@pytest.mark.parametrize("frames", [1024, 2048])
def test_device_long_calls_decimate_first(cuda, mode, iqmode, kw, frames):
    """AM / SAM calls longer than one front wave's 512 frames (two or four front launches per
    call, each carrying the pass-1 history to the next) with the manual I/Q gain / phase
    correction, the Fs/4 exchanges (iq modes 1, 3), the +6 kHz oscillator (iq mode 2) and auto
    I/Q correction: bit-exact to the oracle on a ragged batch."""
    C = 67
    cfg = U.default_config(filter_path=70, dmod_mode=mode, iq_freq_mode=iqmode, **kw)
    iq = synth.am_iq(np.arange(C), 0, 2 * frames)
    a1, dst = run_device(cfg, iq, frames)
    ref_a1, ref_dst = oracle.OracleRx(U.build_plan(cfg), C).process(iq, threads=8)
    assert_bitexact(a1, ref_a1, f"mode {mode} iq {iqmode} {kw} frames={frames}")
    np.testing.assert_array_equal(dst, ref_dst)


@pytest.mark.parametrize("path,channels", [(48, 1000), (35, 333), (55, 130), (4, 65)])
def test_device_matches_oracle_ragged_batches(cuda, back, path, channels):
    mode = U.DEMOD_CW if path == 4 else U.DEMOD_USB
    cfg = U.default_config(filter_path=path, dmod_mode=mode)
    iq = synth.ssb_iq(np.arange(channels), 0, 1024)
    a1, dst = run_device(cfg, iq, 256)
    ref_a1, ref_dst = oracle.OracleRx(U.build_plan(cfg), channels).process(iq, threads=8)
    assert_bitexact(a1, ref_a1, f"P{path} C={channels}")
    np.testing.assert_array_equal(dst, ref_dst)


NOTCH_CASES = [
    ("p48_usb", dict(filter_path=48), synth.ssb_iq, 200),
    ("p35_lsb", dict(filter_path=35, dmod_mode=U.DEMOD_LSB), synth.ssb_iq, 130),
    ("p55_usb", dict(filter_path=55, notch_mu=40), synth.ssb_iq, 70),
    ("p70_am", dict(filter_path=70, dmod_mode=U.DEMOD_AM), synth.am_iq, 129),
    ("p70_sam", dict(filter_path=70, dmod_mode=U.DEMOD_SAM, notch_mu=25), synth.am_iq, 96),
    ("p75_sam_lsb", dict(filter_path=75, dmod_mode=U.DEMOD_SAM, sam_sideband=U.SAM_SIDEBAND_LSB), synth.am_iq, 65),
    ("p83_am", dict(filter_path=83, dmod_mode=U.DEMOD_AM), synth.am_iq, 64),
]


@pytest.mark.parametrize("name,kw,gen,C", NOTCH_CASES, ids=[c[0] for c in NOTCH_CASES])
def test_device_notch_matches_oracle(cuda, back, name, kw, gen, C):
    """LMS auto notch (rx_notch, + the AM / SAM demodulator ahead of it) on ragged batches over
    the 128-sample delay line's full cycle (1024 calls of 32 frames would be 4 cycles; 48 calls
    here pass the wrap at 16 / 8 calls and the first-call self reference)."""
    cfg = U.default_config(dsp_active=U.DSP_NOTCH_ENABLE, **kw)
    assert U.build_plan(cfg).notch_enabled
    iq = gen(np.arange(C), 0, 48 * 32)
    a1, dst = run_device(cfg, iq, 256)
    ref_a1, ref_dst = oracle.OracleRx(U.build_plan(cfg), C).process(iq, threads=8)
    assert_bitexact(a1, ref_a1, f"notch {name}")
    np.testing.assert_array_equal(dst, ref_dst)


@pytest.mark.parametrize("frames", [32, 64, 512])
def test_device_beep_call_sizes(cuda, back, frames):
    """Key beep across call sizes: started between launches, ending inside one, restarted."""
    import torch
    cfg = U.default_config(beep_frequency=880, beep_loudness=15)
    C, n = 70, 2048
    iq = synth.ssb_iq(np.arange(C), 0, n)
    o = oracle.OracleRx(U.build_plan(cfg), C)
    chain = U.RxChain(cfg, channels=C, frames=frames)
    audio = torch.empty((C, frames), dtype=torch.float32, device="cuda")
    got, ref = [], []
    for k, off in enumerate(range(0, n, frames)):
        if k in (1, 5):
            chain.key_beep(21 if k == 1 else 3)
            o.key_beep(21 if k == 1 else 3)
        blk = np.ascontiguousarray(iq[:, off:off + frames])
        chain.process(torch.from_numpy(blk).cuda(), audio, None)
        torch.cuda.synchronize()
        got.append(audio.cpu().numpy())
        ref.append(o.process(blk)[0])
    chain.close()
    assert_bitexact(np.concatenate(got, axis=1), np.concatenate(ref, axis=1), f"beep frames={frames}")


def test_device_fm_tone_detector_matches_oracle(cuda):
    """FM subaudible tone detector on 100 channels, half carrying the selected CTCSS tone."""
    cfg = U.default_config(filter_path=1, dmod_mode=U.DEMOD_FM, fm_tone_det=10)
    C, n = 100, 1600 * 32
    iq = np.concatenate([synth.fm_iq(np.arange(50), 0, n, subtone=91.5), synth.fm_iq(np.arange(50, 100), 0, n)])
    a1, dst = run_device(cfg, iq, 2048)
    ref_a1, ref_dst = oracle.OracleRx(U.build_plan(cfg), C).process(iq, threads=8)
    assert_bitexact(a1, ref_a1, "fm tone detector")
    np.testing.assert_array_equal(dst, ref_dst)
    assert np.abs(a1[:50, -2048:]).max() > 1000 and np.abs(a1[50:, -2048:]).max() == 0


STEREO_CASES = [
    ("p48_ssbstereo", dict(filter_path=48, dmod_mode=U.DEMOD_SSBSTEREO), synth.ssb_iq, 130, 256),
    ("p35_ssbstereo", dict(filter_path=35, dmod_mode=U.DEMOD_SSBSTEREO), synth.ssb_iq, 65, 512),
    ("p55_iq", dict(filter_path=55, dmod_mode=U.DEMOD_IQ), synth.ssb_iq, 100, 64),
    ("p44_iq", dict(filter_path=44, dmod_mode=U.DEMOD_IQ, agc_mode=1, agc_hang_enable=1), synth.ssb_iq, 64, 256),
    ("p70_sam_st", dict(filter_path=70, dmod_mode=U.DEMOD_SAM, sam_sideband=U.SAM_SIDEBAND_STEREO), synth.am_iq, 96, 256),
    ("p86_sam_st", dict(filter_path=86, dmod_mode=U.DEMOD_SAM, sam_sideband=U.SAM_SIDEBAND_STEREO), synth.am_iq, 70, 128),
    ("p48_ssbstereo_notch", dict(filter_path=48, dmod_mode=U.DEMOD_SSBSTEREO, dsp_active=U.DSP_NOTCH_ENABLE),
     synth.ssb_iq, 66, 256),
    ("p75_sam_st_notch", dict(filter_path=75, dmod_mode=U.DEMOD_SAM, sam_sideband=U.SAM_SIDEBAND_STEREO,
                              dsp_active=U.DSP_NOTCH_ENABLE), synth.am_iq, 65, 256),
]


@pytest.mark.parametrize("name,kw,gen,C,N", STEREO_CASES, ids=[c[0] for c in STEREO_CASES])
def test_device_stereo_matches_oracle(cuda, name, kw, gen, C, N):
    """OVI40 two-channel modes on ragged batches: both output channels and the {l, r} codec frames."""
    cfg = U.default_config(stereo_enable=1, **kw)
    assert U.build_plan(cfg).stereo
    iq = gen(np.arange(C), 0, 2048)
    dev = DeviceStream(cfg, C, N)
    outs = [dev(np.ascontiguousarray(iq[:, off:off + N])) for off in range(0, 2048, N)]
    dev.chain.close()
    a1, a0, dst = (np.concatenate([o[i] for o in outs], axis=1) for i in range(3))
    r1, r0, rdst = oracle.OracleRx(U.build_plan(cfg), C).process2(iq, threads=8)
    assert_bitexact(a1, r1, f"{name} a_buffer[1]")
    assert_bitexact(a0, r0, f"{name} a_buffer[0]")
    np.testing.assert_array_equal(dst, rdst)


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


MCHF_CASES = [
    ("p48_usb_spkr24", dict(filter_path=48, spkr_gain=24), synth.ssb_iq, 1000, 256),
    ("p35_lsb", dict(filter_path=35, dmod_mode=U.DEMOD_LSB), synth.ssb_iq, 333, 512),
    ("p70_sam_spkr30", dict(filter_path=70, dmod_mode=U.DEMOD_SAM, spkr_gain=30), synth.am_iq, 130, 1024),
    ("p1_fm_sql0_spkr20", dict(filter_path=1, dmod_mode=U.DEMOD_FM, fm_sql_threshold=0, spkr_gain=20), synth.fm_iq, 129, 256),
]


@pytest.mark.parametrize("name,kw,gen,C,N", MCHF_CASES, ids=[c[0] for c in MCHF_CASES])
def test_device_mchf_matches_oracle(cuda, back, name, kw, gen, C, N):
    """mcHF output stage (single-channel audio, audio_driver.c:2870-2897) on ragged batches with a
    key beep across calls: a_buffer[1] (speaker, software gain), a_buffer[0] (line out) and the
    codec frames {a1, a0}, every schedule, against the oracle."""
    import torch
    cfg = U.default_config(board=U.BOARD_MCHF, **kw)
    # FM: past the squelch's first decision (every 200 calls, audio_driver.c:1600-1640), which opens it
    n = (28 if kw.get("dmod_mode") == U.DEMOD_FM else 8) * N
    iq = gen(np.arange(C), 0, n)
    o = oracle.OracleRx(U.build_plan(cfg), C)
    chain = U.RxChain(cfg, channels=C, frames=N)
    audio = torch.empty((C, N), dtype=torch.float32, device="cuda")
    audio0 = torch.empty((C, N), dtype=torch.float32, device="cuda")
    dst = torch.empty((C, N, 2), dtype=torch.int32, device="cuda")
    got, ref = [[], [], []], [[], [], []]
    for k in range(n // N):
        if k == 2:
            chain.key_beep(N // 32 + 3)
            o.key_beep(N // 32 + 3)
        blk = np.ascontiguousarray(iq[:, k * N:(k + 1) * N])
        chain.process_stereo(torch.from_numpy(blk).cuda(), audio, audio0, dst)
        torch.cuda.synchronize()
        for lst, t in zip(got, (audio, audio0, dst)):
            lst.append(t.cpu().numpy())
        for lst, r in zip(ref, o.process2(blk)):
            lst.append(r)
    chain.close()
    got = [np.concatenate(x, axis=1) for x in got]
    ref = [np.concatenate(x, axis=1) for x in ref]
    assert_bitexact(got[0], ref[0], f"mcHF {name} a_buffer[1]")
    assert_bitexact(got[1], ref[1], f"mcHF {name} a_buffer[0]")
    np.testing.assert_array_equal(got[2], ref[2])
    assert np.abs(ref[1]).max() > 0
