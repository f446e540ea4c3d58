"""Device spectrum display path (uhsdr_spectrum.hip through the C ABI) against the reference
firmware's own spectrum fixtures (tests/golden/spec_*.npz) and against the CPU oracle on
ragged batches and at the C3 size (32768 channels, 1024 points): bit for bit, both the
per-frame magnitude (sd.FFT_MagData) and the running average (sd.FFT_AVGData)."""
import numpy as np
import pytest

import oracle
import uhsdr_amd as U
from golden_util import assert_bitexact
from test_spectrum_oracle import load_spec, spec_files
from uhsdr_amd import synth

pytestmark = pytest.mark.gpu


def run_spec(cfg, iq, frames, want_mag=True, want_avg=True):
    import torch
    C, n, _ = iq.shape
    spec = U.Spectrum(cfg, channels=C, frames=frames)
    L, D = spec.fft_len, spec.decimation
    mags, avgs = [], []
    d_mag = torch.full(spec.out_shape, -1.0, dtype=torch.float32, device="cuda") if want_mag else None
    d_avg = torch.full(spec.out_shape, -1.0, dtype=torch.float32, device="cuda") if want_avg else None
    d_iq = torch.empty((C, frames, 2), dtype=torch.int32, device="cuda")
    for off in range(0, n, frames):
        d_iq.copy_(torch.from_numpy(np.ascontiguousarray(iq[:, off:off + frames])))
        nf = spec.process(d_iq, d_mag, d_avg)
        torch.cuda.synchronize()
        nd = frames // D
        assert nf == (nd // L if nd >= L else int((off + frames) // D % L == 0))
        if nf:
            if want_mag:
                mags.append(d_mag[:, :nf].cpu().numpy())
            if want_avg:
                avgs.append(d_avg[:, :nf].cpu().numpy())
    spec.close()
    cat = lambda xs: np.concatenate(xs, axis=1) if xs else None  # noqa: E731
    return cat(mags), cat(avgs)


@pytest.mark.parametrize("path", spec_files(), ids=lambda p: p.split("spec_")[-1][:-4])
def test_device_spectrum_matches_reference_firmware(cuda, path):
    g = load_spec(path)
    mag, avg = run_spec(U.spectrum_config_from_ref_args(g["args"]), g["iq"], 1024)
    assert_bitexact(mag, g["mag"], "FFT_MagData")
    assert_bitexact(avg, g["avg"], "FFT_AVGData")


@pytest.mark.parametrize("frames", [32, 128, 512, 2048, 4096])
@pytest.mark.parametrize("name", ["p48_iqauto_256", "p70_sam_1024", "p48_iqman2_512"])
def test_device_spectrum_call_granularity(cuda, frames, name):
    g = load_spec(spec_files()[[n.split("spec_")[-1][:-4] for n in spec_files()].index(name)])
    mag, avg = run_spec(U.spectrum_config_from_ref_args(g["args"]), g["iq"], frames)
    assert_bitexact(mag, g["mag"], f"mag N={frames}")
    assert_bitexact(avg, g["avg"], f"avg N={frames}")


def test_device_spectrum_optional_outputs(cuda):
    g = load_spec(spec_files()[0])
    cfg = U.spectrum_config_from_ref_args(g["args"])
    _, avg = run_spec(cfg, g["iq"], 1024, want_mag=False)
    assert_bitexact(avg, g["avg"], "avg only")
    mag, _ = run_spec(cfg, g["iq"], 1024, want_avg=False)
    assert_bitexact(mag, g["mag"], "mag only")


@pytest.mark.parametrize("L,auto,filt,channels", [(1024, 0, 4, 333), (512, 1, 9, 130), (256, 0, 1, 65),
                                                  (1024, 1, 20, 7)])
def test_device_spectrum_matches_oracle_ragged(cuda, L, auto, filt, channels):
    cfg = U.default_spectrum_config(fft_len=L, iq_auto_correction=auto, spectrum_filter=filt,
                                    iq_gain_i=1.01, iq_gain_q=0.99, iq_phase_balance=-0.003)
    iq = synth.ssb_iq(np.arange(channels), 7, 4096)
    plan = U.build_spectrum_plan(cfg)
    om, oa = oracle.OracleSpectrum(plan, channels).process(iq, threads=8)
    mag, avg = run_spec(cfg, iq, 2048)
    assert_bitexact(mag, om, "mag")
    assert_bitexact(avg, oa, "avg")


def test_device_spectrum_reset(cuda):
    import torch
    g = load_spec(spec_files()[0])
    cfg = U.spectrum_config_from_ref_args(g["args"])
    C = g["iq"].shape[0]
    spec = U.Spectrum(cfg, channels=C, frames=g["iq"].shape[1])
    d_iq = torch.from_numpy(g["iq"]).cuda()
    d_avg = torch.empty(spec.out_shape, dtype=torch.float32, device="cuda")
    spec.process(d_iq, None, d_avg)
    spec.reset()
    spec.process(d_iq, None, d_avg)
    torch.cuda.synchronize()
    assert_bitexact(d_avg.cpu().numpy(), g["avg"], "after reset")
    spec.close()


def test_device_spectrum_c3_sampled(cuda):
    """C3: 32768 channels x 1024-point frames on AM input; 64 channels checked against the oracle"""
    import torch
    C, n = 32768, 2048
    cfg = U.default_spectrum_config(fft_len=1024)
    spec = U.Spectrum(cfg, channels=C, frames=n)
    d_iq = torch.from_numpy(synth.am_iq(np.arange(C), 0, n)).cuda()
    d_avg = torch.empty(spec.out_shape, dtype=torch.float32, device="cuda")
    d_mag = torch.empty(spec.out_shape, dtype=torch.float32, device="cuda")
    assert spec.process(d_iq, d_mag, d_avg) == 2
    torch.cuda.synchronize()
    pick = np.random.default_rng(3).choice(C, 64, replace=False)
    pick[:2] = [0, C - 1]
    om, oa = oracle.OracleSpectrum(U.build_spectrum_plan(cfg), 64).process(d_iq.cpu().numpy()[pick], threads=8)
    assert_bitexact(d_mag.cpu().numpy()[pick], om, "mag")
    assert_bitexact(d_avg.cpu().numpy()[pick], oa, "avg")
    spec.close()


def zoom_names():
    return [n.split("spec_")[-1][:-4] for n in spec_files() if "_zoom" in n]


@pytest.mark.parametrize("frames", [32, 256, 2048, 8192])
@pytest.mark.parametrize("name", zoom_names())
def test_device_zoom_call_granularity(cuda, frames, name):
    """zoom producer (spectrum_zoom: biquad / decimator / oscillator / auto-I/Q state carried
    across calls) against the reference firmware's zoom fixtures, for call sizes from one ISR
    call to several display frames"""
    g = load_spec(spec_files()[[n.split("spec_")[-1][:-4] for n in spec_files()].index(name)])
    cfg = U.spectrum_config_from_ref_args(g["args"])
    L, D = cfg.fft_len, 1 << cfg.magnify
    nd = frames // D
    if nd == 0 or (nd % L and L % nd) or g["iq"].shape[1] % frames:
        pytest.skip("call size not allowed for this zoom / fft_len")
    mag, avg = run_spec(cfg, g["iq"], frames)
    assert_bitexact(mag, g["mag"], f"zoom mag N={frames}")
    assert_bitexact(avg, g["avg"], f"zoom avg N={frames}")


@pytest.mark.parametrize("m,L,iqmode,auto,channels", [(1, 512, 4, 0, 333), (3, 256, 2, 1, 130), (5, 1024, 0, 0, 65),
                                                      (2, 256, 3, 1, 200)])
def test_device_zoom_matches_oracle_ragged(cuda, m, L, iqmode, auto, channels):
    cfg = U.default_spectrum_config(fft_len=L, magnify=m, iq_freq_mode=iqmode, iq_auto_correction=auto,
                                    iq_gain_i=1.01, iq_gain_q=0.99, iq_phase_balance=0.004)
    n = max(4096, 2 * L << m)
    iq = synth.ssb_iq(np.arange(channels), 3, n)
    plan = U.build_spectrum_plan(cfg)
    om, oa = oracle.OracleSpectrum(plan, channels).process(iq, threads=8)
    mag, avg = run_spec(cfg, iq, 1024)
    assert_bitexact(mag, om, "zoom mag")
    assert_bitexact(avg, oa, "zoom avg")


def test_device_zoom_reset(cuda):
    """reset() restarts the zoom filters, decimator, oscillator and ring"""
    import torch
    cfg = U.default_spectrum_config(fft_len=256, magnify=2, iq_freq_mode=2)
    C, N = 64, 1024
    iq = synth.ssb_iq(np.arange(C), 0, N)
    spec = U.Spectrum(cfg, channels=C, frames=N)
    d_iq = torch.from_numpy(iq).cuda()
    d_mag = torch.empty(spec.out_shape, dtype=torch.float32, device="cuda")
    spec.process(d_iq, d_mag, None)
    first = d_mag.cpu().numpy()
    spec.process(d_iq, d_mag, None)
    spec.reset()
    spec.process(d_iq, d_mag, None)
    again = d_mag.cpu().numpy()
    spec.close()
    assert_bitexact(again, first, "after reset")
