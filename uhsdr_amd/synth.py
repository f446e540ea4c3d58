"""Synthetic 48 kHz I/Q workloads.

Every channel is an independent radio receiving a two-tone SSB signal that sits at
+12 kHz in the I/Q spectrum (so the default ``iq_freq_mode`` = -12 kHz conversion,
audio_driver.h:526 / freq_shift.c:219-262, brings it to baseband) plus white noise.
Samples are delivered exactly as the codec DMA delivers them to
``AudioDriver_RxProcessor`` (audio_driver.c:2660-2685): interleaved ``IqSample_t``
``{int32 l, int32 r}`` frames holding ``(int16) value << 16``.

All randomness is counter-based (splitmix64 of (channel seed, sample index)), so the
samples of channel ``c`` do not depend on how many channels are generated or in which
chunks — a 4-channel fixture and a 4096-channel bench batch agree on channel 0..3.
"""
from __future__ import annotations

import numpy as np

FS = 48000.0
SEED_BASE = 0x5EED0000
_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _splitmix64(x: np.ndarray) -> np.ndarray:
    x = (x + np.uint64(0x9E3779B97F4A7C15)) & _M64
    z = x
    z = ((z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & _M64
    z = ((z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & _M64
    return z ^ (z >> np.uint64(31))


def _uniform(key: np.ndarray) -> np.ndarray:
    """(0, 1) doubles from 64-bit keys."""
    return ((_splitmix64(key) >> np.uint64(11)).astype(np.float64) + 0.5) * (1.0 / 9007199254740992.0)


def channel_params(channels: np.ndarray, kind: str = "ssb2tone"):
    """Per-channel tone parameters (frequencies in Hz relative to the +12 kHz carrier)."""
    ch = channels.astype(np.uint64)
    base = (np.uint64(SEED_BASE) + ch) << np.uint64(20)
    u = [_uniform(base + np.uint64(k)) for k in range(6)]
    if kind == "c1":   # C1: fixed 700 + 1900 Hz, peak 3000 LSB16 (1500 each)
        f1 = np.full(ch.shape, 700.0)
        f2 = np.full(ch.shape, 1900.0)
        a1 = np.full(ch.shape, 1500.0)
        a2 = np.full(ch.shape, 1500.0)
    else:              # C2: audio tones in [300, 2500] Hz, summed peak in [300, 3000] LSB16
        f1 = 300.0 + 2200.0 * u[0]
        f2 = 300.0 + 2200.0 * u[1]
        a1 = 150.0 + 1350.0 * u[2]
        a2 = 150.0 + 1350.0 * u[3]
    p1 = 2.0 * np.pi * u[4]
    p2 = 2.0 * np.pi * u[5]
    return f1, f2, a1, a2, p1, p2


def ssb_iq(channels, start: int, nframes: int, kind: str = "ssb2tone",
           noise_sigma: float = 30.0, lsb: bool = False, carrier: float = 12000.0) -> np.ndarray:
    """int32 frames, shape [len(channels), nframes, 2] = {l (I), r (Q)} per IqSample_t.

    Sample index ``start + i`` is absolute, so consecutive calls continue the stream.
    ``carrier`` is where the suppressed carrier sits in the I/Q spectrum: +12 kHz for the
    default -12 kHz conversion, -12/+-6/0 kHz for the other FREQ_IQ_CONV modes.
    """
    channels = np.asarray(channels, dtype=np.int64)
    f1, f2, a1, a2, p1, p2 = channel_params(channels, kind)
    sgn = -1.0 if lsb else 1.0
    n = np.arange(start, start + nframes, dtype=np.float64)[None, :]
    w1 = 2.0 * np.pi * (carrier + sgn * f1[:, None]) / FS
    w2 = 2.0 * np.pi * (carrier + sgn * f2[:, None]) / FS
    ph1 = w1 * n + p1[:, None]
    ph2 = w2 * n + p2[:, None]
    i_sig = a1[:, None] * np.cos(ph1) + a2[:, None] * np.cos(ph2)
    q_sig = a1[:, None] * np.sin(ph1) + a2[:, None] * np.sin(ph2)
    if noise_sigma > 0:
        ch = channels.astype(np.uint64)[:, None]
        idx = np.arange(start, start + nframes, dtype=np.uint64)[None, :]
        key = ((np.uint64(SEED_BASE) + ch) << np.uint64(40)) ^ (idx << np.uint64(1))
        u1 = _uniform(key)
        u2 = _uniform(key ^ np.uint64(1))
        r = np.sqrt(-2.0 * np.log(u1)) * noise_sigma
        i_sig = i_sig + r * np.cos(2.0 * np.pi * u2)
        q_sig = q_sig + r * np.sin(2.0 * np.pi * u2)
    out = np.empty((len(channels), nframes, 2), dtype=np.int32)
    out[:, :, 0] = np.clip(np.rint(i_sig), -32768, 32767).astype(np.int32) << 16
    out[:, :, 1] = np.clip(np.rint(q_sig), -32768, 32767).astype(np.int32) << 16
    return out


def _noise(channels, start, nframes, noise_sigma):
    ch = channels.astype(np.uint64)[:, None]
    idx = np.arange(start, start + nframes, dtype=np.uint64)[None, :]
    key = ((np.uint64(SEED_BASE) + ch) << np.uint64(40)) ^ (idx << np.uint64(1))
    u1 = _uniform(key)
    u2 = _uniform(key ^ np.uint64(1))
    r = np.sqrt(-2.0 * np.log(u1)) * noise_sigma
    return r * np.cos(2.0 * np.pi * u2), r * np.sin(2.0 * np.pi * u2)


def _frames(i_sig, q_sig):
    out = np.empty(i_sig.shape + (2,), dtype=np.int32)
    out[..., 0] = np.clip(np.rint(i_sig), -32768, 32767).astype(np.int32) << 16
    out[..., 1] = np.clip(np.rint(q_sig), -32768, 32767).astype(np.int32) << 16
    return out


def am_iq(channels, start: int, nframes: int, noise_sigma: float = 30.0, carrier: float = 12000.0,
          depth: float = 0.5, tone: float = 1000.0, amplitude: float = 2000.0, offset_hz: float = 200.0):
    """C3: AM, carrier at `carrier` + U(-offset_hz, offset_hz) Hz per channel,
    `depth` modulation with a `tone` Hz audio tone, peak carrier `amplitude` LSB16, plus noise.
    The SAM PLL has to acquire and track each channel's carrier offset."""
    channels = np.asarray(channels, dtype=np.int64)
    ch = channels.astype(np.uint64)
    base = (np.uint64(SEED_BASE) + ch) << np.uint64(20)
    off = offset_hz * (2.0 * _uniform(base + np.uint64(7)) - 1.0)
    ph_c = 2.0 * np.pi * _uniform(base + np.uint64(8))
    ph_m = 2.0 * np.pi * _uniform(base + np.uint64(9))
    n = np.arange(start, start + nframes, dtype=np.float64)[None, :]
    env = amplitude * (1.0 + depth * np.cos(2.0 * np.pi * tone / FS * n + ph_m[:, None]))
    ph = 2.0 * np.pi * (carrier + off[:, None]) / FS * n + ph_c[:, None]
    i_sig, q_sig = env * np.cos(ph), env * np.sin(ph)
    if noise_sigma > 0:
        ni, nq = _noise(channels, start, nframes, noise_sigma)
        i_sig, q_sig = i_sig + ni, q_sig + nq
    return _frames(i_sig, q_sig)


def cw_iq(channels, start: int, nframes: int, noise_sigma: float = 30.0, carrier: float = 12000.0,
          tone: float = 750.0, amplitude: float = 1500.0, element: int = 2400):
    """C5 CW: an on/off keyed carrier at `carrier` + `tone` +- 40 Hz per
    channel (the receiver's sidetone pitch), keyed in elements of `element` frames (50 ms =
    24 wpm at 48 ksps) with a per-channel pseudo-random pattern, plus noise."""
    channels = np.asarray(channels, dtype=np.int64)
    ch = channels.astype(np.uint64)
    base = (np.uint64(SEED_BASE) + ch) << np.uint64(20)
    off = 40.0 * (2.0 * _uniform(base + np.uint64(11)) - 1.0)
    ph_c = 2.0 * np.pi * _uniform(base + np.uint64(12))
    n = np.arange(start, start + nframes, dtype=np.float64)[None, :]
    el = (np.arange(start, start + nframes) // element).astype(np.uint64)[None, :]
    key = _uniform((base[:, None] + np.uint64(1 << 19)) + el) < 0.55
    ph = 2.0 * np.pi * (carrier + tone + off[:, None]) / FS * n + ph_c[:, None]
    i_sig, q_sig = amplitude * key * np.cos(ph), amplitude * key * np.sin(ph)
    if noise_sigma > 0:
        ni, nq = _noise(channels, start, nframes, noise_sigma)
        i_sig, q_sig = i_sig + ni, q_sig + nq
    return _frames(i_sig, q_sig)


def fm_iq(channels, start: int, nframes: int, noise_sigma: float = 30.0, carrier: float = 12000.0,
          deviation: float = 2500.0, tone: float = 1000.0, amplitude: float = 3000.0,
          subtone: float = 0.0, subtone_dev: float = 300.0):
    """C4 FM-RX: carrier at `carrier` Hz, a `tone` Hz audio tone at
    `deviation` Hz peak deviation, `amplitude` LSB16, plus noise; optionally a CTCSS
    subaudible tone of `subtone` Hz at `subtone_dev` Hz deviation (the FM tone detector's
    input, audio_driver.c:1665-1734)."""
    channels = np.asarray(channels, dtype=np.int64)
    ch = channels.astype(np.uint64)
    base = (np.uint64(SEED_BASE) + ch) << np.uint64(20)
    ph_c = 2.0 * np.pi * _uniform(base + np.uint64(10))
    ph_m = 2.0 * np.pi * _uniform(base + np.uint64(11))
    n = np.arange(start, start + nframes, dtype=np.float64)[None, :]
    ph = (2.0 * np.pi * carrier / FS * n + ph_c[:, None]
          + (deviation / tone) * np.sin(2.0 * np.pi * tone / FS * n + ph_m[:, None]))
    if subtone > 0:
        ph = ph + (subtone_dev / subtone) * np.sin(2.0 * np.pi * subtone / FS * n)
    i_sig, q_sig = amplitude * np.cos(ph), amplitude * np.sin(ph)
    if noise_sigma > 0:
        ni, nq = _noise(channels, start, nframes, noise_sigma)
        i_sig, q_sig = i_sig + ni, q_sig + nq
    return _frames(i_sig, q_sig)


STATUS_PHASE_DEG = (0.0, 12.0, 30.0, 60.0, 89.0)


def status_iq(channels, start: int, nframes: int, noise_sigma: float = 30.0, burst_every: int = 3000,
              burst_len: int = 256):
    """Status side outputs (ADC clip flags, twin-peaks detector; audio_driver.c:2660-2676,
    2173-2248): the two-tone SSB signal of ``ssb_iq`` with an I/Q phase error of
    STATUS_PHASE_DEG[channel % 5] degrees on Q (Q = A sin(theta + phi); the Moseley & Slump
    estimate asin(teta1 / teta3) sees -phi), and every `burst_every` frames a `burst_len`-frame
    burst at 1.5 + (channel*7 + k) % 6 times the level, so |I| crosses the quarter / half / full
    ADC clip thresholds (1024 / 2048 / 4096 LSB16) on different calls per channel.  Peak stays
    below 32767 (no full-scale samples)."""
    channels = np.asarray(channels, dtype=np.int64)
    f1, f2, a1, a2, p1, p2 = channel_params(channels, "ssb2tone")
    phi = np.deg2rad(np.array(STATUS_PHASE_DEG)[channels % len(STATUS_PHASE_DEG)])[:, None]
    n = np.arange(start, start + nframes, dtype=np.float64)[None, :]
    k = (np.arange(start, start + nframes) // burst_every)[None, :]
    inb = (np.arange(start, start + nframes) % burst_every) < burst_len
    gain = np.where(inb[None, :], 1.5 + ((channels[:, None] * 7 + k) % 6), 1.0)
    ph1 = 2.0 * np.pi * (12000.0 + f1[:, None]) / FS * n + p1[:, None]
    ph2 = 2.0 * np.pi * (12000.0 + f2[:, None]) / FS * n + p2[:, None]
    i_sig = gain * (a1[:, None] * np.cos(ph1) + a2[:, None] * np.cos(ph2))
    q_sig = gain * (a1[:, None] * np.sin(ph1 + phi) + a2[:, None] * np.sin(ph2 + phi))
    if noise_sigma > 0:
        ni, nq = _noise(channels, start, nframes, noise_sigma)
        i_sig, q_sig = i_sig + ni, q_sig + nq
    return _frames(i_sig, q_sig)


def tx_audio(channels, start: int, nframes: int, kind: str = "ssb2tone", noise_sigma: float = 10.0):
    """C4 SSB-TX input: the codec's microphone frames (AudioSample_t {int32 l, r}, the sample in
    both channels as (int16) value << 16) carrying a per-channel two-tone audio signal."""
    channels = np.asarray(channels, dtype=np.int64)
    f1, f2, a1, a2, p1, p2 = channel_params(channels, kind)
    n = np.arange(start, start + nframes, dtype=np.float64)[None, :]
    s = (a1[:, None] * np.cos(2.0 * np.pi * f1[:, None] / FS * n + p1[:, None])
         + a2[:, None] * np.cos(2.0 * np.pi * f2[:, None] / FS * n + p2[:, None]))
    if noise_sigma > 0:
        s = s + _noise(channels, start, nframes, noise_sigma)[0]
    return _frames(s, s)


def ssb_iq_torch(c0: int, nch: int, start: int, nframes: int, device, noise_sigma: float = 30.0):
    """Same signal model as ``ssb_iq`` (kind "ssb2tone"), generated on the GPU for large
    benchmark batches: channels c0 .. c0+nch-1.  Tone parameters and noise come from the
    same splitmix64 counters; the float64 transcendentals are the device's, so a sample may
    differ from the numpy version by one LSB16 of rounding -- benchmark input only, parity
    tests use ``ssb_iq``."""
    import torch
    f1, f2, a1, a2, p1, p2 = (torch.from_numpy(x).to(device) for x in channel_params(np.arange(c0, c0 + nch)))
    n = torch.arange(start, start + nframes, dtype=torch.float64, device=device)[None, :]
    ph1 = (2.0 * np.pi * (12000.0 + f1[:, None]) / FS) * n + p1[:, None]
    ph2 = (2.0 * np.pi * (12000.0 + f2[:, None]) / FS) * n + p2[:, None]
    i_sig = a1[:, None] * torch.cos(ph1) + a2[:, None] * torch.cos(ph2)
    q_sig = a1[:, None] * torch.sin(ph1) + a2[:, None] * torch.sin(ph2)
    del ph1, ph2
    if noise_sigma > 0:
        g = torch.Generator(device=device)
        g.manual_seed(SEED_BASE + c0 * 7919 + start)
        i_sig += noise_sigma * torch.randn(i_sig.shape, dtype=torch.float64, device=device, generator=g)
        q_sig += noise_sigma * torch.randn(q_sig.shape, dtype=torch.float64, device=device, generator=g)
    out = torch.empty((nch, nframes, 2), dtype=torch.int32, device=device)
    out[:, :, 0] = torch.clamp(torch.round(i_sig), -32768, 32767).to(torch.int32) * 65536
    out[:, :, 1] = torch.clamp(torch.round(q_sig), -32768, 32767).to(torch.int32) * 65536
    return out
