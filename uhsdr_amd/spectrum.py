"""Host-side mirror of the reference spectrum display path for the batched device kernel.

    spec = Spectrum(config, channels=C, frames=N)   # UiSpectrum_InitSpectrumDisplayData
    nf = spec.process(iq_dev, mag_dev, avg_dev)     # N input frames: producer ring + states 0-3

``iq`` is the RX input, [C][N][2] int32 IqSample_t; ``mag`` / ``avg`` are optional [C][F][L] f32
(F = max(1, N/L)): sd.FFT_MagData and sd.FFT_AVGData after each display frame completed by the
call; ``nf`` is how many were completed.  All arithmetic runs in libuhsdr_amd.so
(uhsdr_spectrum.hip); torch tensors only provide device memory.
"""
from __future__ import annotations

import ctypes as C

from . import _abi


class Spectrum:
    def __init__(self, config: _abi.SpectrumConfig | None = None, channels: int = 1, frames: int = 1024,
                 stream: int | None = None, **overrides):
        self.lib = _abi.load()
        self.config = config if config is not None else _abi.default_spectrum_config(**overrides)
        self.channels, self.frames = int(channels), int(frames)
        h = C.c_void_p()
        _abi.check(self.lib.uhsdr_spectrum_create(C.byref(self.config), self.channels, self.frames,
                                                  C.c_void_p(stream or 0), C.byref(h)), "uhsdr_spectrum_create")
        self.handle = h
        self.plan = _abi.SpectrumPlan()
        _abi.check(self.lib.uhsdr_spectrum_get_plan(h, C.byref(self.plan)), "uhsdr_spectrum_get_plan")
        self.fft_len = self.plan.fft_len
        self.decimation = 1 << int(self.config.magnify)          # zoom: ring samples per frame
        self.frames_out = max(1, self.frames // self.decimation // self.fft_len)

    @property
    def out_shape(self):
        return (self.channels, self.frames_out, self.fft_len)

    def reset(self) -> None:
        _abi.check(self.lib.uhsdr_spectrum_reset(self.handle), "uhsdr_spectrum_reset")

    def process(self, iq, mag=None, avg=None) -> int:
        if tuple(iq.shape) != (self.channels, self.frames, 2):
            raise ValueError(f"iq must be {(self.channels, self.frames, 2)}")
        for t in (mag, avg):
            if t is not None and tuple(t.shape) != self.out_shape:
                raise ValueError(f"mag / avg must be {self.out_shape}")
        nf = C.c_int32(0)
        _abi.check(self.lib.uhsdr_spectrum_process(
            self.handle, C.c_void_p(iq.data_ptr()), C.c_void_p(mag.data_ptr() if mag is not None else 0),
            C.c_void_p(avg.data_ptr() if avg is not None else 0), C.byref(nf)), "uhsdr_spectrum_process")
        return nf.value

    def close(self) -> None:
        if self.handle:
            self.lib.uhsdr_spectrum_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
