"""Host-side mirror of the reference SSB transmit interface for the batched device chain.

    chain = TxChain(config, channels=C, frames=N)   # TxProcessor_Init + TxProcessor_Set
    chain.process(audio_dev, iq_dev, a0_dev)         # N/32 x TX-mode AudioDriver_I2SCallback

``audio`` is [C][N][2] int32 AudioSample_t codec frames, ``iq`` [C][N][2] int32 IqSample_t DAC
frames, ``a0`` optional [C][N] f32 compressed audio (adb.a_buffer[0]).  All arithmetic runs in
libuhsdr_amd.so (uhsdr_tx.hip); torch tensors only provide device memory.
"""
from __future__ import annotations

import ctypes as C

from . import _abi


class TxChain:
    def __init__(self, config: _abi.TxConfig | None = None, channels: int = 1, frames: int = 32,
                 stream: int | None = None, **overrides):
        self.lib = _abi.load()
        self.config = config if config is not None else _abi.default_tx_config(**overrides)
        self.channels, self.frames = int(channels), int(frames)
        h = C.c_void_p()
        _abi.check(self.lib.uhsdr_tx_create(C.byref(self.config), self.channels, self.frames,
                                            C.c_void_p(stream or 0), C.byref(h)), "uhsdr_tx_create")
        self.handle = h
        self.plan = _abi.TxPlan()
        _abi.check(self.lib.uhsdr_tx_get_plan(h, C.byref(self.plan)), "uhsdr_tx_get_plan")

    def reset(self) -> None:
        _abi.check(self.lib.uhsdr_tx_reset(self.handle), "uhsdr_tx_reset")

    def process(self, audio, iq, a0=None) -> None:
        want = (self.channels, self.frames, 2)
        if tuple(audio.shape) != want or tuple(iq.shape) != want:
            raise ValueError(f"audio / iq must be {want}")
        if a0 is not None and tuple(a0.shape) != want[:2]:
            raise ValueError(f"a0 must be {want[:2]}")
        _abi.check(self.lib.uhsdr_tx_process(self.handle, C.c_void_p(audio.data_ptr()), C.c_void_p(iq.data_ptr()),
                                             C.c_void_p(a0.data_ptr() if a0 is not None else 0)), "uhsdr_tx_process")

    def set_pipelined(self, enable: bool) -> None:
        """tx_iq on a side stream, overlapping the next call's tx_voice (uhsdr_tx_set_pipelined);
        call join() before reading iq."""
        _abi.check(self.lib.uhsdr_tx_set_pipelined(self.handle, int(bool(enable))), "uhsdr_tx_set_pipelined")

    @property
    def pipelined(self) -> bool:
        return bool(self.lib.uhsdr_tx_get_pipelined(self.handle))

    def set_precision(self, precision: int) -> None:
        """PRECISION_EXACT (bit-identical, default) or PRECISION_FMA (fused MACs in the Hilbert pair,
        1e-5 normwise on the DAC frames; uhsdr_tx_set_precision)."""
        _abi.check(self.lib.uhsdr_tx_set_precision(self.handle, int(precision)), "uhsdr_tx_set_precision")

    @property
    def precision(self) -> int:
        return self.lib.uhsdr_tx_get_precision(self.handle)

    def join(self) -> None:
        """order the handle's stream after the pipelined mode's side stream (uhsdr_tx_join)"""
        _abi.check(self.lib.uhsdr_tx_join(self.handle), "uhsdr_tx_join")

    def set_tune(self, tune: int) -> None:
        """TUNE for the following calls: TUNE_OFF, TUNE_SINGLE (750 Hz) or TUNE_TWO (750 + 1950 Hz)."""
        _abi.check(self.lib.uhsdr_tx_set_tune(self.handle, int(tune)), "uhsdr_tx_set_tune")

    def set_tone_burst(self, active: bool) -> None:
        """FM tone burst (whistle-up) on / off for the following calls."""
        _abi.check(self.lib.uhsdr_tx_set_tone_burst(self.handle, int(bool(active))), "uhsdr_tx_set_tone_burst")

    def close(self) -> None:
        if self.handle:
            self.lib.uhsdr_tx_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
