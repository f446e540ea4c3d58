"""One transceiver behind the firmware's ISR entry: uhsdr_i2s_* (include/uhsdr.h), the
batched device chains driven the way AudioDriver_I2SCallback (audio_driver.c:2962-3049) drives
AudioDriver_RxProcessor / TxProcessor_Run, with the firmware's host DMA half-buffers."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _abi


class Transceiver:
    def __init__(self, rx: _abi.RxConfig | None = None, tx: _abi.TxConfig | None = None, block: int = 32,
                 stream: int | None = None):
        self.lib = _abi.load()
        self.rx_cfg = rx if rx is not None else _abi.default_config()
        self.tx_cfg = tx
        self.block = int(block)
        h = C.c_void_p()
        _abi.check(self.lib.uhsdr_i2s_create(C.byref(self.rx_cfg), C.byref(tx) if tx is not None else None,
                                             self.block, C.c_void_p(stream or 0), C.byref(h)), "uhsdr_i2s_create")
        self.handle = h

    def set_txrx_mode(self, tx: bool) -> None:
        _abi.check(self.lib.uhsdr_i2s_set_txrx_mode(self.handle, 1 if tx else 0), "uhsdr_i2s_set_txrx_mode")

    def set_input_mute(self, calls: int) -> None:
        _abi.check(self.lib.uhsdr_i2s_set_input_mute(self.handle, int(calls)), "uhsdr_i2s_set_input_mute")

    def callback(self, audio: np.ndarray, iq: np.ndarray, audio_dst: np.ndarray | None = None) -> None:
        """AudioDriver_I2SCallback(audio, iq, audioDst, blockSize) on int32 [block][2] host arrays,
        updated in place exactly as the firmware's DMA buffers are."""
        for a in (audio, iq) + ((audio_dst,) if audio_dst is not None else ()):
            if a.dtype != np.int32 or a.shape != (self.block, 2) or not a.flags.c_contiguous:
                raise ValueError(f"buffers must be contiguous int32 [{self.block}][2]")
        _abi.check(self.lib.uhsdr_i2s_callback(self.handle, C.c_void_p(audio.ctypes.data), C.c_void_p(iq.ctypes.data),
                                               C.c_void_p(audio_dst.ctypes.data) if audio_dst is not None else None,
                                               self.block), "uhsdr_i2s_callback")

    def close(self) -> None:
        if self.handle:
            self.lib.uhsdr_i2s_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
