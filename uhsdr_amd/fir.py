"""Batched CMSIS arm_fir_f32 over channels on the device (uhsdr_fir_*, include/uhsdr.h):
EXACT (bit-identical to the reference) or MFMA (FIR as a GEMM on the matrix cores)."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _abi

EXACT, MFMA = 0, 1


class FirBatch:
    def __init__(self, taps, channels: int, block: int, mode: int = EXACT, stream: int | None = None):
        self.lib = _abi.load()
        self.taps = np.ascontiguousarray(taps, np.float32)
        self.channels, self.block, self.mode = int(channels), int(block), int(mode)
        h = C.c_void_p()
        _abi.check(self.lib.uhsdr_fir_create(self.taps.ctypes.data_as(C.c_void_p), len(self.taps), self.channels,
                                             self.block, self.mode, C.c_void_p(stream or 0), C.byref(h)),
                   "uhsdr_fir_create")
        self.handle = h

    @property
    def waves(self) -> int:
        """waves per workgroup of the FIR kernel (1, 2 or 4)"""
        return int(self.lib.uhsdr_fir_get_waves(self.handle))

    def set_waves(self, waves: int) -> None:
        _abi.check(self.lib.uhsdr_fir_set_waves(self.handle, int(waves)), "uhsdr_fir_set_waves")

    def reset(self) -> None:
        _abi.check(self.lib.uhsdr_fir_reset(self.handle), "uhsdr_fir_reset")

    def process(self, src, dst) -> None:
        """src, dst: torch float32 cuda tensors [C][B] (device memory only)."""
        want = (self.channels, self.block)
        if tuple(src.shape) != want or tuple(dst.shape) != want:
            raise ValueError(f"src / dst must be {want}")
        _abi.check(self.lib.uhsdr_fir_process(self.handle, C.c_void_p(src.data_ptr()), C.c_void_p(dst.data_ptr())),
                   "uhsdr_fir_process")

    def close(self) -> None:
        if self.handle:
            self.lib.uhsdr_fir_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
