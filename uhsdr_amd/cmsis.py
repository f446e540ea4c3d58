"""ctypes view of include/uhsdr_cmsis.h: the CMSIS-DSP signature shims of libuhsdr_cmsis.so.

The instance structs mirror CMSIS-DSP V1.4.5 (basesw/ovi40/Drivers/CMSIS/Include/arm_math.h)
field for field.  `Fir`, `FirDecimate`, `FirInterpolate`, `IirLattice`, `BiquadDf1`, `LmsNorm` wrap one
instance with its caller-owned state and coefficient arrays the way firmware code holds them
(audio_filter.c:1084-1115), and call the shims exactly like the firmware calls CMSIS.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "lib", "libuhsdr_cmsis.so")

FP = C.POINTER(C.c_float)


class arm_fir_instance_f32(C.Structure):
    _fields_ = [("numTaps", C.c_uint16), ("pState", FP), ("pCoeffs", FP)]


class arm_fir_decimate_instance_f32(C.Structure):
    _fields_ = [("M", C.c_uint8), ("numTaps", C.c_uint16), ("pCoeffs", FP), ("pState", FP)]


class arm_fir_interpolate_instance_f32(C.Structure):
    _fields_ = [("L", C.c_uint8), ("phaseLength", C.c_uint16), ("pCoeffs", FP), ("pState", FP)]


class arm_iir_lattice_instance_f32(C.Structure):
    _fields_ = [("numStages", C.c_uint16), ("pState", FP), ("pkCoeffs", FP), ("pvCoeffs", FP)]


class arm_biquad_casd_df1_inst_f32(C.Structure):
    _fields_ = [("numStages", C.c_uint32), ("pState", FP), ("pCoeffs", FP)]


class arm_cfft_instance_f32(C.Structure):
    _fields_ = [("fftLen", C.c_uint16), ("pTwiddle", FP), ("pBitRevTable", C.POINTER(C.c_uint16)),
                ("bitRevLength", C.c_uint16)]


class arm_lms_norm_instance_f32(C.Structure):
    _fields_ = [("numTaps", C.c_uint16), ("pState", FP), ("pCoeffs", FP), ("mu", C.c_float),
                ("energy", C.c_float), ("x0", C.c_float)]


P = C.POINTER
SIGNATURES = {
    "arm_fir_init_f32": (None, [P(arm_fir_instance_f32), C.c_uint16, FP, FP, C.c_uint32]),
    "arm_fir_f32": (None, [P(arm_fir_instance_f32), FP, FP, C.c_uint32]),
    "arm_fir_decimate_init_f32": (C.c_int, [P(arm_fir_decimate_instance_f32), C.c_uint16, C.c_uint8, FP, FP,
                                            C.c_uint32]),
    "arm_fir_decimate_f32": (None, [P(arm_fir_decimate_instance_f32), FP, FP, C.c_uint32]),
    "arm_fir_interpolate_init_f32": (C.c_int, [P(arm_fir_interpolate_instance_f32), C.c_uint8, C.c_uint16, FP, FP,
                                               C.c_uint32]),
    "arm_fir_interpolate_f32": (None, [P(arm_fir_interpolate_instance_f32), FP, FP, C.c_uint32]),
    "arm_iir_lattice_init_f32": (None, [P(arm_iir_lattice_instance_f32), C.c_uint16, FP, FP, FP, C.c_uint32]),
    "arm_iir_lattice_f32": (None, [P(arm_iir_lattice_instance_f32), FP, FP, C.c_uint32]),
    "arm_biquad_cascade_df1_init_f32": (None, [P(arm_biquad_casd_df1_inst_f32), C.c_uint8, FP, FP]),
    "arm_biquad_cascade_df1_f32": (None, [P(arm_biquad_casd_df1_inst_f32), FP, FP, C.c_uint32]),
    "arm_cfft_f32": (None, [P(arm_cfft_instance_f32), FP, C.c_uint8, C.c_uint8]),
    "arm_cmplx_mag_f32": (None, [FP, FP, C.c_uint32]),
    "arm_lms_norm_init_f32": (None, [P(arm_lms_norm_instance_f32), C.c_uint16, FP, FP, C.c_float, C.c_uint32]),
    "arm_lms_norm_f32": (None, [P(arm_lms_norm_instance_f32), FP, FP, FP, FP, C.c_uint32]),
    "uhsdr_cmsis_last_status": (C.c_int32, []),
}

_lib = None


def load(path: str | None = None) -> C.CDLL:
    """Load libuhsdr_cmsis.so (built in-tree by `make`); raises if it is missing."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise OSError(f"{p} not built: run `make` (the CMSIS shims have no CPU fallback)")
    from ._abi import _one_hip_runtime
    _one_hip_runtime()
    lib = C.CDLL(p)
    for name, (res, args) in SIGNATURES.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    if path is None:
        _lib = lib
    return lib


def _fp(a: np.ndarray):
    assert a.dtype == np.float32 and a.flags.c_contiguous
    return a.ctypes.data_as(FP)


def _check(lib):
    st = lib.uhsdr_cmsis_last_status()
    if st != 0:
        from . import _abi
        msg = _abi.load().uhsdr_last_error()
        raise RuntimeError(f"CMSIS shim failed ({st}): {msg.decode() if msg else ''}")


class _Inst:
    """One instance with its caller-owned arrays (kept alive here)."""

    in_place = False   # pDst == pSrc, as the firmware calls FIR / decimate / lattice / biquad

    def _run(self, fn, x: np.ndarray, nout: int) -> np.ndarray:
        x = np.array(x, np.float32, copy=True)
        if self.in_place and nout <= len(x):
            fn(C.byref(self.S), _fp(x), _fp(x), len(x))
            _check(self.lib)
            return x[:nout].copy()
        y = np.zeros(nout, np.float32)
        fn(C.byref(self.S), _fp(x), _fp(y), len(x))
        _check(self.lib)
        return y


class Fir(_Inst):
    def __init__(self, coeffs, block: int):
        self.lib = load()
        self.c = np.ascontiguousarray(coeffs, np.float32)
        self.state = np.zeros(len(self.c) + block - 1, np.float32)
        self.S = arm_fir_instance_f32()
        self.lib.arm_fir_init_f32(C.byref(self.S), len(self.c), _fp(self.c), _fp(self.state), block)

    def __call__(self, x):
        return self._run(self.lib.arm_fir_f32, x, len(x))


class FirDecimate(_Inst):
    def __init__(self, coeffs, M: int, block: int):
        self.lib = load()
        self.c = np.ascontiguousarray(coeffs, np.float32)
        self.M = M
        self.state = np.zeros(len(self.c) + block - 1, np.float32)
        self.S = arm_fir_decimate_instance_f32()
        st = self.lib.arm_fir_decimate_init_f32(C.byref(self.S), len(self.c), M, _fp(self.c), _fp(self.state), block)
        if st != 0:
            raise ValueError(f"arm_fir_decimate_init_f32: {st}")

    def __call__(self, x):
        return self._run(self.lib.arm_fir_decimate_f32, x, len(x) // self.M)


class FirInterpolate(_Inst):
    def __init__(self, coeffs, L: int, block: int):
        self.lib = load()
        self.c = np.ascontiguousarray(coeffs, np.float32)
        self.L = L
        self.state = np.zeros(len(self.c) // L + block - 1, np.float32)
        self.S = arm_fir_interpolate_instance_f32()
        st = self.lib.arm_fir_interpolate_init_f32(C.byref(self.S), L, len(self.c), _fp(self.c), _fp(self.state),
                                                   block)
        if st != 0:
            raise ValueError(f"arm_fir_interpolate_init_f32: {st}")

    def __call__(self, x):
        return self._run(self.lib.arm_fir_interpolate_f32, x, len(x) * self.L)


class IirLattice(_Inst):
    def __init__(self, k, v, block: int):
        self.lib = load()
        self.k = np.ascontiguousarray(k, np.float32)
        self.v = np.ascontiguousarray(v, np.float32)
        self.state = np.zeros(len(self.k) + block, np.float32)
        self.S = arm_iir_lattice_instance_f32()
        self.lib.arm_iir_lattice_init_f32(C.byref(self.S), len(self.k), _fp(self.k), _fp(self.v), _fp(self.state),
                                          block)

    def __call__(self, x):
        return self._run(self.lib.arm_iir_lattice_f32, x, len(x))


class BiquadDf1(_Inst):
    def __init__(self, coeffs):
        self.lib = load()
        self.c = np.ascontiguousarray(coeffs, np.float32)
        self.state = np.zeros(4 * (len(self.c) // 5), np.float32)
        self.S = arm_biquad_casd_df1_inst_f32()
        self.lib.arm_biquad_cascade_df1_init_f32(C.byref(self.S), len(self.c) // 5, _fp(self.c), _fp(self.state))

    def __call__(self, x):
        return self._run(self.lib.arm_biquad_cascade_df1_f32, x, len(x))


class LmsNorm:
    """arm_lms_norm_f32 on one instance: coefficients (adapted in place in `coeffs`), the
    carried window `state`, energy / x0 in the struct.  in_place: pErr == pSrc, the way
    AudioDriver_NotchFilter calls it (audio_driver.c:1755)."""

    in_place = False

    def __init__(self, coeffs, mu: float, block: int):
        self.lib = load()
        self.coeffs = np.array(coeffs, np.float32, copy=True)
        self.state = np.zeros(len(self.coeffs) + block - 1, np.float32)
        self.S = arm_lms_norm_instance_f32()
        self.lib.arm_lms_norm_init_f32(C.byref(self.S), len(self.coeffs), _fp(self.coeffs), _fp(self.state),
                                       float(mu), block)

    def __call__(self, x, ref):
        """one block: returns (out, err)"""
        x = np.array(x, np.float32, copy=True)
        d = np.ascontiguousarray(ref, np.float32)
        y = np.zeros(len(x), np.float32)
        e = x if self.in_place else np.zeros(len(x), np.float32)
        self.lib.arm_lms_norm_f32(C.byref(self.S), _fp(x), _fp(d), _fp(y), _fp(e), len(x))
        _check(self.lib)
        return y, e.copy()


def cfft(x: np.ndarray, ifft: bool = False, bitrev: bool = True, twiddle=None, bitrev_table=None) -> np.ndarray:
    """arm_cfft_f32 on a copy of x (interleaved complex float32, 2L values).  The instance carries
    fftLen and, when given, the CMSIS tables of arm_cfft_sR_f32_lenL (twiddleCoef_L as float32,
    the bit-reversal byte offsets as uint16): lengths other than 256 / 512 / 1024 run on them."""
    lib = load()
    p = np.array(x, np.float32, copy=True)
    S = arm_cfft_instance_f32()
    S.fftLen = len(p) // 2
    if twiddle is not None:
        tw = np.ascontiguousarray(twiddle, np.float32)
        S.pTwiddle = _fp(tw)
    if bitrev_table is not None:
        rv = np.ascontiguousarray(bitrev_table, np.uint16)
        S.pBitRevTable = rv.ctypes.data_as(C.POINTER(C.c_uint16))
        S.bitRevLength = len(rv)
    lib.arm_cfft_f32(C.byref(S), _fp(p), 1 if ifft else 0, 1 if bitrev else 0)
    _check(lib)
    return p


def cmplx_mag(x: np.ndarray) -> np.ndarray:
    lib = load()
    x = np.ascontiguousarray(x, np.float32)
    y = np.zeros(len(x) // 2, np.float32)
    lib.arm_cmplx_mag_f32(_fp(x), _fp(y), len(y))
    _check(lib)
    return y
