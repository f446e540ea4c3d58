"""ORACLE -- TEST INFRASTRUCTURE ONLY.

ctypes loader for oracle/build/libuhsdr_oracle.so, the clean-room CPU restatement of the
reference RX chain (oracle/uhsdr_oracle.c).  Only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg may import this module, and only as the checker / CPU baseline.
The product (libuhsdr_amd.so) never links or calls it.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "libuhsdr_oracle.so")
REF_BIN = os.path.join(HERE, "_ref", "uhsdr_ref")
_lib = None


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} not built: run `make`")
        lib = C.CDLL(LIB_PATH)
        lib.uo_rx_state_size.restype = C.c_size_t
        lib.uo_rx_state_init.argtypes = [C.c_void_p, C.c_void_p]
        lib.uo_rx_process.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]
        lib.uo_rx_process_batch.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_int,
                                            C.c_void_p, C.c_void_p, C.c_int]
        lib.uo_rx_process_batch2.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_int,
                                             C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
        lib.uo_rx_key_beep.argtypes = [C.c_void_p, C.c_int, C.c_int]
        lib.uo_rx_status.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_int]
        lib.uo_rx_bench.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_int, C.c_void_p,
                                    C.c_void_p, C.c_int, C.c_int, C.c_double, C.POINTER(C.c_double)]
        lib.uo_rx_bench.restype = C.c_longlong
        lib.uo_rx_process_batch_cw.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_void_p,
                                               C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int]
        lib.uo_tx_state_size.restype = C.c_size_t
        lib.uo_tx_state_init.argtypes = [C.c_void_p, C.c_void_p]
        lib.uo_tx_set_tune.argtypes = [C.c_void_p, C.c_int, C.c_int]
        lib.uo_tx_set_tone_burst.argtypes = [C.c_void_p, C.c_int, C.c_int]
        lib.uo_tx_process_batch.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_int,
                                            C.c_void_p, C.c_void_p, C.c_int]
        lib.uo_spec_state_size.restype = C.c_size_t
        lib.uo_spec_state_init.argtypes = [C.c_void_p, C.c_void_p]
        lib.uo_cfft.argtypes = [C.c_void_p, C.c_void_p]
        lib.uo_spec_process_batch.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_int,
                                              C.c_void_p, C.c_void_p, C.c_int]
        lib.uo_fir_batch.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_void_p]
        _lib = lib
    return _lib


class OracleRx:
    """C channels of the reference RX chain on the CPU, state carried across calls."""

    def __init__(self, plan, channels: int):
        self.lib = load()
        self.plan = plan
        self.channels = channels
        self.ssize = self.lib.uo_rx_state_size()
        self.states = (C.c_char * (self.ssize * channels))()
        for c in range(channels):
            self.lib.uo_rx_state_init(C.byref(plan), C.byref(self.states, c * self.ssize))

    def key_beep(self, calls: int) -> None:
        """AudioManagement_KeyBeep on every channel: the next `calls` calls get the beep."""
        self.lib.uo_rx_key_beep(self.states, self.channels, calls)

    def status(self, rearm: bool = False):
        """(clip flags [C], twinpeaks state [C]): reads and clears the clip flags; rearm = the UI's
        codec restart acknowledgement (CODEC_RESTART -> WAIT)."""
        clip = np.empty(self.channels, np.int32)
        tp = np.empty(self.channels, np.int32)
        self.lib.uo_rx_status(self.states, self.channels, clip.ctypes.data_as(C.c_void_p),
                              tp.ctypes.data_as(C.c_void_p), int(rearm))
        return clip, tp

    def process(self, iq: np.ndarray, threads: int = 1):
        a1, _, dst = self.process2(iq, threads)
        return a1, dst

    def process2(self, iq: np.ndarray, threads: int = 1):
        """(a_buffer[1], a_buffer[0], dst): a_buffer[0] is the second channel in stereo."""
        iq = np.ascontiguousarray(iq, dtype=np.int32)
        Cn, n, _ = iq.shape
        assert Cn == self.channels
        a1 = np.empty((Cn, n), np.float32)
        a0 = np.empty((Cn, n), np.float32)
        dst = np.empty((Cn, n, 2), np.int32)
        st = self.lib.uo_rx_process_batch2(C.byref(self.plan), self.states, Cn, iq.ctypes.data_as(C.c_void_p), n,
                                           a1.ctypes.data_as(C.c_void_p), a0.ctypes.data_as(C.c_void_p),
                                           dst.ctypes.data_as(C.c_void_p), threads)
        if st != 0:
            raise RuntimeError(f"uo_rx_process_batch2 status {st}")
        return a1, a0, dst


def rx_bench(plan, blocks: np.ndarray, threads: int, budget_s: float, pin: bool = True):
    """CPU baseline (bench.py): `threads` persistent workers pinned one per CPU of the affinity
    mask, each owning a contiguous channel slice, cycling through blocks [pool][C][n][2] until
    budget_s has passed.  Returns (channel-calls done, slowest worker's seconds)."""
    lib = load()
    blocks = np.ascontiguousarray(blocks, dtype=np.int32)
    pool, Cn, n, _ = blocks.shape
    ssize = lib.uo_rx_state_size()
    states = (C.c_char * (ssize * Cn))()
    for c in range(Cn):
        lib.uo_rx_state_init(C.byref(plan), C.byref(states, c * ssize))
    a1 = np.empty((Cn, n), np.float32)
    el = C.c_double(0.0)
    done = lib.uo_rx_bench(C.byref(plan), states, Cn, blocks.ctypes.data_as(C.c_void_p), pool, n,
                           a1.ctypes.data_as(C.c_void_p), None, threads, 1 if pin else 0, budget_s, C.byref(el))
    if done < 0:
        raise RuntimeError("uo_rx_bench: bad arguments")
    return int(done), float(el.value)


class OracleTx:
    """C channels of the reference SSB transmit chain on the CPU, state carried across calls."""

    def __init__(self, plan, channels: int):
        self.lib = load()
        self.plan = plan
        self.channels = channels
        self.ssize = self.lib.uo_tx_state_size()
        self.states = (C.c_char * (self.ssize * channels))()
        for c in range(channels):
            self.lib.uo_tx_state_init(C.byref(plan), C.byref(self.states, c * self.ssize))

    def set_tune(self, tune: int) -> None:
        self.lib.uo_tx_set_tune(self.states, self.channels, int(tune))

    def set_tone_burst(self, active: bool) -> None:
        self.lib.uo_tx_set_tone_burst(self.states, self.channels, int(bool(active)))

    def process(self, audio: np.ndarray, threads: int = 1):
        """audio: int32 [C][n][2] codec frames -> (iq int32 [C][n][2], a0 f32 [C][n])"""
        audio = np.ascontiguousarray(audio, dtype=np.int32)
        Cn, n, _ = audio.shape
        assert Cn == self.channels
        iq = np.empty((Cn, n, 2), np.int32)
        a0 = np.empty((Cn, n), np.float32)
        st = self.lib.uo_tx_process_batch(C.byref(self.plan), self.states, Cn, audio.ctypes.data_as(C.c_void_p), n,
                                          iq.ctypes.data_as(C.c_void_p), a0.ctypes.data_as(C.c_void_p), threads)
        if st != 0:
            raise RuntimeError(f"uo_tx_process_batch status {st}")
        return iq, a0


def rx_process_cw(orx, iq: np.ndarray, bmax: int, threads: int = 1):
    """OracleRx.process plus the CW decoder front end: -> (a1, dst, signal [C][n/32], energy [C][bmax])"""
    iq = np.ascontiguousarray(iq, dtype=np.int32)
    Cn, n, _ = iq.shape
    a1 = np.empty((Cn, n), np.float32)
    dst = np.empty((Cn, n, 2), np.int32)
    sig = np.zeros((Cn, n // 32), np.uint8)
    en = np.zeros((Cn, max(bmax, 1)), np.float32)
    st = orx.lib.uo_rx_process_batch_cw(C.byref(orx.plan), orx.states, Cn, iq.ctypes.data_as(C.c_void_p), n,
                                        a1.ctypes.data_as(C.c_void_p), dst.ctypes.data_as(C.c_void_p),
                                        sig.ctypes.data_as(C.c_void_p), en.ctypes.data_as(C.c_void_p), bmax, threads)
    if st != 0:
        raise RuntimeError(f"uo_rx_process_batch_cw: {st}")
    return a1, dst, sig, en[:, :bmax]


class OracleSpectrum:
    """C channels of the spectrum display path (producer ring + UiSpectrum states 0-3) on the CPU."""

    def __init__(self, plan, channels: int):
        self.lib = load()
        self.plan = plan
        self.channels = channels
        self.ssize = self.lib.uo_spec_state_size()
        self.states = (C.c_char * (self.ssize * channels))()
        for c in range(channels):
            self.lib.uo_spec_state_init(C.byref(plan), C.byref(self.states, c * self.ssize))

    def process(self, iq: np.ndarray, threads: int = 1):
        """-> (mag, avg) [C][F][L] for the F frames this call completed"""
        iq = np.ascontiguousarray(iq, dtype=np.int32)
        Cn, n, _ = iq.shape
        assert Cn == self.channels
        L = self.plan.fft_len
        fmax = max(1, n // max(1, self.plan.zoom_decimation) // L)
        mag = np.zeros((Cn, fmax, L), np.float32)
        avg = np.zeros((Cn, fmax, L), np.float32)
        f = self.lib.uo_spec_process_batch(C.byref(self.plan), self.states, Cn, iq.ctypes.data_as(C.c_void_p), n,
                                           mag.ctypes.data_as(C.c_void_p), avg.ctypes.data_as(C.c_void_p), threads)
        if f < 0:
            raise RuntimeError(f"uo_spec_process_batch: {f}")
        return mag[:, :f], avg[:, :f]

    def cfft(self, x: np.ndarray) -> np.ndarray:
        """arm_cfft_f32(S, x, 0, 1) restated, on one interleaved frame"""
        x = np.ascontiguousarray(x, dtype=np.float32).copy()
        self.lib.uo_cfft(C.byref(self.plan), x.ctypes.data_as(C.c_void_p))
        return x


class OracleFir:
    """C channels of CMSIS arm_fir_f32 sharing one tap set, state carried across calls."""

    def __init__(self, taps, channels: int):
        self.lib = load()
        self.c = np.ascontiguousarray(taps, np.float32)
        self.channels = channels
        self.hist = np.zeros((channels, len(self.c) - 1), np.float32)

    def process(self, x: np.ndarray) -> np.ndarray:
        x = np.ascontiguousarray(x, np.float32)
        assert x.shape[0] == self.channels
        y = np.empty_like(x)
        self.lib.uo_fir_batch(self.c.ctypes.data_as(C.c_void_p), len(self.c), self.hist.ctypes.data_as(C.c_void_p),
                              self.channels, x.ctypes.data_as(C.c_void_p), x.shape[1], y.ctypes.data_as(C.c_void_p))
        return y
