"""Host-side mirror of the reference RX interface for the batched device chain.

    chain = RxChain(config, channels=C, frames=N)    # AudioDriver_Init + SetProcessingChain
    chain.process(iq_dev, audio_dev, dst_dev)         # N/32 x AudioDriver_I2SCallback per channel

``iq`` is [C][N][2] int32 IqSample_t frames, ``audio`` [C][N] float (adb.a_buffer[1]),
``dst`` [C][N][2] int32 AudioSample_t frames -- the firmware's DMA formats, channel-major.
Device tensors are torch tensors on cuda:N (torch only provides memory and the stream);
all arithmetic runs in the HIP kernels of libuhsdr_amd.so.  Numpy arrays go through
``process_host`` (copy in, process, copy out).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _abi


# Schedule every new RxChain asks for (tests/conftest.py's `back` fixture sets it to cover each
# kernel schedule); None keeps the library's AUTO choice.  A schedule the handle's path cannot run
# leaves it on AUTO's choice.
DEFAULT_SCHEDULE = None


class RxChain:
    def __init__(self, config: _abi.RxConfig | None = None, channels: int = 1, frames: int = 32,
                 stream: int | None = None, schedule: int | None = None, **overrides):
        self.lib = _abi.load()
        self.config = config if config is not None else _abi.default_config(**overrides)
        self.channels = int(channels)
        self.frames = int(frames)
        h = C.c_void_p()
        _abi.check(self.lib.uhsdr_rx_create(C.byref(self.config), self.channels, self.frames,
                                            C.c_void_p(stream or 0), C.byref(h)), "uhsdr_rx_create")
        self.handle = h
        self._process = self.lib.uhsdr_rx_process
        self.plan = _abi.RxPlan()
        _abi.check(self.lib.uhsdr_rx_get_plan(h, C.byref(self.plan)), "uhsdr_rx_get_plan")
        if schedule is not None:
            self.set_schedule(schedule)
        elif DEFAULT_SCHEDULE is not None:
            self.lib.uhsdr_rx_set_schedule(h, int(DEFAULT_SCHEDULE))   # best effort (see above)

    def set_stream(self, stream: int) -> None:
        _abi.check(self.lib.uhsdr_rx_set_stream(self.handle, C.c_void_p(stream)), "uhsdr_rx_set_stream")

    def reset(self) -> None:
        _abi.check(self.lib.uhsdr_rx_reset(self.handle), "uhsdr_rx_reset")

    def _shape_ok(self, t, last):
        shp = tuple(t.shape)
        want = (self.channels, self.frames) + last
        if shp != want:
            raise ValueError(f"buffer shape {shp} != {want}")

    def process(self, iq, audio=None, dst=None) -> None:
        """Device buffers (torch tensors on the GPU, contiguous): enqueue on the handle's stream."""
        self._shape_ok(iq, (2,))
        for t in (iq, audio, dst):
            if t is not None and not t.is_contiguous():
                raise ValueError("buffers must be contiguous")
        if audio is not None:
            self._shape_ok(audio, ())
        if dst is not None:
            self._shape_ok(dst, (2,))
        _abi.check(self.lib.uhsdr_rx_process(
            self.handle, C.c_void_p(iq.data_ptr()),
            C.c_void_p(audio.data_ptr() if audio is not None else 0),
            C.c_void_p(dst.data_ptr() if dst is not None else 0)), "uhsdr_rx_process")

    def bind(self, iq, audio=None, dst=None):
        """Validate one buffer set once (shapes, contiguity: what process() checks every call) and
        return its raw pointers for process_ptr -- the hot loop's call then costs one ctypes call."""
        self._shape_ok(iq, (2,))
        for t, last in ((audio, ()), (dst, (2,))):
            if t is not None:
                self._shape_ok(t, last)
        for t in (iq, audio, dst):
            if t is not None and not t.is_contiguous():
                raise ValueError("buffers must be contiguous")
        return (iq.data_ptr(), audio.data_ptr() if audio is not None else 0, dst.data_ptr() if dst is not None else 0)

    def process_ptr(self, ptrs) -> None:
        """uhsdr_rx_process on a buffer set bind() validated (the caller keeps the tensors alive)."""
        st = self._process(self.handle, ptrs[0], ptrs[1], ptrs[2])
        if st:
            _abi.check(st, "uhsdr_rx_process")

    def process_stereo(self, iq, audio=None, audio0=None, dst=None) -> None:
        """OVI40 two-channel modes: audio = a_buffer[1] (channel 0), audio0 = a_buffer[0] (channel 1)."""
        self._shape_ok(iq, (2,))
        for t, last in ((audio, ()), (audio0, ()), (dst, (2,))):
            if t is not None:
                self._shape_ok(t, last)
                if not t.is_contiguous():
                    raise ValueError("buffers must be contiguous")
        ptr = lambda t: C.c_void_p(t.data_ptr() if t is not None else 0)  # noqa: E731
        _abi.check(self.lib.uhsdr_rx_process_stereo(self.handle, ptr(iq), ptr(audio), ptr(audio0), ptr(dst)),
                   "uhsdr_rx_process_stereo")

    def process_host(self, iq: np.ndarray):
        """Host numpy in/out: returns (audio [C][N] f32, dst [C][N][2] int32)."""
        iq = np.ascontiguousarray(iq, dtype=np.int32)
        self._shape_ok(iq, (2,))
        audio = np.empty((self.channels, self.frames), np.float32)
        dst = np.empty((self.channels, self.frames, 2), np.int32)
        _abi.check(self.lib.uhsdr_rx_process_host(
            self.handle, iq.ctypes.data_as(C.c_void_p), audio.ctypes.data_as(C.c_void_p),
            dst.ctypes.data_as(C.c_void_p)), "uhsdr_rx_process_host")
        return audio, dst

    def set_cw_outputs(self, signal=None, energy=None) -> None:
        """CW decoder front end outputs of the following calls: signal uint8 [C][N/32] (ads.CW_signal
        after each call), energy f32 [C][cw_blocks_max] (Goertzel energy per completed block)"""
        if signal is not None and tuple(signal.shape) != (self.channels, self.frames // 32):
            raise ValueError("signal must be [C][N/32]")
        if energy is not None and tuple(energy.shape) != (self.channels, max(self.cw_blocks_max, 1)):
            raise ValueError("energy must be [C][cw_blocks_max]")
        self._cw = (signal, energy)   # keep the tensors alive
        _abi.check(self.lib.uhsdr_rx_set_cw_outputs(self.handle, C.c_void_p(signal.data_ptr() if signal is not None else 0),
                                                    C.c_void_p(energy.data_ptr() if energy is not None else 0)),
                   "uhsdr_rx_set_cw_outputs")

    @property
    def cw_blocks_max(self) -> int:
        return self.lib.uhsdr_rx_cw_blocks_max(self.handle)

    @property
    def cw_blocks_last(self) -> int:
        return self.lib.uhsdr_rx_cw_blocks_last(self.handle)

    def set_clip_output(self, clip=None) -> None:
        """ADC clip flags (ads.adc_clip / _half_clip / _quarter_clip as ADC_* bits): the kernels OR
        the bits of every frame into clip, uint32 [C] on the device; the caller reads and clears it
        (the UI's role).  None stops the computation."""
        if clip is not None and (tuple(clip.shape) != (self.channels,) or clip.element_size() != 4):
            raise ValueError("clip must be a 4-byte integer tensor [C]")
        self._clip = clip
        _abi.check(self.lib.uhsdr_rx_set_clip_output(self.handle, C.c_void_p(clip.data_ptr() if clip is not None else 0)),
                   "uhsdr_rx_set_clip_output")

    def twinpeaks_state(self, out) -> None:
        """ts.twinpeaks_tested of every channel into out (int32 [C] on the device), stream-ordered."""
        if tuple(out.shape) != (self.channels,) or out.element_size() != 4:
            raise ValueError("out must be a 4-byte integer tensor [C]")
        _abi.check(self.lib.uhsdr_rx_twinpeaks_state(self.handle, C.c_void_p(out.data_ptr())), "uhsdr_rx_twinpeaks_state")

    def twinpeaks_rearm(self) -> None:
        """The UI's acknowledgement after a codec restart: CODEC_RESTART -> WAIT on every channel."""
        _abi.check(self.lib.uhsdr_rx_twinpeaks_rearm(self.handle), "uhsdr_rx_twinpeaks_rearm")

    def key_beep(self, calls: int) -> None:
        """AudioManagement_KeyBeep for every channel: the beep tone is added to the next `calls`
        32-frame calls (uhsdr_rx_key_beep)."""
        _abi.check(self.lib.uhsdr_rx_key_beep(self.handle, int(calls)), "uhsdr_rx_key_beep")

    def set_pipelined(self, enable=True) -> None:
        """Overlap call k+1's rx_front with call k's rx_back (uhsdr_rx_set_pipelined); outputs
        are complete after synchronize() / a device-wide sync, or join() for the handle's stream.
        enable: False / 0 off, True / 1 (cross-stream event hand-off), 2 (device hand-off: a poll
        that gives up poisons that call's audio with NaN, and process / join / synchronize then
        raise UhsdrError with status UHSDR_TIMEOUT until reset())."""
        _abi.check(self.lib.uhsdr_rx_set_pipelined(self.handle, int(enable)), "uhsdr_rx_set_pipelined")

    def set_precision(self, precision: int) -> None:
        """PRECISION_EXACT (bit-identical, default) or PRECISION_FMA (fused FIR MACs, 1e-5 normwise)."""
        _abi.check(self.lib.uhsdr_rx_set_precision(self.handle, int(precision)), "uhsdr_rx_set_precision")

    @property
    def precision(self) -> int:
        return self.lib.uhsdr_rx_get_precision(self.handle)

    def set_schedule(self, schedule: int) -> None:
        """SCHEDULE_AUTO / _SPLIT_PIPE / _SPLIT_FUSED / _CHAIN (uhsdr_rx_set_schedule): which kernels
        run a call; outputs are identical under every one."""
        _abi.check(self.lib.uhsdr_rx_set_schedule(self.handle, int(schedule)), "uhsdr_rx_set_schedule")

    def handoff_timeouts(self) -> int:
        """1 if a bounded device hand-off poll gave up since reset, else 0 (synchronises;
        uhsdr_rx_handoff_timeouts)."""
        return self.lib.uhsdr_rx_handoff_timeouts(self.handle)

    def set_handoff_bound(self, polls: int) -> None:
        """Polls before the device hand-off gives up (uhsdr_rx_set_handoff_bound; tests of the
        failure contract)."""
        _abi.check(self.lib.uhsdr_rx_set_handoff_bound(self.handle, int(polls)), "uhsdr_rx_set_handoff_bound")

    @property
    def schedule(self) -> int:
        """The resolved schedule (never AUTO)."""
        return self.lib.uhsdr_rx_get_schedule(self.handle)

    def set_front_block(self, outputs_per_lane: int) -> None:
        """FIR outputs per lane of the front passes, 8 or 16 (uhsdr_rx_set_front_block)."""
        _abi.check(self.lib.uhsdr_rx_set_front_block(self.handle, int(outputs_per_lane)), "uhsdr_rx_set_front_block")

    def join(self) -> None:
        _abi.check(self.lib.uhsdr_rx_join(self.handle), "uhsdr_rx_join")

    def synchronize(self) -> None:
        _abi.check(self.lib.uhsdr_rx_synchronize(self.handle), "uhsdr_rx_synchronize")

    def enable_timing(self, enable: bool = True, every: int = 1) -> None:
        """Bracket each kernel of every `every`-th call with HIP events (uhsdr_rx_enable_timing)."""
        _abi.check(self.lib.uhsdr_rx_enable_timing(self.handle, int(every) if enable else 0),
                   "uhsdr_rx_enable_timing")

    def kernel_times(self):
        """{kernel name: (total ms, launches)} accumulated since enable_timing()."""
        ms = (C.c_float * 8)()
        n = (C.c_int32 * 8)()
        k = self.lib.uhsdr_rx_kernel_times(self.handle, ms, n, 8)
        # kernel slots that ran (rx_front + rx_back, or rx_chain)
        return {self.lib.uhsdr_rx_kernel_name(i).decode(): (ms[i], n[i]) for i in range(k) if n[i] > 0}

    def close(self) -> None:
        if self.handle:
            self.lib.uhsdr_rx_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
