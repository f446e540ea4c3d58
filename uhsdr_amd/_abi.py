"""ctypes view of include/uhsdr.h (the C ABI of libuhsdr_amd.so).

Python is only the test / benchmark driver here: every call below crosses the same C ABI
that firmware-side C code links against.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "lib", "libuhsdr_amd.so")

MAX_FIR_TAPS = 200
MAX_DEC_TAPS = 96
MAX_LATTICE = 10
MAX_INTERP = 16
IQ_BLOCK_SIZE = 32
FILTER_PATH_NUM = 87

ABI_VERSION = 5   # include/uhsdr.h UHSDR_ABI_VERSION: checked against the library at load()
UHSDR_OK = 0
UHSDR_ARGUMENT_ERROR = -1
UHSDR_LENGTH_ERROR = -2
UHSDR_UNSUPPORTED = -10
UHSDR_DEVICE_ERROR = -11
UHSDR_TIMEOUT = -12          # a bounded device-side hand-off poll gave up (uhsdr_rx_set_pipelined 2)

DEMOD_USB, DEMOD_LSB, DEMOD_CW, DEMOD_AM, DEMOD_SAM, DEMOD_FM, DEMOD_DIGI, DEMOD_SSBSTEREO, DEMOD_IQ = range(9)
SAM_SIDEBAND_BOTH, SAM_SIDEBAND_LSB, SAM_SIDEBAND_USB, SAM_SIDEBAND_STEREO = range(4)
BOARD_OVI40, BOARD_MCHF = 0, 1                 # uhsdr_rx_config.board: the UI board's output stage
DSP_NOTCH_ENABLE, DSP_MNOTCH_ENABLE, DSP_MPEAK_ENABLE = 0x04, 0x10, 0x20
PRECISION_EXACT, PRECISION_FMA = 0, 1          # uhsdr_rx_set_precision
SCHEDULE_AUTO, SCHEDULE_SPLIT_PIPE, SCHEDULE_SPLIT_FUSED, SCHEDULE_CHAIN = range(4)   # uhsdr_rx_set_schedule
ADC_CLIP, ADC_HALF_CLIP, ADC_QUARTER_CLIP = 1, 2, 4   # uhsdr_rx_set_clip_output bits
TWINPEAKS_SAMPLING, TWINPEAKS_DONE, TWINPEAKS_WAIT, TWINPEAKS_UNCORRECTABLE, TWINPEAKS_CODEC_RESTART = range(5)


class RxConfig(C.Structure):
    _fields_ = [
        ("dmod_mode", C.c_int32), ("filter_path", C.c_int32), ("iq_freq_mode", C.c_int32),
        ("iq_auto_correction", C.c_int32), ("iq_gain_i", C.c_float), ("iq_gain_q", C.c_float),
        ("iq_phase_balance", C.c_float), ("dsp_active", C.c_int32), ("notch_frequency", C.c_int32),
        ("peak_frequency", C.c_int32), ("bass_gain", C.c_int32), ("treble_gain", C.c_int32),
        ("cw_lsb", C.c_int32), ("digi_lsb", C.c_int32), ("agc_mode", C.c_int32), ("agc_slope", C.c_int32),
        ("agc_thresh", C.c_int32), ("agc_hang_enable", C.c_int32), ("agc_hang_time", C.c_int32),
        ("agc_hang_thresh", C.c_int32), ("agc_tau_decay", C.c_int32 * 6), ("agc_tau_hang_decay", C.c_int32),
        ("sam_sideband", C.c_int32), ("sam_pll_fmax", C.c_int32), ("sam_zeta", C.c_int32), ("sam_omega_n", C.c_int32),
        ("fade_leveler", C.c_int32), ("fm_sql_threshold", C.c_int32), ("fm_deviation_5k", C.c_int32),
        ("cw_sidetone_freq", C.c_int32), ("cw_decoder_blocksize", C.c_int32), ("cw_decoder_thresh", C.c_int32),
        ("cw_decoder_noisecancel", C.c_int32),
        ("notch_mu", C.c_int32), ("fm_tone_det", C.c_int32), ("beep_frequency", C.c_int32),
        ("beep_loudness", C.c_int32), ("stereo_enable", C.c_int32),
        ("board", C.c_int32), ("spkr_gain", C.c_int32), ("reserved", C.c_int32 * 9),
    ]


_AGC_INT = ["mode", "hang_enable", "remove_dc", "ring_buffsize", "attack_buffsize", "out_index0",
            "in_index0", "hang_counter_init"]
_AGC_FLT = ["sample_rate", "fixed_gain", "attack_mult", "decay_mult", "fast_decay_mult", "fast_backmult",
            "onemfast_backmult", "hang_backmult", "onemhang_backmult", "hang_decay_mult", "pop_ratio",
            "hang_level", "min_volts", "inv_max_input", "out_target", "slope_constant", "hangtime",
            "hang_thresh", "var_gain", "max_gain", "inv_out_target"]


class AgcPlan(C.Structure):
    _fields_ = [(n, C.c_int32) for n in _AGC_INT] + [(n, C.c_float) for n in _AGC_FLT]


class RxPlan(C.Structure):
    _fields_ = [
        ("dmod_mode", C.c_int32), ("filter_path", C.c_int32), ("lsb", C.c_int32),
        ("decimation_rate", C.c_int32), ("decimated_freq", C.c_int32), ("use_decimated_iq", C.c_int32),
        ("iq_auto_correction", C.c_int32), ("iq_gain_i", C.c_float), ("iq_gain_q", C.c_float),
        ("iq_phase_balance", C.c_float), ("freq_shift_hz", C.c_int32), ("shift_kind", C.c_int32),
        ("shift_up", C.c_int32), ("osc_cos", C.c_float), ("osc_sin", C.c_float),
        ("hilbert_taps", C.c_int32), ("hilbert_i", C.c_float * MAX_FIR_TAPS), ("hilbert_q", C.c_float * MAX_FIR_TAPS),
        ("dec_taps", C.c_int32), ("dec", C.c_float * MAX_DEC_TAPS),
        ("pre_stages", C.c_int32), ("pre_k", C.c_float * MAX_LATTICE), ("pre_v", C.c_float * (MAX_LATTICE + 1)),
        ("interp_L", C.c_int32), ("interp_phase", C.c_int32), ("interp", C.c_float * MAX_INTERP),
        ("aa_stages", C.c_int32), ("aa_k", C.c_float * MAX_LATTICE), ("aa_v", C.c_float * (MAX_LATTICE + 1)),
        ("biquad1", C.c_float * 20), ("biquad2", C.c_float * 5),
        ("post_agc_scale", C.c_float), ("line_out_scale", C.c_float),
        ("agc", AgcPlan),
        ("dec_q", C.c_float * MAX_DEC_TAPS), ("sam_sideband", C.c_int32), ("fade_leveler", C.c_int32),
        ("sam_omega_min", C.c_float), ("sam_omega_max", C.c_float), ("sam_g1", C.c_float), ("sam_g2", C.c_float),
        ("fade_mtauR", C.c_float), ("fade_onem_mtauR", C.c_float), ("fade_mtauI", C.c_float),
        ("fade_onem_mtauI", C.c_float),
        ("fm_scale", C.c_float), ("fm_sql_threshold", C.c_int32), ("sq_stages", C.c_int32),
        ("sq_k", C.c_float * MAX_LATTICE), ("sq_v", C.c_float * (MAX_LATTICE + 1)),
        ("cw_enabled", C.c_int32), ("cw_blocksize", C.c_int32), ("cw_noisecancel", C.c_int32),
        ("cw_thresh", C.c_float), ("cw_r", C.c_float), ("cw_cos", C.c_float), ("cw_sin", C.c_float),
        ("notch_enabled", C.c_int32), ("notch_taps", C.c_int32), ("notch_delay_len", C.c_int32),
        ("notch_mu", C.c_float), ("tone_det_enabled", C.c_int32), ("tone_r", C.c_float * 3),
        ("tone_cos", C.c_float * 3), ("tone_sin", C.c_float * 3), ("beep_step", C.c_uint32),
        ("beep_scale", C.c_float), ("stereo", C.c_int32), ("dds_table", C.c_int16 * 1024),
        ("single_channel", C.c_int32), ("line_out0_scale", C.c_float), ("spkr_scale", C.c_float),
        ("reserved", C.c_int32 * 29),
    ]


TX_HILBERT_TAPS = 201
TX_AUDIO_MIC, TX_AUDIO_LINEIN_L, TX_AUDIO_LINEIN_R, TX_AUDIO_DIG, TX_AUDIO_DIGIQ = range(5)


class TxConfig(C.Structure):
    _fields_ = [
        ("dmod_mode", C.c_int32), ("iq_freq_mode", C.c_int32), ("audio_source", C.c_int32),
        ("mic_gain_mult", C.c_int32), ("mic_boost", C.c_int32), ("comp_level", C.c_int32), ("alc_decay", C.c_int32),
        ("alc_postfilt_gain", C.c_int32), ("tx_filter", C.c_int32), ("bass_gain", C.c_int32),
        ("treble_gain", C.c_int32), ("filter_disable", C.c_int32), ("power_factor", C.c_float),
        ("gain_i", C.c_float), ("gain_q", C.c_float), ("phase_balance", C.c_float),
        ("fm_deviation_5k", C.c_int32), ("fm_subaudible_tone", C.c_int32), ("fm_tone_burst_mode", C.c_int32),
        ("reserved", C.c_int32 * 13),
    ]


class TxPlan(C.Structure):
    _fields_ = [
        ("dmod_mode", C.c_int32), ("lsb", C.c_int32), ("audio_source", C.c_int32), ("in_gain", C.c_float),
        ("apply_in_gain", C.c_int32), ("run_lattice", C.c_int32), ("run_biquad", C.c_int32),
        ("lat_stages", C.c_int32), ("lat_k", C.c_float * MAX_LATTICE), ("lat_v", C.c_float * (MAX_LATTICE + 1)),
        ("biquad", C.c_float * 15), ("comp_on", C.c_int32), ("postfilt_gain", C.c_float), ("alc_decay", C.c_float),
        ("alc_gain_scaling", C.c_float), ("hilbert_i", C.c_float * (TX_HILBERT_TAPS + 7)),
        ("hilbert_q", C.c_float * (TX_HILBERT_TAPS + 7)), ("freq_shift_hz", C.c_int32), ("shift_kind", C.c_int32),
        ("shift_up", C.c_int32), ("osc_cos", C.c_float), ("osc_sin", C.c_float), ("final_i_gain", C.c_float),
        ("final_q_gain", C.c_float), ("phase_balance", C.c_float),
        ("fm", C.c_int32), ("fm_mod_mult", C.c_float), ("fm_word", C.c_uint32), ("fm_swap", C.c_int32),
        ("fm_sub_on", C.c_int32), ("fm_sub_step", C.c_uint32), ("fm_sub_scale", C.c_float),
        ("dds_table", C.c_int16 * 1024), ("tune_step", C.c_uint32 * 2), ("tone_burst_step", C.c_uint32),
        ("tone_burst_scale", C.c_float), ("am", C.c_int32), ("digiq", C.c_int32), ("digiq_i_gain", C.c_float),
        ("digiq_q_gain", C.c_float), ("reserved", C.c_int32 * 24),
    ]


SPECTRUM_MAX_LEN = 1024
SPECTRUM_MAX_BITREV = 1800


class SpectrumConfig(C.Structure):
    _fields_ = [
        ("fft_len", C.c_int32), ("spectrum_filter", C.c_int32), ("iq_auto_correction", C.c_int32),
        ("iq_gain_i", C.c_float), ("iq_gain_q", C.c_float), ("iq_phase_balance", C.c_float),
        ("magnify", C.c_int32), ("iq_freq_mode", C.c_int32),
        ("reserved", C.c_int32 * 8),
    ]


class SpectrumPlan(C.Structure):
    _fields_ = [
        ("fft_len", C.c_int32), ("window_formula", C.c_int32), ("iq_auto_correction", C.c_int32),
        ("iq_gain_i", C.c_float), ("iq_gain_q", C.c_float), ("iq_phase_balance", C.c_float),
        ("filt_factor", C.c_float), ("bitrev_len", C.c_int32),
        ("window", C.c_float * (2 * SPECTRUM_MAX_LEN)), ("twiddle", C.c_float * (2 * SPECTRUM_MAX_LEN)),
        ("bitrev", C.c_uint16 * SPECTRUM_MAX_BITREV), ("perm", C.c_uint16 * SPECTRUM_MAX_LEN),
        ("iperm", C.c_uint16 * SPECTRUM_MAX_LEN), ("tw_lane", C.c_float * (8 * 64 * 2)),
        ("magnify", C.c_int32), ("zoom_decimation", C.c_int32), ("zoom_taps", C.c_int32),
        ("freq_shift_hz", C.c_int32), ("shift_kind", C.c_int32), ("shift_up", C.c_int32),
        ("osc_cos", C.c_float), ("osc_sin", C.c_float),
        ("zoom_biquad", C.c_float * 20), ("zoom_fir", C.c_float * 8),
        ("reserved", C.c_int32 * 16),
    ]


# every exported entry point of include/uhsdr.h: name -> (restype, argtypes)
SIGNATURES = {
    "uhsdr_rx_config_default": (None, [C.POINTER(RxConfig)]),
    "uhsdr_rx_plan_build": (C.c_int, [C.POINTER(RxConfig), C.POINTER(RxPlan)]),
    "uhsdr_rx_plan_supported": (C.c_int, [C.POINTER(RxPlan)]),
    "uhsdr_rx_plan_fma_ok": (C.c_int, [C.POINTER(RxPlan)]),
    "uhsdr_rx_create": (C.c_int, [C.POINTER(RxConfig), C.c_int32, C.c_int32, C.c_void_p, C.POINTER(C.c_void_p)]),
    "uhsdr_rx_reset": (C.c_int, [C.c_void_p]),
    "uhsdr_rx_process": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "uhsdr_rx_process_host": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "uhsdr_rx_process_stereo": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "uhsdr_rx_get_plan": (C.c_int, [C.c_void_p, C.POINTER(RxPlan)]),
    "uhsdr_rx_set_stream": (C.c_int, [C.c_void_p, C.c_void_p]),
    "uhsdr_rx_destroy": (C.c_int, [C.c_void_p]),
    "uhsdr_version": (C.c_char_p, []),
    "uhsdr_last_error": (C.c_char_p, []),
    "uhsdr_sizeof_config": (C.c_int32, []),
    "uhsdr_abi_version": (C.c_int32, []),
    "uhsdr_sizeof_plan": (C.c_int32, []),
    "uhsdr_rx_kernel_count": (C.c_int32, [C.c_void_p]),
    "uhsdr_rx_enable_timing": (C.c_int, [C.c_void_p, C.c_int32]),
    "uhsdr_rx_kernel_times": (C.c_int32, [C.c_void_p, C.POINTER(C.c_float), C.POINTER(C.c_int32), C.c_int32]),
    "uhsdr_rx_kernel_name": (C.c_char_p, [C.c_int32]),
    "uhsdr_rx_synchronize": (C.c_int, [C.c_void_p]),
    "uhsdr_rx_set_pipelined": (C.c_int, [C.c_void_p, C.c_int32]),
    "uhsdr_rx_join": (C.c_int, [C.c_void_p]),
    "uhsdr_rx_set_precision": (C.c_int, [C.c_void_p, C.c_int32]),
    "uhsdr_rx_get_precision": (C.c_int32, [C.c_void_p]),
    "uhsdr_rx_set_schedule": (C.c_int, [C.c_void_p, C.c_int32]),
    "uhsdr_rx_get_schedule": (C.c_int32, [C.c_void_p]),
    "uhsdr_rx_handoff_timeouts": (C.c_int32, [C.c_void_p]),
    "uhsdr_rx_set_handoff_bound": (C.c_int, [C.c_void_p, C.c_uint32]),
    "uhsdr_rx_debug_persist": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint32)]),
    "uhsdr_rx_set_front_block": (C.c_int, [C.c_void_p, C.c_int32]),
    "uhsdr_rx_set_cw_outputs": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
    "uhsdr_rx_cw_blocks_max": (C.c_int32, [C.c_void_p]),
    "uhsdr_rx_cw_blocks_last": (C.c_int32, [C.c_void_p]),
    "uhsdr_rx_key_beep": (C.c_int, [C.c_void_p, C.c_int32]),
    "uhsdr_rx_set_clip_output": (C.c_int, [C.c_void_p, C.c_void_p]),
    "uhsdr_rx_twinpeaks_state": (C.c_int, [C.c_void_p, C.c_void_p]),
    "uhsdr_rx_twinpeaks_rearm": (C.c_int, [C.c_void_p]),
    "uhsdr_device_alloc": (C.c_void_p, [C.c_uint64]),
    "uhsdr_device_free": (None, [C.c_void_p]),
    "uhsdr_copy_to_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64]),
    "uhsdr_copy_to_host": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64]),
    "uhsdr_tx_config_default": (None, [C.POINTER(TxConfig)]),
    "uhsdr_tx_plan_build": (C.c_int, [C.POINTER(TxConfig), C.POINTER(TxPlan)]),
    "uhsdr_tx_create": (C.c_int, [C.POINTER(TxConfig), C.c_int32, C.c_int32, C.c_void_p, C.POINTER(C.c_void_p)]),
    "uhsdr_tx_reset": (C.c_int, [C.c_void_p]),
    "uhsdr_tx_process": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "uhsdr_tx_get_plan": (C.c_int, [C.c_void_p, C.POINTER(TxPlan)]),
    "uhsdr_tx_destroy": (C.c_int, [C.c_void_p]),
    "uhsdr_tx_prepare_run": (C.c_int, [C.c_void_p]),
    "uhsdr_tx_set_tune": (C.c_int, [C.c_void_p, C.c_int32]),
    "uhsdr_tx_set_tone_burst": (C.c_int, [C.c_void_p, C.c_int32]),
    "uhsdr_tx_set_pipelined": (C.c_int, [C.c_void_p, C.c_int32]),
    "uhsdr_tx_get_pipelined": (C.c_int32, [C.c_void_p]),
    "uhsdr_tx_join": (C.c_int, [C.c_void_p]),
    "uhsdr_tx_set_precision": (C.c_int, [C.c_void_p, C.c_int32]),
    "uhsdr_tx_get_precision": (C.c_int32, [C.c_void_p]),
    "uhsdr_fir_create": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_void_p,
                                   C.POINTER(C.c_void_p)]),
    "uhsdr_fir_reset": (C.c_int, [C.c_void_p]),
    "uhsdr_fir_process": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
    "uhsdr_fir_synchronize": (C.c_int, [C.c_void_p]),
    "uhsdr_fir_destroy": (C.c_int, [C.c_void_p]),
    "uhsdr_fir_set_waves": (C.c_int, [C.c_void_p, C.c_int32]),
    "uhsdr_fir_get_waves": (C.c_int32, [C.c_void_p]),
    "uhsdr_i2s_create": (C.c_int, [C.POINTER(RxConfig), C.POINTER(TxConfig), C.c_int32, C.c_void_p,
                                   C.POINTER(C.c_void_p)]),
    "uhsdr_i2s_set_txrx_mode": (C.c_int, [C.c_void_p, C.c_int32]),
    "uhsdr_i2s_set_input_mute": (C.c_int, [C.c_void_p, C.c_int32]),
    "uhsdr_i2s_callback": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int16]),
    "uhsdr_i2s_destroy": (C.c_int, [C.c_void_p]),
    "uhsdr_sizeof_tx_config": (C.c_int32, []),
    "uhsdr_sizeof_tx_plan": (C.c_int32, []),
    "uhsdr_spectrum_config_default": (None, [C.POINTER(SpectrumConfig)]),
    "uhsdr_spectrum_plan_build": (C.c_int, [C.POINTER(SpectrumConfig), C.POINTER(SpectrumPlan)]),
    "uhsdr_spectrum_create": (C.c_int, [C.POINTER(SpectrumConfig), C.c_int32, C.c_int32, C.c_void_p,
                                        C.POINTER(C.c_void_p)]),
    "uhsdr_spectrum_reset": (C.c_int, [C.c_void_p]),
    "uhsdr_spectrum_process": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.POINTER(C.c_int32)]),
    "uhsdr_spectrum_get_plan": (C.c_int, [C.c_void_p, C.POINTER(SpectrumPlan)]),
    "uhsdr_spectrum_destroy": (C.c_int, [C.c_void_p]),
    "uhsdr_sizeof_spectrum_config": (C.c_int32, []),
    "uhsdr_sizeof_spectrum_plan": (C.c_int32, []),
}

_lib = None


def _one_hip_runtime() -> None:
    """torch ships its own libamdhip64 (file libamdhip64.so, soname libamdhip64.so.7).  Loaded
    after it, this library's NEEDED libamdhip64.so.7 binds to torch's copy; loaded first, it
    maps /opt/rocm's and torch later maps a second runtime, whose device pointers this one does
    not know ("no ROCm-capable device" on the first allocation).  So torch goes first."""
    try:
        import torch  # noqa: F401
    except ImportError:
        pass


def load(path: str | None = None) -> C.CDLL:
    """Load libuhsdr_amd.so (built in-tree by `make`); raises if it is missing."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    # UHSDR_LIB: an alternative build of the same library (A/B measurements of compile variants)
    p = path or os.environ.get("UHSDR_LIB") or LIB_PATH
    if not os.path.exists(p):
        raise RuntimeError(f"{p} not built: run `make` (or __graft_entry__.build())")
    _one_hip_runtime()
    lib = C.CDLL(p)
    variant = p != LIB_PATH
    for name, (res, args) in SIGNATURES.items():
        if variant and not hasattr(lib, name):
            continue        # an A/B build of an earlier revision: entry points added since are absent
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if not variant and lib.uhsdr_abi_version() != ABI_VERSION:
        raise RuntimeError(f"{p} was built for ABI {lib.uhsdr_abi_version()}, this binding mirrors include/uhsdr.h "
                           f"ABI {ABI_VERSION}: rebuild with `make`")
    if lib.uhsdr_sizeof_config() != C.sizeof(RxConfig) or lib.uhsdr_sizeof_plan() != C.sizeof(RxPlan):
        raise RuntimeError("ctypes layout of uhsdr_rx_config / uhsdr_rx_plan does not match include/uhsdr.h")
    if lib.uhsdr_sizeof_tx_config() != C.sizeof(TxConfig) or lib.uhsdr_sizeof_tx_plan() != C.sizeof(TxPlan):
        raise RuntimeError("ctypes layout of uhsdr_tx_config / uhsdr_tx_plan does not match include/uhsdr.h")
    if (lib.uhsdr_sizeof_spectrum_config() != C.sizeof(SpectrumConfig)
            or lib.uhsdr_sizeof_spectrum_plan() != C.sizeof(SpectrumPlan)):
        raise RuntimeError("ctypes layout of uhsdr_spectrum_config / _plan does not match include/uhsdr.h")
    if path is None:
        _lib = lib
    return lib


class UhsdrError(RuntimeError):
    """A uhsdr_status other than UHSDR_OK; .status holds it (UHSDR_TIMEOUT: the device hand-off's
    failure contract, include/uhsdr.h uhsdr_rx_set_pipelined)."""

    def __init__(self, msg: str, status: int):
        super().__init__(msg)
        self.status = status


def check(status: int, what: str = "") -> None:
    if status != UHSDR_OK:
        err = load().uhsdr_last_error().decode()
        raise UhsdrError(f"{what} failed with status {status}: {err}", status)


def default_config(**overrides) -> RxConfig:
    cfg = RxConfig()
    load().uhsdr_rx_config_default(C.byref(cfg))
    for k, v in overrides.items():
        if k == "agc_tau_decay":
            for i, x in enumerate(v):
                cfg.agc_tau_decay[i] = x
        else:
            setattr(cfg, k, v)
    return cfg


def build_plan(cfg: RxConfig) -> RxPlan:
    plan = RxPlan()
    check(load().uhsdr_rx_plan_build(C.byref(cfg), C.byref(plan)), "uhsdr_rx_plan_build")
    return plan


def plan_supported(plan: RxPlan) -> bool:
    """uhsdr_rx_plan_supported: the device has a kernel instantiation for this plan's family."""
    return bool(load().uhsdr_rx_plan_supported(C.byref(plan)))


def plan_fma_ok(plan: RxPlan) -> bool:
    """uhsdr_rx_plan_fma_ok: uhsdr_rx_set_precision takes UHSDR_PRECISION_FMA for this plan."""
    return bool(load().uhsdr_rx_plan_fma_ok(C.byref(plan)))


# uhsdr_ref key=value names (tests/golden) -> RxConfig fields
REF_ARG_MAP = {
    "mode": "dmod_mode", "path": "filter_path", "iqmode": "iq_freq_mode", "iq_auto": "iq_auto_correction",
    "gain_i": "iq_gain_i", "gain_q": "iq_gain_q", "phase": "iq_phase_balance", "dsp": "dsp_active",
    "notch": "notch_frequency", "peak": "peak_frequency", "bass": "bass_gain", "treble": "treble_gain",
    "agc_mode": "agc_mode", "agc_thresh": "agc_thresh", "agc_slope": "agc_slope", "agc_hang": "agc_hang_enable",
    "sam_sb": "sam_sideband", "pll_fmax": "sam_pll_fmax", "zeta": "sam_zeta", "omegan": "sam_omega_n",
    "fade": "fade_leveler", "sql": "fm_sql_threshold", "fm5k": "fm_deviation_5k",
    "sidetone": "cw_sidetone_freq", "cwblock": "cw_decoder_blocksize", "cwthresh": "cw_decoder_thresh",
    "cwnc": "cw_decoder_noisecancel", "notch_mu": "notch_mu", "tonedet": "fm_tone_det",
    "beepfreq": "beep_frequency", "beeploud": "beep_loudness", "stereo": "stereo_enable",
    "board": "board", "spkr": "spkr_gain",
}
# uhsdr_ref run-time controls that are calls, not configuration (tests drive them through the ABI)
REF_RUNTIME_ARGS = {"beep", "uiperiod"}


def config_from_ref_args(args: dict) -> RxConfig:
    return default_config(**{REF_ARG_MAP[k]: v for k, v in args.items() if k not in REF_RUNTIME_ARGS})


# uhsdr_ref TX key=value names (tests/golden/tx_*.npz) -> TxConfig fields
TX_ARG_MAP = {
    "mode": "dmod_mode", "iqmode": "iq_freq_mode", "micmult": "mic_gain_mult", "boost": "mic_boost",
    "comp": "comp_level", "txfilter": "tx_filter", "txbass": "bass_gain", "txtreble": "treble_gain",
    "txpwr": "power_factor", "txgi": "gain_i", "txgq": "gain_q", "txphase": "phase_balance",
    "fm5k": "fm_deviation_5k", "subtone": "fm_subaudible_tone", "burstmode": "fm_tone_burst_mode",
    "txsrc": "audio_source",
}
FLAGS1_AM_TX_FILTER_DISABLE, FLAGS1_SSB_TX_FILTER_DISABLE = 0x08, 0x40   # hardware/uhsdr_board.h:513,516
TUNE_OFF, TUNE_SINGLE, TUNE_TWO = range(3)      # uhsdr_tx_set_tune


def default_tx_config(**overrides) -> TxConfig:
    cfg = TxConfig()
    load().uhsdr_tx_config_default(C.byref(cfg))
    for k, v in overrides.items():
        setattr(cfg, k, v)
    return cfg


def tx_config_from_ref_args(args: dict) -> TxConfig:
    kw = {TX_ARG_MAP[k]: v for k, v in args.items() if k in TX_ARG_MAP}
    # ts.flags1: the filter-disable flag of the configured mode (tx_processor.c:991, :1003)
    flag = FLAGS1_AM_TX_FILTER_DISABLE if args.get("mode", 0) == DEMOD_AM else FLAGS1_SSB_TX_FILTER_DISABLE
    kw["filter_disable"] = int(bool(int(args.get("flags1", 0)) & flag))
    return default_tx_config(**kw)


def build_tx_plan(cfg: TxConfig) -> TxPlan:
    plan = TxPlan()
    check(load().uhsdr_tx_plan_build(C.byref(cfg), C.byref(plan)), "uhsdr_tx_plan_build")
    return plan


# uhsdr_ref spectrum key=value names (tests/golden/spec_*.npz) -> SpectrumConfig fields
SPEC_ARG_MAP = {
    "spec": "fft_len", "specfilt": "spectrum_filter", "iq_auto": "iq_auto_correction",
    "gain_i": "iq_gain_i", "gain_q": "iq_gain_q", "phase": "iq_phase_balance",
    "mag": "magnify", "iqmode": "iq_freq_mode",
}


def default_spectrum_config(**overrides) -> SpectrumConfig:
    cfg = SpectrumConfig()
    load().uhsdr_spectrum_config_default(C.byref(cfg))
    for k, v in overrides.items():
        setattr(cfg, k, v)
    return cfg


def spectrum_config_from_ref_args(args: dict) -> SpectrumConfig:
    return default_spectrum_config(**{SPEC_ARG_MAP[k]: v for k, v in args.items() if k in SPEC_ARG_MAP})


def build_spectrum_plan(cfg: SpectrumConfig) -> SpectrumPlan:
    plan = SpectrumPlan()
    check(load().uhsdr_spectrum_plan_build(C.byref(cfg), C.byref(plan)), "uhsdr_spectrum_plan_build")
    return plan
