"""uhsdr_amd -- MI355X (gfx950) batched implementation of the UHSDR per-block RX DSP chain.

The product is ``uhsdr_amd/lib/libuhsdr_amd.so`` (C ABI: ``include/uhsdr.h``).  This
package is the thin host-side mirror used by tests and the benchmark.
"""
from ._abi import (RxConfig, RxPlan, build_plan, plan_supported, plan_fma_ok, config_from_ref_args, default_config, load,  # noqa: F401
                   DEMOD_USB, DEMOD_LSB, DEMOD_CW, DEMOD_AM, DEMOD_SAM, DEMOD_FM, DEMOD_DIGI,
                   DEMOD_SSBSTEREO, DEMOD_IQ, SAM_SIDEBAND_BOTH, SAM_SIDEBAND_LSB, SAM_SIDEBAND_USB,
                   SAM_SIDEBAND_STEREO, DSP_NOTCH_ENABLE, BOARD_OVI40, BOARD_MCHF,
                   UHSDR_OK, UHSDR_ARGUMENT_ERROR, UHSDR_UNSUPPORTED, UHSDR_TIMEOUT, UhsdrError,
                   PRECISION_EXACT, PRECISION_FMA,
                   SCHEDULE_AUTO, SCHEDULE_SPLIT_PIPE, SCHEDULE_SPLIT_FUSED, SCHEDULE_CHAIN, ADC_CLIP, ADC_HALF_CLIP, ADC_QUARTER_CLIP,
                   TWINPEAKS_SAMPLING, TWINPEAKS_DONE, TWINPEAKS_WAIT, TWINPEAKS_UNCORRECTABLE,
                   TWINPEAKS_CODEC_RESTART,
                   TUNE_OFF, TUNE_SINGLE, TUNE_TWO,
                   TxConfig, TxPlan, build_tx_plan, default_tx_config, tx_config_from_ref_args,
                   SpectrumConfig, SpectrumPlan, build_spectrum_plan, default_spectrum_config,
                   spectrum_config_from_ref_args)
from .rx import RxChain  # noqa: F401
from .tx import TxChain  # noqa: F401
from .spectrum import Spectrum  # noqa: F401
from .i2s import Transceiver  # noqa: F401
from .fir import FirBatch  # noqa: F401
