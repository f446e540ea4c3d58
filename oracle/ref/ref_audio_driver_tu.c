/*
 * ORACLE TEST INFRASTRUCTURE -- compiles the reference's own audio driver for the x86 host.
 *
 * The reference translation unit is included from where it lies under /root/reference
 * (drivers/audio/audio_driver.c); nothing is copied.  Two things are done around it:
 *  - USE_PENDSV_FOR_HIGHPRIO_TASKS is undefined: the ISR tail at audio_driver.c:3045-3048
 *    pokes the Cortex-M SCB->ICSR register, which is not memory on x86.
 *  - read-only accessors expose the driver's file-static filter instances so that the
 *    oracle can dump the exact coefficients / state lengths the firmware configured
 *    (used to pin the product's host setup layer bit-for-bit).
 */
#include "uhsdr_board_config.h"
#undef USE_PENDSV_FOR_HIGHPRIO_TASKS
#include "audio_driver.c"

const arm_biquad_casd_df1_inst_f32* oracle_ref_biquad1(void) { return &IIR_biquad_1[0]; }
const arm_biquad_casd_df1_inst_f32* oracle_ref_biquad2(void) { return &IIR_biquad_2[0]; }
const arm_iir_lattice_instance_f32* oracle_ref_prefilter(void) { return &IIR_PreFilter[0]; }
const arm_iir_lattice_instance_f32* oracle_ref_antialias(void) { return &IIR_AntiAlias[0]; }
const arm_fir_interpolate_instance_f32* oracle_ref_interpolate(void) { return &INTERPOLATE_RX[0]; }

/* layout fingerprint of TransceiverState as audio_driver.c sees it */
unsigned long oracle_driver_layout(void) { return (unsigned long)sizeof(TransceiverState) * 100000ul + (unsigned long)((char*)&ts.dsp.active - (char*)&ts); }
const arm_iir_lattice_instance_f32* oracle_ref_squelch(void) { return &IIR_Squelch_HPF; }

/* zoom spectrum producer (AudioDriver_SpectrumZoomProcessSamples, audio_driver.c:1860-1909):
   select the magnification the way the firmware's spectrum setup does (AudioDriver_Spectrum_Set,
   :1055-1086, which re-inits the zoom decimators), and read back its tables */
void oracle_ref_spec_magnify(int m) { sd.magnify = (uint8_t)m; AudioDriver_Spectrum_Set(); }
const float* oracle_ref_zoom_biquad(int m) { return mag_coeffs[m]; }
const arm_fir_decimate_instance_f32* oracle_ref_zoom_decim(void) { return &DECIMATE_ZOOM_FFT_I; }

/* LMS auto notch instance (AudioDriver_NotchFilter, audio_driver.c:1746-1763) */
float oracle_ref_notch_mu(void) { return lmsData.lms2Norm_instance.mu; }
