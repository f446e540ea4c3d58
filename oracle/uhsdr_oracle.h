/*
 * ORACLE -- TEST INFRASTRUCTURE ONLY.  Never linked into libuhsdr_amd.so; only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg load it (as the checker / the
 * CPU baseline, never as the thing measured or shipped).
 *
 * Clean-room CPU restatement of the reference RX chain (AudioDriver_RxProcessor,
 * drivers/audio/audio_driver.c:2603-2942, and the CMSIS-DSP V1.4.5 f32 kernels under it),
 * one state struct per channel, driven by the same uhsdr_rx_plan the device consumes.
 * Pinned bit-for-bit against the reference firmware compiled for x86 (oracle/ref/,
 * fixtures tests/golden/rx_*.npz) by tests/test_oracle.py.
 */
#ifndef UHSDR_ORACLE_H
#define UHSDR_ORACLE_H

#include <stdint.h>
#include <stddef.h>
#include "../include/uhsdr.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct uo_rx_state
{
    /* adb.iq_corr (audio_driver.h:125-135) */
    float teta1_old, teta2_old, teta3_old;
    /* FreqShift_Approx oscillator (freq_shift.c:22-27) */
    float osc_vi, osc_vq;
    /* CMSIS state arrays: history part only (the numTaps-1 / numStages values that
       survive a call, arm_fir_f32.c:565-580) */
    float hil_i[UHSDR_MAX_FIR_TAPS];
    float hil_q[UHSDR_MAX_FIR_TAPS];
    float dec_i[UHSDR_MAX_DEC_TAPS];
    float dec_q[UHSDR_MAX_DEC_TAPS];
    float pre[UHSDR_MAX_LATTICE + 1];
    float aa[UHSDR_MAX_LATTICE + 1];
    float bq1[16];
    float bq2[4];
    float interp[UHSDR_MAX_INTERP];
    /* agc_wdsp run-time variables (audio_agc.c:24-94) */
    float ring[UHSDR_AGC_RING];
    float abs_ring[UHSDR_AGC_RING];
    int32_t out_index, in_index, hang_counter, decay_type, state;
    float ring_max, volts, save_volts, fast_backaverage, hang_backaverage, wold;
    /* sam_data (audio_driver.c:1955-1976) and the fade leveler statics (:1911-1923) */
    float sam_phs, sam_omega2, sam_fil_out, sam_dsI, sam_dsQ;
    float sam_a[24], sam_b[24], sam_c[24], sam_d[24];
    float fade_dc27, fade_dc_insert;
    /* fm_data (audio_driver.c:1515-1531), ads.fm_conf squelch (:470-486), IIR_Squelch_HPF state */
    float fm_i_prev, fm_q_prev, fm_lpf_prev, fm_hpf_prev_a, fm_hpf_prev_b, fm_sql_avg;
    float fm_sq[UHSDR_MAX_LATTICE + 1];
    int32_t fm_squelched, fm_count;
    /* CW decoder front end: cw_goertzel.buf[1..2], CW_Decode_exe's statics old_siglevel /
       prevstate-free cw_state / change, CwDecode_RxProcessor's sample_counter (cw_decoder.c) */
    float cw_g1, cw_g2, cw_old;
    int32_t cw_state, cw_change, cw_count;
    /* outputs of the current call: energies of blocks completed, ads.CW_signal */
    float cw_energy_out;
    int32_t cw_blocks_out, cw_signal_out;
    /* lmsData (audio_driver.c:58-66) and AudioDriver_NotchFilter's statics lms2_inbuf/_outbuf */
    float notch_w[64], notch_st[64 + 16], notch_delay[128];
    float notch_energy, notch_x0;
    int32_t notch_in, notch_out;
    /* FM subaudible tone detector: ads.fm_conf.goertzel[3].buf[1..2], fm_data.subdet / tdet /
       gcount, ads.fm_conf.subaudible_tone_detected */
    float fm_g[3][2], fm_subdet;
    int32_t fm_tdet, fm_gcount, fm_tone_detected;
    /* OVI40 second audio channel (use_stereo): instances [1] of IIR_PreFilter, IIR_AntiAlias,
       IIR_biquad_1 / _2, INTERPOLATE_RX (audio_driver.c:78-161), agc ring[2*i+1], wold[1],
       the fade leveler's dc27[1] / dc_insert[1] (:1915-1916) */
    float pre1[UHSDR_MAX_LATTICE + 1], aa1[UHSDR_MAX_LATTICE + 1], bq1_1[16], bq2_1[4], interp1[UHSDR_MAX_INTERP];
    float ring1[UHSDR_AGC_RING], wold1, fade_dc27_1, fade_dc_insert_1;
    /* key beep: ts.beep_timing as calls left, ads.beep.acc */
    int32_t beep_left;
    uint32_t beep_acc;
    /* side outputs: ads.adc_clip / adc_half_clip / adc_quarter_clip as UHSDR_ADC_* bits, sticky
       until read (audio_driver.c:2660-2676); ts.twinpeaks_tested and AudioDriver_RxHandleTwinpeaks'
       statics twinpeaks_counter, codec_restarts, phase_IQ, phase_IQ_runs (:2173-2248) */
    int32_t clip;
    int32_t tp_state, tp_counter, tp_restarts, tp_runs;
    float tp_phase;
} uo_rx_state;

size_t uo_rx_state_size(void);
void uo_rx_state_init(const uhsdr_rx_plan* p, uo_rx_state* s);
/* one channel, n frames (n % 32 == 0): iq [n][2] int32 -> a1 [n] f32, dst [n][2] int32 */
int uo_rx_process(const uhsdr_rx_plan* p, uo_rx_state* s, const int32_t* iq, int n, float* a1, int32_t* dst);
/* the same with both output channels: a0 = adb.a_buffer[0] (the second channel in stereo, a copy
   of a_buffer[1] otherwise) */
int uo_rx_process2(const uhsdr_rx_plan* p, uo_rx_state* s, const int32_t* iq, int n, float* a1, float* a0,
                   int32_t* dst);
/* AudioManagement_KeyBeep on C channel states: the next `calls` calls get the beep tone */
void uo_rx_key_beep(uo_rx_state* states, int C, int calls);
/* the UI's side of the status outputs: read and clear the clip flags, read ts.twinpeaks_tested,
   and (rearm != 0) the codec restart acknowledgement CODEC_RESTART -> WAIT (ui_driver.c:7422-7426) */
void uo_rx_status(uo_rx_state* states, int C, int32_t* clip, int32_t* twinpeaks, int rearm);
/* C channels, channel-major buffers, `threads` POSIX threads (0 = 1) */
long long uo_rx_bench(const uhsdr_rx_plan* p, uo_rx_state* states, int C, const int32_t* iq, int pool, int n,
                      float* a1, int32_t* dst, int threads, int pin, double budget_s, double* elapsed);
int uo_rx_process_batch(const uhsdr_rx_plan* p, uo_rx_state* states, int C, const int32_t* iq, int n,
                        float* a1, int32_t* dst, int threads);
int uo_rx_process_batch2(const uhsdr_rx_plan* p, uo_rx_state* states, int C, const int32_t* iq, int n,
                         float* a1, float* a0, int32_t* dst, int threads);
/* the same, also recording the CW decoder front end: cw_signal [C][n/32] (ads.CW_signal after
   each call), cw_energy [C][bmax] (Goertzel energy of each block completed, in order) */
int uo_rx_process_batch_cw(const uhsdr_rx_plan* p, uo_rx_state* states, int C, const int32_t* iq, int n,
                           float* a1, int32_t* dst, uint8_t* cw_signal, float* cw_energy, int bmax, int threads);

/* transmit: TxProcessor_Run voice paths (SSB, AM, FM) and the USB I/Q source
   (drivers/audio/tx_processor.c:891-1078) */
typedef struct uo_tx_state
{
    float lat[UHSDR_MAX_LATTICE + 1];        /* IIR_TXFilter state */
    float bq[12];                             /* IIR_TX_biquad state */
    float alc_val;                            /* ads.alc_val (TxProcessor_Init: 1) */
    float delay[UHSDR_TX_DELAY];              /* audio_delay_buffer */
    int32_t delay_in;                         /* alc_delay_inbuf (function static) */
    float hil_i[UHSDR_TX_HILBERT_TAPS], hil_q[UHSDR_TX_HILBERT_TAPS];
    float osc_vi, osc_vq;
    /* TxProcessor_FM statics (tx_processor.c:536-537) and the sub-audible tone softdds */
    float fm_hpf_a, fm_hpf_b;
    uint32_t fm_accum, fm_sub_acc;
    /* softdds tones: ts.tune / tune_tone_mode with dbldds[0..1] (softdds.c:19), FM tone burst
       (ads.fm_conf.tone_burst_active, tone_burst_dds) */
    int32_t tune, burst;
    uint32_t tune_acc[2], burst_acc;
    float a0[32];                             /* adb.a_buffer[0] as the last voice call left it */
} uo_tx_state;

size_t uo_tx_state_size(void);
void uo_tx_state_init(const uhsdr_tx_plan* p, uo_tx_state* s);
int uo_tx_process_batch(const uhsdr_tx_plan* p, uo_tx_state* states, int C, const int32_t* audio, int n,
                        int32_t* iq, float* a0, int threads);
/* TUNE on / off (0 off, 1 single tone, 2 two-tone) and the FM tone burst, on C channel states */
void uo_tx_set_tune(uo_tx_state* states, int C, int tune);
void uo_tx_set_tone_burst(uo_tx_state* states, int C, int active);

/* spectrum display: producer ring + UiSpectrum_RedrawSpectrum states 0-3
   (audio_driver.c:1811-1851, ui_spectrum.c:1350-1446) */
typedef struct uo_spec_state
{
    float teta1_old, teta2_old, teta3_old;          /* the I/Q correction the ring sees */
    float frame[2 * UHSDR_SPECTRUM_MAX_LEN];        /* the [Q, I] ring, oldest first */
    float avg[UHSDR_SPECTRUM_MAX_LEN];              /* sd.FFT_AVGData */
    int32_t fill;                                   /* samples in frame[] */
    /* zoom producer (magnify > 0): IIR_biquad_Zoom_FFT_I/_Q states, DECIMATE_ZOOM_FFT_I/_Q
       histories, FreqShift_Approx oscillator */
    float zbq_i[16], zbq_q[16];
    float zdec_i[8], zdec_q[8];
    float osc_vi, osc_vq;
} uo_spec_state;

size_t uo_spec_state_size(void);
void uo_spec_state_init(const uhsdr_spectrum_plan* p, uo_spec_state* s);
/* arm_cfft_f32(S, x, 0, 1) restated: forward CFFT in place, natural order out */
void uo_cfft(const uhsdr_spectrum_plan* p, float* x);
/* batched arm_fir_f32: hist [C][T-1] carried in / out, x / y [C][n] */
void uo_fir_batch(const float* c, int T, float* hist, int C, const float* x, int n, float* y);
/* n samples of C channels; mag / avg [C][F][L] with F = frames completed (same for every
   channel); returns F, or a negative status */
int uo_spec_process_batch(const uhsdr_spectrum_plan* p, uo_spec_state* states, int C, const int32_t* iq, int n,
                          float* mag, float* avg, int threads);

#ifdef __cplusplus
}
#endif
#endif
