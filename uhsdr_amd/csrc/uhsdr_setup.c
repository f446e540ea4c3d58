/*
 * Host setup layer: builds a uhsdr_rx_plan exactly as the firmware configures its RX chain.
 *
 * Restates (behaviour, types and evaluation order -- this file must be compiled without
 * FP contraction, like the reference, so every rounding matches):
 *   AudioDriver_SetProcessingChain       drivers/audio/audio_driver.c:1093-1251
 *   AudioDriver_SetRxTxAudioProcessingAudioFilters  audio_driver.c:994-1050
 *   AudioDriver_CalcBandstop/Bandpass/HighShelf/LowShelf  audio_driver.c:831-964
 *   AudioFilter_SetRxHilbertAndDecimationFIR  drivers/audio/audio_filter.c:1134-1223
 *   AudioAgc_AgcWdsp_Init / AudioAgc_SetupAgcWdsp  drivers/audio/audio_agc.c:104-339
 *   FreqShift front end / FreqShift_Approx_Prepare  drivers/audio/freq_shift.c:40-52, 275-334
 *   AudioDriver_GetTranslateFreq          audio_driver.c:445-464
 *   RadioManagement_LSBActive             drivers/ui/radio_management.c:1665-1692
 * The reference's pow10f is glibc's exp10f (identical results; pow10f was only an alias).
 * Parity of every field is pinned against the reference build by tests/test_setup.py.
 */
#define _GNU_SOURCE
#include <math.h>
#include <string.h>
#include <stdarg.h>
#include <stdio.h>
#include "uhsdr_internal.h"

#define CMSIS_PI 3.14159265358979f          /* CMSIS/Include/arm_math.h:334 */
#define AUDIO_SAMPLE_RATE 48000             /* hardware/uhsdr_board_config.h:208 */
#define IQ_SAMPLE_RATE 48000
#define ADC_CLIP_WARN_THRESHOLD 4096        /* audio_driver.h:81 */
#define POST_AGC_GAIN_SCALING_DECIMATE_4 3.46                               /* audio_driver.h:362 */
#define POST_AGC_GAIN_SCALING_DECIMATE_2 (POST_AGC_GAIN_SCALING_DECIMATE_4 * 0.6) /* :364 */
#define LINE_OUT_SCALING_FACTOR 10          /* audio_driver.h:396 */
#define MCHF_SPEAKER_MAX_VOLUME 16          /* CODEC_SPEAKER_MAX_VOLUME with UI_BRD_MCHF, codec.h:26-27 */
#define FILTER_MODE_CW 0
#define FILTER_MODE_SSB 1
#define FILTER_MODE_AM 2
#define FILTER_MODE_FM 3

static __thread char g_err[256];
void uhsdr_set_error(const char* fmt, ...)
{
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
}
const char* uhsdr_last_error(void) { return g_err; }

static float fbits(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static void copy_bits(float* dst, const uint32_t* src, int n)
{
    for (int i = 0; i < n; i++) dst[i] = fbits(src[i]);
}

void uhsdr_rx_config_default(uhsdr_rx_config* c)
{
    memset(c, 0, sizeof *c);
    c->dmod_mode = UHSDR_DEMOD_USB;
    c->filter_path = 48;                       /* "3.8k LPF" SSB path */
    c->iq_freq_mode = UHSDR_IQ_CONV_M12KHZ;    /* FREQ_IQ_CONV_MODE_DEFAULT */
    c->iq_auto_correction = 0;
    c->iq_gain_i = 1.0f;
    c->iq_gain_q = 1.0f;
    c->iq_phase_balance = 0.0f;
    c->notch_frequency = 800;
    c->peak_frequency = 750;
    c->bass_gain = 2;
    c->treble_gain = 0;
    c->agc_mode = 2;
    c->agc_slope = 70;
    c->agc_thresh = 20;
    c->agc_hang_enable = 0;
    c->agc_hang_time = 500;                    /* AudioAgc_AgcWdsp_Init, audio_agc.c:116-121 */
    c->agc_hang_thresh = 45;
    c->agc_tau_decay[0] = 4000;
    c->agc_tau_decay[1] = 2000;
    c->agc_tau_decay[2] = 500;
    c->agc_tau_decay[3] = 250;
    c->agc_tau_decay[4] = 50;
    c->agc_tau_decay[5] = 1;
    c->agc_tau_hang_decay = 500;
    c->sam_sideband = UHSDR_SAM_SIDEBAND_BOTH;   /* ui_configuration.c:214-219 */
    c->sam_pll_fmax = 2500;
    c->sam_zeta = 65;
    c->sam_omega_n = 250;
    c->fade_leveler = 1;
    c->fm_sql_threshold = 12;                    /* FM_SQUELCH_DEFAULT, audio_driver.h:449 */
    c->fm_deviation_5k = 0;
    c->cw_sidetone_freq = 750;                   /* CW_SIDETONE_FREQ_DEFAULT, uhsdr_board.h:396 */
    c->cw_decoder_blocksize = 88;                /* CW_DECODER_BLOCKSIZE_DEFAULT, cw_decoder.h:13 */
    c->cw_decoder_thresh = 32000;                /* CW_DECODER_THRESH_DEFAULT, cw_decoder.h:17 */
    c->cw_decoder_noisecancel = 1;               /* CW_DECODER_FLAGS_DEFAULT bit 0, cw_decoder.h:19 */
    c->notch_mu = 10;                            /* DSP_NOTCH_MU_DEFAULT, audio_driver.h:495 */
    c->fm_tone_det = 0;                          /* FM_SUBAUDIBLE_TONE_OFF */
    c->beep_frequency = 1000;                    /* DEFAULT_BEEP_FREQUENCY, audio_driver.h:455 */
    c->beep_loudness = 10;                       /* DEFAULT_BEEP_LOUDNESS, audio_driver.h:460 */
    c->stereo_enable = 0;
    c->board = UHSDR_BOARD_OVI40;
    c->spkr_gain = 16;                           /* AUDIO_GAIN_DEFAULT, ui_configuration.h:74; ui_configuration.c:71 */
}

/* AudioFilter_CalcGoertzel, audio_filter.c:1281-1288 (Goertzel.a is an int) */
static void calc_goertzel(float* r, float* co, float* si, float freq, uint32_t size, float goertzel_coeff,
                          float samplerate)
{
    const int a = (0.5 + (freq * goertzel_coeff) * size / samplerate);
    const float b = (2 * CMSIS_PI * a) / size;
    *si = sinf(b);
    *co = cosf(b);
    *r = 2 * *co;
}

/* softdds_stepForSampleRate, softdds.c:26-32 (DDS_TBL_SIZE 1024, SOFTDDS_ACC_SHIFT 22) */
static uint32_t softdds_step(float freq, uint32_t samp_rate)
{
    uint64_t freq64_shifted = freq * 1024;
    freq64_shifted <<= 22;
    return (uint32_t)(freq64_shifted / samp_rate);
}

/* IIR_15k_hpf (drivers/audio/filters/iir_15k_hpf_fm_squelch.c): 6-stage lattice high-pass of
   the FM squelch noise detector, as raw binary32 bits (pinned against the reference build by
   tests/test_setup.py) */
static const uint32_t squelch_k_bits[6] = { 0x3dafcf3cu, 0x3e98cf2fu, 0x3f1b1449u, 0x3f362601u, 0x3f451263u, 0x3f49b75cu };
static const uint32_t squelch_v_bits[7] = { 0x3bb81eb1u, 0xbcd76eb4u, 0x3d8c17f0u, 0xbdea21a5u, 0x3def82c3u, 0xbd953da8u, 0x3ccfa56fu };

/* AudioFilter_GetFilterModeFromDemodMode, audio_filter.c:929-955 */
static int filter_mode_of(int dmod)
{
    switch (dmod)
    {
    case UHSDR_DEMOD_AM: return FILTER_MODE_AM;
    case UHSDR_DEMOD_FM: return FILTER_MODE_FM;
    case UHSDR_DEMOD_CW: return FILTER_MODE_CW;
    case UHSDR_DEMOD_SAM: return FILTER_MODE_AM;
    default: return FILTER_MODE_SSB;
    }
}

/* ---- biquad designers, audio_driver.c:821-964 (B0..A2 = 0..4) ---- */
static void scale_biquad(float c[5], const float scalingA, const float scalingB)
{
    c[3] = c[3] / scalingA;
    c[4] = c[4] / scalingA;
    c[0] = c[0] / scalingB;
    c[1] = c[1] / scalingB;
    c[2] = c[2] / scalingB;
}

static void calc_bandstop(float c[5], float f0, float FS)
{
    float Q = 10;
    float w0 = 2 * CMSIS_PI * f0 / FS;
    float alpha = sinf(w0) / (2 * Q);
    c[0] = 1;
    c[1] = -2 * cosf(w0);
    c[2] = 1;
    float scaling = 1 + alpha;
    c[3] = 2 * cosf(w0);
    c[4] = alpha - 1;
    scale_biquad(c, scaling, scaling);
}

static void calc_bandpass(float c[5], float f0, float FS)
{
    float Q = 4;
    float BW = 0.03;
    float w0 = 2 * CMSIS_PI * f0 / FS;
    float alpha = sinf(w0) * sinhf(log(2) / 2 * BW * w0 / sinf(w0));
    c[0] = Q * alpha;
    c[1] = 0;
    c[2] = -Q * alpha;
    float scaling = 1 + alpha;
    c[3] = 2 * cosf(w0);
    c[4] = alpha - 1;
    scale_biquad(c, scaling, scaling);
}

static void calc_highshelf(float c[5], float f0, float S, float gain, float FS)
{
    float w0 = 2 * CMSIS_PI * f0 / FS;
    float A = exp10f(gain / 40.0);
    float alpha = sinf(w0) / 2 * sqrtf((A + 1 / A) * (1 / S - 1) + 2);
    float cosw0 = cosf(w0);
    float twoAa = 2 * sqrtf(A) * alpha;
    c[0] = A * ((A + 1) + (A - 1) * cosw0 + twoAa);
    c[1] = -2 * A * ((A - 1) + (A + 1) * cosw0);
    c[2] = A * ((A + 1) + (A - 1) * cosw0 - twoAa);
    float scaling = (A + 1) - (A - 1) * cosw0 + twoAa;
    c[3] = -2 * ((A - 1) - (A + 1) * cosw0);
    c[4] = twoAa - (A + 1) + (A - 1) * cosw0;
    float DCgain = 1.0 * scaling;
    scale_biquad(c, scaling, DCgain);
}

static void calc_lowshelf(float c[5], float f0, float S, float gain, float FS)
{
    float w0 = 2 * CMSIS_PI * f0 / FS;
    float A = exp10f(gain / 40.0);
    float alpha = sinf(w0) / 2 * sqrtf((A + 1 / A) * (1 / S - 1) + 2);
    float cosw0 = cosf(w0);
    float twoAa = 2 * sqrtf(A) * alpha;
    c[0] = A * ((A + 1) - (A - 1) * cosw0 + twoAa);
    c[1] = 2 * A * ((A - 1) - (A + 1) * cosw0);
    c[2] = A * ((A + 1) - (A - 1) * cosw0 - twoAa);
    float scaling = (A + 1) + (A - 1) * cosw0 + twoAa;
    c[3] = 2 * ((A - 1) + (A + 1) * cosw0);
    c[4] = twoAa - (A + 1) - (A - 1) * cosw0;
    float DCgain = 1.0 * scaling;
    scale_biquad(c, scaling, DCgain);
}

static const float biquad_passthrough[5] = { 1, 0, 0, 0, 0 };

/* ---- AGC parameter math, audio_agc.c:126-339 (fresh channel: first setup after Init) ---- */
static void setup_agc(uhsdr_agc_plan* a, const uhsdr_rx_config* cfg, float sample_rate, int remove_dc)
{
    memset(a, 0, sizeof *a);
    a->remove_dc = remove_dc;
    a->mode = cfg->agc_mode;
    a->hang_enable = cfg->agc_hang_enable;
    a->sample_rate = sample_rate;
    /* one-time initialisation (:176-223) */
    a->ring_buffsize = UHSDR_AGC_RING;
    a->out_index0 = -1;
    float tau_attack = 0.001;
    int n_tau = 4;
    float max_input = (float)ADC_CLIP_WARN_THRESHOLD;
    float out_targ = (float)ADC_CLIP_WARN_THRESHOLD;
    float tau_fast_backaverage = 0.250;
    float tau_fast_decay = 0.005;
    a->pop_ratio = 5.0;
    float tau_hang_backmult = 0.500;

    a->var_gain = exp10f((float)cfg->agc_slope / 20.0 / 10.0);
    a->hangtime = (float)cfg->agc_hang_time / 1000.0;
    /* switch_mode == 1 on the first setup after AudioAgc_AgcWdsp_Init (:232-275) */
    switch (cfg->agc_mode)
    {
    case 5: break;
    case 1: a->hangtime = 2.000; break;
    case 2: a->hangtime = 1.000; break;
    case 3: a->hangtime = 0.250; break;
    case 4: a->hangtime = 0.100; break;
    case 0:
        a->hangtime = 3.000;
        tau_hang_backmult = 0.500;
        tau_fast_decay = 0.05;
        tau_fast_backaverage = 0.250;
        break;
    default: break;
    }
    float tau_hang_decay = (float)cfg->agc_tau_hang_decay / 1000.0;
    int dm = cfg->agc_mode;
    if (dm < 0) dm = 0;
    if (dm > 5) dm = 5;
    float tau_decay = (float)cfg->agc_tau_decay[dm] / 1000.0;
    a->max_gain = exp10f((float)cfg->agc_thresh / 20.0);
    a->fixed_gain = a->max_gain / 10.0;
    a->attack_buffsize = ceilf(sample_rate * n_tau * tau_attack);
    a->in_index0 = a->attack_buffsize + a->out_index0;
    a->in_index0 %= a->ring_buffsize;

    a->attack_mult = 1.0 - expf(-1.0 / (sample_rate * tau_attack));
    a->decay_mult = 1.0 - expf(-1.0 / (sample_rate * tau_decay));
    a->fast_decay_mult = 1.0 - expf(-1.0 / (sample_rate * tau_fast_decay));
    a->fast_backmult = 1.0 - expf(-1.0 / (sample_rate * tau_fast_backaverage));
    a->onemfast_backmult = 1.0 - a->fast_backmult;

    a->out_target = out_targ * (1.0 - expf(-(float)n_tau)) * 0.9999;
    a->min_volts = a->out_target / (a->var_gain * a->max_gain);
    a->inv_out_target = 1.0 / a->out_target;

    float tmpA = log10f(a->out_target / (max_input * a->var_gain * a->max_gain));
    if (tmpA == 0.0)
    {
        tmpA = 1e-16;
    }
    a->slope_constant = (a->out_target * (1.0 - 1.0 / a->var_gain)) / tmpA;
    a->inv_max_input = 1.0 / max_input;

    if (max_input > a->min_volts)
    {
        float convert = exp10f((float)cfg->agc_hang_thresh / 20.0);
        float tmpB = (convert - a->min_volts) / (max_input - a->min_volts);
        if (tmpB < 1e-8)
        {
            tmpB = 1e-8;
        }
        a->hang_thresh = 1.0 + 0.125 * log10f(tmpB);
    }
    else
    {
        a->hang_thresh = 1.0;
    }
    float tmpC = exp10f((a->hang_thresh - 1.0) / 0.125);
    a->hang_level = (max_input * tmpC + (a->out_target / (a->var_gain * a->max_gain)) * (1.0 - tmpC)) * 0.637;
    a->hang_backmult = 1.0 - expf(-1.0 / (sample_rate * tau_hang_backmult));
    a->onemhang_backmult = 1.0 - a->hang_backmult;
    a->hang_decay_mult = 1.0 - expf(-1.0 / (sample_rate * tau_hang_decay));
    a->hang_counter_init = (int)(a->hangtime * a->sample_rate);   /* audio_agc.c:469 */
}

/* FreqShift parameters for ts.iq_freq_mode: AudioDriver_GetTranslateFreq (audio_driver.c:445-464),
   FreqShift's kind selection (freq_shift.c:294-319) and FreqShift_Approx_Prepare (:40-52) */
static void shift_plan(int32_t iq_freq_mode, int32_t* hz, int32_t* kind, int32_t* up, float* oc, float* os)
{
    switch (iq_freq_mode)
    {
    case UHSDR_IQ_CONV_P6KHZ: *hz = 6000; break;
    case UHSDR_IQ_CONV_M6KHZ: *hz = -6000; break;
    case UHSDR_IQ_CONV_P12KHZ: *hz = 12000; break;
    case UHSDR_IQ_CONV_M12KHZ: *hz = -12000; break;
    default: *hz = 0; break;
    }
    if (*hz != 0)
    {
        const int32_t conv = *hz < 0 ? -*hz : *hz;
        const float rate = conv / (float)IQ_SAMPLE_RATE;       /* IQ_SAMPLE_RATE_F */
        *kind = (rate == 0.25) ? 1 : 2;                /* freq_shift.c:294-319 */
        const double r = (2 * M_PI * conv) / (float)IQ_SAMPLE_RATE;
        *oc = cos(r);
        *os = sin(r);
        *up = !(*hz > 0);                 /* dir = shift > 0 => DOWN */
    }
}

uhsdr_status uhsdr_rx_plan_build(const uhsdr_rx_config* cfg, uhsdr_rx_plan* p)
{
    if (!cfg || !p) { uhsdr_set_error("null argument"); return UHSDR_ARGUMENT_ERROR; }
    if (cfg->filter_path <= 0 || cfg->filter_path >= UHSDR_FILTER_PATH_NUM)
    {
        uhsdr_set_error("filter_path %d out of range 1..%d", cfg->filter_path, UHSDR_FILTER_PATH_NUM - 1);
        return UHSDR_ARGUMENT_ERROR;
    }
    if (cfg->dmod_mode < UHSDR_DEMOD_USB || cfg->dmod_mode > UHSDR_DEMOD_IQ)
    {
        uhsdr_set_error("dmod_mode %d unknown", cfg->dmod_mode);
        return UHSDR_ARGUMENT_ERROR;
    }
    const uhsdr_filter_path_desc* f = &uhsdr_filter_paths[cfg->filter_path];
    if ((f->mode & (1u << filter_mode_of(cfg->dmod_mode))) == 0)
    {
        /* the firmware only ever selects applicable paths (audio_filter.c:975-1011) */
        uhsdr_set_error("filter_path %d not applicable to dmod_mode %d", cfg->filter_path, cfg->dmod_mode);
        return UHSDR_ARGUMENT_ERROR;
    }
    memset(p, 0, sizeof *p);
    const int mode = cfg->dmod_mode;
    p->dmod_mode = mode;
    p->filter_path = cfg->filter_path;
    switch (mode)
    {
    case UHSDR_DEMOD_LSB: p->lsb = 1; break;
    case UHSDR_DEMOD_CW: p->lsb = cfg->cw_lsb != 0; break;
    case UHSDR_DEMOD_DIGI: p->lsb = cfg->digi_lsb != 0; break;
    default: p->lsb = 0; break;
    }
    p->decimation_rate = f->sample_rate_dec;
    p->decimated_freq = IQ_SAMPLE_RATE / f->sample_rate_dec;

    /* input stage */
    p->iq_auto_correction = cfg->iq_auto_correction != 0;
    p->iq_gain_i = cfg->iq_gain_i;
    p->iq_gain_q = cfg->iq_gain_q;
    p->iq_phase_balance = cfg->iq_phase_balance;
    shift_plan(cfg->iq_freq_mode, &p->freq_shift_hz, &p->shift_kind, &p->shift_up, &p->osc_cos, &p->osc_sin);

    /* Hilbert / decimation FIRs, audio_filter.c:1134-1223 and audio_driver.c:2718-2720 */
    const int is_am = (mode == UHSDR_DEMOD_AM || mode == UHSDR_DEMOD_SAM);
    p->use_decimated_iq = ((f->fir_i == uhsdr_filter_paths[4].fir_i) && mode != UHSDR_DEMOD_FM) || is_am;
    p->hilbert_taps = is_am ? 0 : f->fir_taps;
    copy_bits(p->hilbert_i, f->fir_i, f->fir_taps);
    copy_bits(p->hilbert_q, f->fir_q, f->fir_taps);
    if (is_am)
    {
        p->dec_taps = f->fir_taps;           /* AM/SAM: the path's I / Q tables as decimators */
        copy_bits(p->dec, f->fir_i, f->fir_taps);
        copy_bits(p->dec_q, f->fir_q, f->fir_taps);
    }
    else if (f->dec_taps)
    {
        p->dec_taps = f->dec_taps;
        copy_bits(p->dec, f->dec, f->dec_taps);
    }
    /* IIR lattice pre-filter and anti-alias filter, audio_driver.c:1112-1151 */
    p->pre_stages = f->pre_stages;
    copy_bits(p->pre_k, f->pre_k, f->pre_stages);
    if (f->pre_stages) copy_bits(p->pre_v, f->pre_v, f->pre_stages + 1);
    p->aa_stages = f->aa_stages;
    copy_bits(p->aa_k, f->aa_k, f->aa_stages);
    if (f->aa_stages) copy_bits(p->aa_v, f->aa_v, f->aa_stages + 1);
    /* interpolator, audio_driver.c:1209-1224: the descriptor's phaseLength is passed as numTaps */
    if (f->interp_taps)
    {
        p->interp_L = p->decimation_rate;
        if (f->interp_taps % p->interp_L) { uhsdr_set_error("interpolator length"); return UHSDR_LENGTH_ERROR; }
        p->interp_phase = f->interp_taps / p->interp_L;
        copy_bits(p->interp, f->interp, f->interp_taps);
    }

    /* biquads, audio_driver.c:994-1050 */
    const float FSdec = AUDIO_SAMPLE_RATE / (f->sample_rate_dec != 0 ? f->sample_rate_dec : 1);
    float c[5];
    if (cfg->dsp_active & UHSDR_DSP_MNOTCH_ENABLE) { calc_bandstop(c, cfg->notch_frequency, FSdec); memcpy(p->biquad1 + 0, c, sizeof c); }
    else memcpy(p->biquad1 + 0, biquad_passthrough, sizeof c);
    memcpy(p->biquad1 + 15, biquad_passthrough, sizeof c);
    if (cfg->dsp_active & UHSDR_DSP_MPEAK_ENABLE) { calc_bandpass(c, cfg->peak_frequency, FSdec); memcpy(p->biquad1 + 5, c, sizeof c); }
    else memcpy(p->biquad1 + 5, biquad_passthrough, sizeof c);
    calc_lowshelf(c, 250, 0.7, cfg->bass_gain, FSdec);
    memcpy(p->biquad1 + 10, c, sizeof c);
    calc_highshelf(c, 3500, 0.9, cfg->treble_gain, AUDIO_SAMPLE_RATE);
    memcpy(p->biquad2, c, sizeof c);

    /* post-AGC scaling, audio_driver.c:2513-2524 */
    const float post_agc_gain_scaling = (f->sample_rate_dec == 4) ? POST_AGC_GAIN_SCALING_DECIMATE_4
                                                                  : POST_AGC_GAIN_SCALING_DECIMATE_2;
    p->post_agc_scale = post_agc_gain_scaling * (is_am ? 0.5 : 0.333);
    /* output stage of the board, audio_driver.c:2856-2885 */
    if (cfg->board != UHSDR_BOARD_OVI40 && cfg->board != UHSDR_BOARD_MCHF)
    { uhsdr_set_error("board %d: UHSDR_BOARD_OVI40 or UHSDR_BOARD_MCHF", cfg->board); return UHSDR_ARGUMENT_ERROR; }
    p->single_channel = cfg->board == UHSDR_BOARD_MCHF;
    if (p->single_channel)
    {
        /* no USE_TWO_CHANNEL_AUDIO: use_stereo is false (:2620), the two-channel demodulators are
           not compiled (:2769-2778) and SAM_SIDEBAND_STEREO does not exist (audio_driver.h:186-188) */
        if (mode == UHSDR_DEMOD_SSBSTEREO || mode == UHSDR_DEMOD_IQ)
        { uhsdr_set_error("dmod_mode %d needs two-channel audio (OVI40)", mode); return UHSDR_UNSUPPORTED; }
        if (mode == UHSDR_DEMOD_SAM && cfg->sam_sideband == UHSDR_SAM_SIDEBAND_STEREO)
        { uhsdr_set_error("SAM stereo sideband needs two-channel audio (OVI40)"); return UHSDR_ARGUMENT_ERROR; }
        /* UiDriver's volume update (ui_driver.c:3083-3092) feeds the software gain the driver
           applies above the codec's range (audio_driver.c:2880-2885, CODEC_SPEAKER_MAX_VOLUME 16
           for UI_BRD_MCHF, codec.h:26-27) */
        float active_value = 1;
        if (cfg->spkr_gain > MCHF_SPEAKER_MAX_VOLUME) active_value = (((float)cfg->spkr_gain) / 2.5) - 5.35;
        p->line_out_scale = 1;
        p->line_out0_scale = LINE_OUT_SCALING_FACTOR;
        p->spkr_scale = active_value;
    }
    else
    {
        p->line_out_scale = LINE_OUT_SCALING_FACTOR;
        p->line_out0_scale = LINE_OUT_SCALING_FACTOR;
        p->spkr_scale = 1;
    }

    setup_agc(&p->agc, cfg, (float)p->decimated_freq, is_am);

    /* AudioDriver_SetSamPllParameters, audio_driver.c:709-745 (PI = 3.14159265358979f) */
    if (cfg->sam_sideband < UHSDR_SAM_SIDEBAND_BOTH || cfg->sam_sideband > UHSDR_SAM_SIDEBAND_STEREO)
    { uhsdr_set_error("sam_sideband %d outside 0..3", cfg->sam_sideband); return UHSDR_ARGUMENT_ERROR; }
    p->sam_sideband = cfg->sam_sideband;
    /* OVI40 two-channel audio: use_stereo (audio_driver.c:2618) */
    {
        const int two = mode == UHSDR_DEMOD_IQ || mode == UHSDR_DEMOD_SSBSTEREO ||
                        (mode == UHSDR_DEMOD_SAM && cfg->sam_sideband == UHSDR_SAM_SIDEBAND_STEREO);
        p->stereo = (two && cfg->stereo_enable) ? (mode == UHSDR_DEMOD_SSBSTEREO ? 1 : mode == UHSDR_DEMOD_IQ ? 2 : 3) : 0;
    }
    p->fade_leveler = cfg->fade_leveler != 0;
    /* the menu's ranges (ui_configuration.c:214-216); within them the PLL's per-sample phase
       step |g1 * phzerror + omega2| <= g1 * pi + 2 pi fmax / 12000 < 4.7 stays below 2 pi, so the
       phase wrap (audio_driver.c:2143-2146) takes at most one iteration each way and the device
       demodulator (DemodStage::step) evaluates it as two selects */
    if (mode == UHSDR_DEMOD_SAM && (cfg->sam_pll_fmax < 50 || cfg->sam_pll_fmax > 8000 || cfg->sam_zeta < 1 || cfg->sam_zeta > 100 ||
        cfg->sam_omega_n < 15 || cfg->sam_omega_n > 1000))
    {
        uhsdr_set_error("SAM PLL parameters (fmax %d, zeta %d, omegaN %d) outside 50..8000, 1..100, 15..1000",
                        cfg->sam_pll_fmax, cfg->sam_zeta, cfg->sam_omega_n);
        return UHSDR_ARGUMENT_ERROR;
    }
    {
        const float decimSampleRate = p->decimated_freq;
        const float pll_fmax = cfg->sam_pll_fmax;
        const float omegaN = cfg->sam_omega_n;
        const float zeta = (float)cfg->sam_zeta / 100.0;
        p->sam_omega_min = -(2.0 * CMSIS_PI * pll_fmax / decimSampleRate);
        p->sam_omega_max = (2.0 * CMSIS_PI * pll_fmax / decimSampleRate);
        p->sam_g1 = (1.0 - expf(-2.0 * omegaN * zeta / decimSampleRate));
        p->sam_g2 = (-p->sam_g1 + 2.0 * (1 - expf(-omegaN * zeta / decimSampleRate)
                     * cosf(omegaN / decimSampleRate * sqrtf(1.0 - zeta * zeta))));
        const float tauR = 0.02;
        const float tauI = 1.4;
        p->fade_mtauR = (expf(-1 / (decimSampleRate * tauR)));
        p->fade_onem_mtauR = (1.0 - p->fade_mtauR);
        p->fade_mtauI = (expf(-1 / (decimSampleRate * tauI)));
        p->fade_onem_mtauI = (1.0 - p->fade_mtauI);
    }
    /* FM: AudioDriver_DemodFM (audio_driver.c:1544-1737), FM_RX_SCALING_* (:1494-1495) */
    p->fm_scale = cfg->fm_deviation_5k ? 5000 : 10000;
    p->fm_sql_threshold = cfg->fm_sql_threshold;
    p->sq_stages = 6;
    copy_bits(p->sq_k, squelch_k_bits, 6);
    copy_bits(p->sq_v, squelch_v_bits, 7);
    /* CW decoder front end: CwDecode_RxProcessor runs on a_buffer[0] in CW, AM and SAM when the
       decimated rate is 12 ksps (audio_driver.c:2536-2557); CwDecode_Filter_Set (cw_decoder.c:
       69-74, called from SetProcessingChain :1158) -> AudioFilter_CalcGoertzel (audio_filter.c:
       1281-1288) with coefficient 1.0 and cw_decoder_config.sampling_freq = 12000.0 */
    if (cfg->cw_decoder_blocksize < 1 || cfg->cw_decoder_blocksize > 128)
    { uhsdr_set_error("cw_decoder_blocksize %d outside 1..128", cfg->cw_decoder_blocksize); return UHSDR_ARGUMENT_ERROR; }
    p->cw_enabled = (p->dmod_mode == UHSDR_DEMOD_CW || p->dmod_mode == UHSDR_DEMOD_AM || p->dmod_mode == UHSDR_DEMOD_SAM)
                    && p->decimated_freq == 12000;
    p->cw_blocksize = cfg->cw_decoder_blocksize;
    p->cw_noisecancel = cfg->cw_decoder_noisecancel != 0;
    p->cw_thresh = (float)(uint32_t)cfg->cw_decoder_thresh;
    {
        const float freq = (float)(uint32_t)cfg->cw_sidetone_freq;
        const float goertzel_coeff = 1.0f;
        const uint32_t size = (uint32_t)cfg->cw_decoder_blocksize;
        const float samplerate = 12000.0f;
        const int ga = (0.5 + (freq * goertzel_coeff) * size / samplerate);
        const float gb = (2 * CMSIS_PI * ga) / size;
        p->cw_sin = sinf(gb);
        p->cw_cos = cosf(gb);
        p->cw_r = 2 * p->cw_cos;
    }
    /* LMS auto notch: AudioDriver_SetProcessingChain (audio_driver.c:1166-1186) and the call
       condition of RxProcessor_DemodAudioPostprocessing (:2441-2443): not in CW, not in SAM at
       24 ksps, not in FM (FM skips the post-processing, :2792-2830) */
    if (cfg->notch_mu < 0 || cfg->notch_mu > 40)
    { uhsdr_set_error("notch_mu %d outside 0..40 (DSP_NOTCH_MU_MAX)", cfg->notch_mu); return UHSDR_ARGUMENT_ERROR; }
    p->notch_enabled = (cfg->dsp_active & UHSDR_DSP_NOTCH_ENABLE) && mode != UHSDR_DEMOD_CW && mode != UHSDR_DEMOD_FM
                       && !(mode == UHSDR_DEMOD_SAM && p->decimated_freq == 24000);
    p->notch_taps = 64;                          /* DSP_NOTCH_NUMTAPS_DEFAULT (= MIN = MAX), audio_driver.h:486-488 */
    p->notch_delay_len = 128;                    /* DSP_NOTCH_DELAYBUF_DEFAULT (= MIN = MAX), :490-492 */
    p->notch_mu = log10f(((cfg->notch_mu + 1.0) / 1500.0) + 1.0);
    /* FM subaudible tone detector: AudioManagement_CalcSubaudibleDetFreq (audio_management.c:313-326),
       window FM_SUBAUDIBLE_GOERTZEL_WINDOW * AUDIO_BLOCK_SIZE = 400 * 32 samples */
    if (cfg->fm_tone_det < 0 || cfg->fm_tone_det >= uhsdr_fm_subaudible_count)
    { uhsdr_set_error("fm_tone_det %d outside 0..%d", cfg->fm_tone_det, uhsdr_fm_subaudible_count - 1); return UHSDR_ARGUMENT_ERROR; }
    {
        float freq;
        memcpy(&freq, &uhsdr_fm_subaudible[cfg->fm_tone_det], 4);
        p->tone_det_enabled = freq != 0;
        if (freq > 0)
        {
            const uint32_t size = 400 * 32;
            calc_goertzel(&p->tone_r[0], &p->tone_cos[0], &p->tone_sin[0], freq, size, 1.04, IQ_SAMPLE_RATE);  /* FM_HIGH */
            calc_goertzel(&p->tone_r[1], &p->tone_cos[1], &p->tone_sin[1], freq, size, 0.95, IQ_SAMPLE_RATE);  /* FM_LOW */
            calc_goertzel(&p->tone_r[2], &p->tone_cos[2], &p->tone_sin[2], freq, size, 1.0, IQ_SAMPLE_RATE);   /* FM_CTR */
        }
    }
    /* key beep: AudioManagement_KeyBeepPrepare (audio_management.c:354-363), ts.samp_rate 48000 */
    p->beep_step = softdds_step((float)cfg->beep_frequency, 48000);
    {
        float calc = (float)(cfg->beep_loudness - 1);
        calc /= 2;
        calc *= calc;
        calc += 3;
        p->beep_scale = calc / 400;
    }
    memcpy(p->dds_table, uhsdr_dds_table, sizeof p->dds_table);
    return UHSDR_OK;
}

/* uhsdr_rx_plan_supported() lives with the device kernels (uhsdr_rx.hip): it answers
   whether a kernel variant exists for the plan's filter-path family. */
int uhsdr_rx_mode_supported(const uhsdr_rx_plan* p)
{
    /* device chain: SSB / CW / DIGI (I +- Q), AM, SAM, FM (FM needs the I/Q translation: without
       it AudioDriver_DemodFM leaves a_buffer[0] untouched, audio_driver.c:1548) */
    if (!p) return 0;
    return p->dmod_mode != UHSDR_DEMOD_FM || p->freq_shift_hz != 0;
}

const char* uhsdr_version(void) { return "uhsdr_amd 0.1 (gfx950)"; }
int32_t uhsdr_sizeof_config(void) { return (int32_t)sizeof(uhsdr_rx_config); }
int32_t uhsdr_abi_version(void) { return UHSDR_ABI_VERSION; }
int32_t uhsdr_sizeof_plan(void) { return (int32_t)sizeof(uhsdr_rx_plan); }

/* ================================ transmit ================================ */

/* defaults: drivers/ui/ui_configuration.c:91,140-141,161,211-213; codec.c:321 (mic gain 15) */
void uhsdr_tx_config_default(uhsdr_tx_config* c)
{
    memset(c, 0, sizeof *c);
    c->dmod_mode = UHSDR_DEMOD_USB;
    c->iq_freq_mode = UHSDR_IQ_CONV_M12KHZ;
    c->audio_source = UHSDR_TX_AUDIO_MIC;
    c->mic_gain_mult = 15;                       /* MIC_GAIN_DEFAULT, hardware/uhsdr_board.h:142 */
    c->mic_boost = 0;
    c->comp_level = 2;                           /* TX_AUDIO_COMPRESSION_DEFAULT, audio_driver.h:467 */
    c->alc_decay = 10;                           /* ALC_DECAY_DEFAULT, audio_driver.h:410 */
    c->alc_postfilt_gain = 1;                    /* ALC_POSTFILT_GAIN_DEFAULT, audio_driver.h:415 */
    c->tx_filter = 0;
    c->bass_gain = 4;
    c->treble_gain = 4;
    c->filter_disable = 0;
    c->power_factor = 0.5f;
    c->gain_i = 1.0f;
    c->gain_q = 1.0f;
    c->phase_balance = 0.0f;
}

/* AudioManagement_CalcTxCompLevel preset table, audio_management.c:250-265 */
static const uint8_t alc_params[13][2] = { { 1, 15 }, { 2, 12 }, { 4, 10 }, { 6, 9 }, { 7, 8 }, { 8, 7 }, { 10, 6 },
                                           { 12, 5 }, { 15, 4 }, { 17, 3 }, { 20, 2 }, { 25, 1 }, { 25, 0 } };

/* TxProcessor_Init / TxProcessor_Set / AudioFilter_SetTxHilbertFIR / AudioManagement_CalcTxCompLevel
   (tx_processor.c:72-144, audio_filter.c:1231-1256, audio_management.c:15-19,267-290) and the
   constant parts of TxProcessor_AudioBufferFill / _VoiceCompressor / _IqFinalProcessing */
uhsdr_status uhsdr_tx_plan_build(const uhsdr_tx_config* cfg, uhsdr_tx_plan* p)
{
    if (!cfg || !p) { uhsdr_set_error("null argument"); return UHSDR_ARGUMENT_ERROR; }
    const int fm = cfg->dmod_mode == UHSDR_DEMOD_FM, am = cfg->dmod_mode == UHSDR_DEMOD_AM;
    if (cfg->dmod_mode != UHSDR_DEMOD_USB && cfg->dmod_mode != UHSDR_DEMOD_LSB && !fm && !am)
    {
        uhsdr_set_error("transmit mode %d: SSB (USB/LSB), AM and FM voice are implemented", cfg->dmod_mode);
        return UHSDR_UNSUPPORTED;
    }
    if ((fm || am) && cfg->iq_freq_mode == UHSDR_IQ_CONV_OFF && cfg->audio_source != UHSDR_TX_AUDIO_DIGIQ)
    {
        /* "No AM / FM possible unless in frequency translate mode" (tx_processor.c:1000-1011).
           With the USB I/Q source the passthrough branch (:950-961) comes first and transmits
           the I/Q as is; only TUNE then reaches the AM / FM branch, which produces no signal
           (uhsdr_tx_process writes zero I/Q, the reference's signal_active == false) */
        uhsdr_set_error("AM / FM transmit needs the I/Q frequency translation");
        return UHSDR_UNSUPPORTED;
    }
    if (cfg->fm_tone_burst_mode < 0 || cfg->fm_tone_burst_mode > 2)   /* FM_TONE_BURST_MAX, audio_driver.h:440 */
    {
        uhsdr_set_error("fm_tone_burst_mode %d outside 0..2", cfg->fm_tone_burst_mode);
        return UHSDR_ARGUMENT_ERROR;
    }
    if (fm && (cfg->fm_subaudible_tone < 0 || cfg->fm_subaudible_tone >= uhsdr_fm_subaudible_count))
    {
        uhsdr_set_error("fm_subaudible_tone %d outside 0..%d", cfg->fm_subaudible_tone, uhsdr_fm_subaudible_count - 1);
        return UHSDR_ARGUMENT_ERROR;
    }
    if (cfg->audio_source < UHSDR_TX_AUDIO_MIC || cfg->audio_source > UHSDR_TX_AUDIO_DIGIQ)
    {
        uhsdr_set_error("transmit audio source %d: mic, line in L / R, USB audio, USB I/Q", cfg->audio_source);
        return UHSDR_ARGUMENT_ERROR;
    }
    memset(p, 0, sizeof *p);
    p->dmod_mode = cfg->dmod_mode;
    p->lsb = cfg->dmod_mode == UHSDR_DEMOD_LSB;
    p->audio_source = cfg->audio_source;

    /* TxProcessor_AudioBufferFill gain (tx_processor.c:354-381) */
    float gain_calc;
    if (cfg->audio_source == UHSDR_TX_AUDIO_MIC)
    {
        gain_calc = (uint32_t)cfg->mic_gain_mult;
        gain_calc /= 2;                                      /* MIC_GAIN_RESCALE, audio_driver.h:399 */
        if (cfg->mic_boost > 0) gain_calc += 25.1;
    }
    else if (cfg->audio_source == UHSDR_TX_AUDIO_LINEIN_L || cfg->audio_source == UHSDR_TX_AUDIO_LINEIN_R)
    {
        gain_calc = 20;                                      /* LINE_IN_GAIN_RESCALE, audio_driver.h:398 */
    }
    else
    {
        gain_calc = 1;                                       /* TX_AUDIO_DIG and the default (:374-381) */
    }
    gain_calc *= 0.0000152587890625;                         /* AUDIO_BIT_SCALE_DOWN, audio_driver.h:605 */
    p->in_gain = gain_calc;
    p->apply_in_gain = gain_calc != 1.0;

    /* TxProcessor_FilterAudio: lattice band-pass unless disabled (FM always filters,
       tx_processor.c:1012), biquads for codec sources; FM uses IIR_TX_2k7_FM (:104-107) */
    p->run_lattice = fm || !cfg->filter_disable;           /* FLAGS1_SSB / _AM_TX_FILTER_DISABLE (:991, :1003) */
    p->run_biquad = cfg->audio_source != UHSDR_TX_AUDIO_DIG;   /* do_bass_treble (:445) */
    const int sel = fm ? 3 : cfg->tx_filter == 2 ? 1 : cfg->tx_filter == 3 ? 2 : 0;   /* TENOR, BASS, default SOPRANO */
    const uhsdr_lattice_desc* l = &uhsdr_tx_lattices[sel];
    p->lat_stages = l->stages;
    copy_bits(p->lat_k, l->k, l->stages);
    copy_bits(p->lat_v, l->v, l->stages + 1);
    float c[5];
    calc_highshelf(c, 1700, 0.9, cfg->treble_gain, AUDIO_SAMPLE_RATE);
    memcpy(p->biquad + 0, c, sizeof c);
    calc_lowshelf(c, 300, 0.7, cfg->bass_gain, AUDIO_SAMPLE_RATE);
    memcpy(p->biquad + 5, c, sizeof c);
    memcpy(p->biquad + 10, biquad_passthrough, sizeof c);

    /* voice compressor */
    p->comp_on = cfg->comp_level > -1;
    uint32_t postfilt, decay_var;
    if (-1 < cfg->comp_level && cfg->comp_level < 13) { postfilt = alc_params[cfg->comp_level][0]; decay_var = alc_params[cfg->comp_level][1]; }
    else if (cfg->comp_level == 13) { postfilt = cfg->alc_postfilt_gain; decay_var = cfg->alc_decay; }
    else { postfilt = 4; decay_var = 10; }
    p->postfilt_gain = ((float)postfilt) / 2.0 + 0.5;
    p->alc_decay = exp10f(-((((float)decay_var) + 35.0) / 10.0));
    p->alc_gain_scaling = fm ? 0.95 : am ? 0.23 : 1.00;      /* FM_ALC_GAIN_CORRECTION (tx_processor.c:521) /
                                                                AM_ALC_GAIN_CORRECTION (audio_driver.h:428) /
                                                                SSB_ALC_GAIN_CORRECTION (audio_driver.h:417) */
    p->am = am;

    /* TX Hilbert pair, swapped for LSB (tx_processor.c:477-478) */
    const int T = uhsdr_tx_hilbert_taps;
    copy_bits(p->hilbert_i, p->lsb ? uhsdr_tx_hilbert_q : uhsdr_tx_hilbert_i, T);
    copy_bits(p->hilbert_q, p->lsb ? uhsdr_tx_hilbert_i : uhsdr_tx_hilbert_q, T);

    /* FreqShift by AudioDriver_GetTranslateFreq (tx_processor.c:484-487) */
    switch (cfg->iq_freq_mode)
    {
    case UHSDR_IQ_CONV_P6KHZ: p->freq_shift_hz = 6000; break;
    case UHSDR_IQ_CONV_M6KHZ: p->freq_shift_hz = -6000; break;
    case UHSDR_IQ_CONV_P12KHZ: p->freq_shift_hz = 12000; break;
    case UHSDR_IQ_CONV_M12KHZ: p->freq_shift_hz = -12000; break;
    default: p->freq_shift_hz = 0; break;
    }
    if (p->freq_shift_hz != 0)
    {
        const int32_t conv = p->freq_shift_hz < 0 ? -p->freq_shift_hz : p->freq_shift_hz;
        const float rate = conv / (float)IQ_SAMPLE_RATE;
        p->shift_kind = (rate == 0.25) ? 1 : 2;
        const double r = (2 * M_PI * conv) / (float)IQ_SAMPLE_RATE;
        p->osc_cos = cos(r);
        p->osc_sin = sin(r);
        p->shift_up = !(p->freq_shift_hz > 0);
    }

    /* TxProcessor_IqFinalProcessing (tx_processor.c:282-330) with iq_gain_comp = SSB_GAIN_COMP
       or FM_MOD_AMPLITUDE_SCALING (:500, :1014) */
    float scaling = fm ? 0.875 : 1.133;                      /* SSB_GAIN_COMP = AM_GAIN_COMP, audio_driver.h:419-421 */
    scaling *= (1 << 16);                                    /* IQ_BIT_SCALE_UP */
    p->final_i_gain = cfg->power_factor * cfg->gain_i * scaling;
    p->final_q_gain = cfg->power_factor * cfg->gain_q * scaling;
    /* TX_AUDIO_DIGIQ (:950-961): the USB I/Q goes straight to the final stage with iq_gain_comp 1.0 */
    p->digiq = cfg->audio_source == UHSDR_TX_AUDIO_DIGIQ;
    float scaling1 = 1.0;
    scaling1 *= (1 << 16);
    p->digiq_i_gain = cfg->power_factor * cfg->gain_i * scaling1;
    p->digiq_q_gain = cfg->power_factor * cfg->gain_q * scaling1;
    p->phase_balance = cfg->phase_balance;

    /* FM modulator (TxProcessor_FM, tx_processor.c:534-588) and its softdds tables */
    memcpy(p->dds_table, uhsdr_dds_table, sizeof p->dds_table);
    if (fm)
    {
        p->fm = 1;
        p->fm_mod_mult = cfg->fm_deviation_5k ? 2 : 1;
        const int32_t tf = p->freq_shift_hz;
        p->fm_word = (uint32_t)(((1 << 16) * (tf < 0 ? -tf : tf)) / IQ_SAMPLE_RATE);   /* FM_MOD_ACC_MAX_VALUE */
        p->fm_swap = tf < 0;
        float tone;
        memcpy(&tone, &uhsdr_fm_subaudible[cfg->fm_subaudible_tone], 4);
        /* AudioManagement_CalcSubaudibleGenFreq -> softdds_setFreqDDS (softdds.c:26-47) */
        p->fm_sub_on = tone > 0;
        uint64_t freq64_shifted = tone * 1024;                /* DDS_TBL_SIZE */
        freq64_shifted <<= 22;                                /* SOFTDDS_ACC_SHIFT */
        p->fm_sub_step = (uint32_t)(freq64_shifted / IQ_SAMPLE_RATE);
        const float fm_mod_mult = p->fm_mod_mult;
        p->fm_sub_scale = 0.00045 * fm_mod_mult;              /* FM_SUBAUDIBLE_TONE_AMPLITUDE_SCALING */
        /* tone burst: fm_tone_burst_freq[] = { 0, 1750, 2135 } (audio_management.c:328),
           FM_TONE_BURST_AMPLITUDE_SCALING = FM_MOD_SCALING / 4266.0 (tx_processor.c:519) */
        static const uint32_t burst_hz[3] = { 0, 1750, 2135 };
        p->tone_burst_step = softdds_step((float)burst_hz[cfg->fm_tone_burst_mode], IQ_SAMPLE_RATE);
        p->tone_burst_scale = (16 / 4266.0) * fm_mod_mult;
    }
    /* TUNE tones of the voice modes: SSB_TUNE_FREQ (hardware/uhsdr_board.h:114) and + 1200 Hz */
    p->tune_step[0] = softdds_step(750.0f, IQ_SAMPLE_RATE);
    p->tune_step[1] = softdds_step(750.0f + 1200, IQ_SAMPLE_RATE);
    return UHSDR_OK;
}

int32_t uhsdr_sizeof_tx_config(void) { return (int32_t)sizeof(uhsdr_tx_config); }
int32_t uhsdr_sizeof_tx_plan(void) { return (int32_t)sizeof(uhsdr_tx_plan); }

/* ---- spectrum display (UiSpectrum_InitSpectrumDisplayData, ui_spectrum.c:955-990; window and
   averaging of UiSpectrum_RedrawSpectrum, :1350-1446) ---- */
void uhsdr_spectrum_config_default(uhsdr_spectrum_config* cfg)
{
    if (!cfg) return;
    memset(cfg, 0, sizeof *cfg);
    cfg->fft_len = 1024;                  /* C3; the firmware's displays use 256 / 512 */
    cfg->spectrum_filter = 4;             /* SPECTRUM_FILTER_DEFAULT */
    cfg->iq_auto_correction = 0;
    cfg->iq_gain_i = 1.0f;
    cfg->iq_gain_q = 1.0f;
    cfg->iq_phase_balance = 0.0f;
    cfg->magnify = 0;
    cfg->iq_freq_mode = UHSDR_IQ_CONV_M12KHZ;   /* as uhsdr_rx_config_default */
}

uhsdr_status uhsdr_spectrum_plan_build(const uhsdr_spectrum_config* cfg, uhsdr_spectrum_plan* p)
{
    if (!cfg || !p) { uhsdr_set_error("null argument"); return UHSDR_ARGUMENT_ERROR; }
    const uhsdr_spectrum_desc* d = NULL;
    for (int i = 0; i < 3; ++i)
        if (uhsdr_spectrum_tables[i].fft_len == cfg->fft_len) d = &uhsdr_spectrum_tables[i];
    if (!d) { uhsdr_set_error("fft_len %d: need 256, 512 or 1024", cfg->fft_len); return UHSDR_ARGUMENT_ERROR; }
    if (cfg->spectrum_filter < 1 || cfg->spectrum_filter > 20)
    { uhsdr_set_error("spectrum_filter %d outside 1..20", cfg->spectrum_filter); return UHSDR_ARGUMENT_ERROR; }
    memset(p, 0, sizeof *p);
    const int L = d->fft_len;
    p->fft_len = L;
    p->window_formula = d->window_formula;
    p->iq_auto_correction = cfg->iq_auto_correction != 0;
    p->iq_gain_i = cfg->iq_gain_i;
    p->iq_gain_q = cfg->iq_gain_q;
    p->iq_phase_balance = cfg->iq_phase_balance;
    p->filt_factor = 1 / (float)cfg->spectrum_filter;
    if (cfg->magnify < 0 || cfg->magnify > 5)
    { uhsdr_set_error("magnify %d outside 0..5 (MAGNIFY_MIN..MAGNIFY_MAX)", cfg->magnify); return UHSDR_ARGUMENT_ERROR; }
    p->magnify = cfg->magnify;
    p->zoom_decimation = 1 << cfg->magnify;
    shift_plan(cfg->iq_freq_mode, &p->freq_shift_hz, &p->shift_kind, &p->shift_up, &p->osc_cos, &p->osc_sin);
    if (cfg->magnify > 0)
    {
        const uhsdr_zoom_desc* z = &uhsdr_zoom_tables[cfg->magnify - 1];
        p->zoom_taps = z->taps;
        memcpy(p->zoom_biquad, z->biquad, sizeof p->zoom_biquad);
        memcpy(p->zoom_fir, z->fir, sizeof(float) * z->taps);
    }
    p->bitrev_len = d->bitrev_len;
    memcpy(p->window, d->window, sizeof(float) * 2 * L);
    memcpy(p->twiddle, d->twiddle, sizeof(float) * 2 * L);
    memcpy(p->bitrev, d->bitrev, sizeof(uint16_t) * d->bitrev_len);
    /* arm_bitreversal_32 (arm_bitreversal2.S:136-180) swaps the complex values at byte offsets
       bitrev[2k], bitrev[2k+1]; applied to the identity it gives where each output bin comes from */
    for (int k = 0; k < L; ++k) p->perm[k] = (uint16_t)k;
    for (int it = 0; it < ((d->bitrev_len + 1) >> 2); ++it)
        for (int s = 0; s < 2; ++s)
        {
            const int a = d->bitrev[4 * it + 2 * s] >> 3, b = d->bitrev[4 * it + 2 * s + 1] >> 3;
            if (a >= L || b >= L) { uhsdr_set_error("bit-reversal table entry out of range"); return UHSDR_ARGUMENT_ERROR; }
            const uint16_t t = p->perm[a];
            p->perm[a] = p->perm[b];
            p->perm[b] = t;
        }
    for (int k = 0; k < L; ++k) p->iperm[p->perm[k]] = (uint16_t)k;
    /* per-lane copies of the first-stage twiddles (uhsdr_spectrum.hip): radix-8 stage of span
       L (512 / 1024: twiddle k * lane * tm, tm = 1024 / L) or the radix-4 rows of the 256-point
       split (twiddles t, 2t, 3t of row t = lane <= 32 ? lane : 64 - lane) */
    for (int lane = 0; lane < 64; ++lane)
        for (int k = 0; k < 8; ++k)
        {
            int idx = 0;
            if (L == 256) idx = k >= 1 && k <= 3 ? k * (lane <= 32 ? lane : 64 - lane) : 0;
            else idx = k * lane * (L == 1024 ? 2 : 1);
            p->tw_lane[k][lane][0] = p->twiddle[2 * idx];
            p->tw_lane[k][lane][1] = p->twiddle[2 * idx + 1];
        }
    return UHSDR_OK;
}

int32_t uhsdr_sizeof_spectrum_config(void) { return (int32_t)sizeof(uhsdr_spectrum_config); }
int32_t uhsdr_sizeof_spectrum_plan(void) { return (int32_t)sizeof(uhsdr_spectrum_plan); }
