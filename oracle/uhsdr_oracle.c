#define _GNU_SOURCE
/*
 * ORACLE -- TEST INFRASTRUCTURE ONLY (see uhsdr_oracle.h).  Compile without FP contraction
 * (-ffp-contract=off, no -march): every float operation below is one IEEE-754 binary32
 * rounding in the reference's order, so results are bit-identical to the reference firmware
 * built for x86.
 *
 * Processing is per 32-frame call, the ISR granularity of AudioDriver_I2SCallback
 * (audio_driver.c:2962-3049), because several state updates happen once per call
 * (auto I/Q statistics, oscillator gain renormalisation).
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>
#include "uhsdr_oracle.h"

#define BLK UHSDR_IQ_BLOCK_SIZE
#define IQ_BIT_SCALE_DOWN 0.0000152587890625f   /* audio_driver.h:596 (2^-16) */
#define CMSIS_PI 3.14159265358979f              /* PI, CMSIS/Include/arm_math.h:334 */

size_t uo_rx_state_size(void) { return sizeof(uo_rx_state); }

void uo_rx_state_init(const uhsdr_rx_plan* p, uo_rx_state* s)
{
    memset(s, 0, sizeof *s);
    s->osc_vi = 0.0f;          /* FreqShift_Approx_Prepare, freq_shift.c:48-49 */
    s->osc_vq = 1.0f;
    s->out_index = p->agc.out_index0;
    s->in_index = p->agc.in_index0;
    s->fm_squelched = 1;       /* AudioDriver_FM_Rx_Init: "we start squelched" (audio_driver.c:475) */
    s->cw_old = 0.001f;        /* static float32_t old_siglevel = 0.001 (cw_decoder.c:189) */
    s->tp_state = UHSDR_TWINPEAKS_WAIT;   /* ts.twinpeaks_tested at boot, src/uhsdr_main.c:339 */
}

void uo_rx_status(uo_rx_state* states, int C, int32_t* clip, int32_t* twinpeaks, int rearm)
{
    for (int c = 0; c < C; c++)
    {
        uo_rx_state* s = &states[c];
        if (clip) clip[c] = s->clip;
        s->clip = 0;
        if (twinpeaks) twinpeaks[c] = s->tp_state;
        if (rearm && s->tp_state == UHSDR_TWINPEAKS_CODEC_RESTART) s->tp_state = UHSDR_TWINPEAKS_WAIT;
    }
}

/* AudioDriver_RxHandleTwinpeaks (audio_driver.c:2173-2248), once per call after the auto I/Q
   statistics, on this call's low-passed teta1 / teta3 */
static void twinpeaks(uo_rx_state* s, float teta1, float teta3)
{
    if (s->tp_state == UHSDR_TWINPEAKS_WAIT) s->tp_counter++;
    if (s->tp_counter > 1000)
    {
        s->tp_state = UHSDR_TWINPEAKS_SAMPLING;
        s->tp_counter = 0;
        s->tp_phase = 0.0;
        s->tp_runs = 0;
    }
    if (teta3 != 0.0 && s->tp_state == UHSDR_TWINPEAKS_SAMPLING)
    {
        const float cur = asinf(teta1 / teta3);
        if (s->tp_runs == 0) s->tp_phase = cur;
        else s->tp_phase = 0.05 * cur + 0.95 * s->tp_phase;
        s->tp_runs++;
        if (s->tp_runs == 50)
        {
            if (fabsf(s->tp_phase) > (M_PI / 8.0))
            {
                s->tp_state = UHSDR_TWINPEAKS_CODEC_RESTART;
                s->tp_restarts++;
                if (s->tp_restarts >= 4)
                {
                    s->tp_state = UHSDR_TWINPEAKS_UNCORRECTABLE;
                    s->tp_restarts = 0;
                }
            }
            else
            {
                s->tp_state = UHSDR_TWINPEAKS_DONE;
                s->tp_restarts = 0;
            }
        }
    }
}

/* CwDecode_RxProcessor (cw_decoder.c:383-397) and CW_Decode_exe steps 1-5 (:182-316) with the
   default configuration (one Goertzel, cw_decoder.h:19): Goertzel over the first blocksize
   samples of each block (AudioFilter_GoertzelInput / _Energy, audio_filter.c:1290-1305),
   exponential smoothing, threshold, two-sample noise cancel -> ads.CW_signal */
static void cw_front(const uhsdr_rx_plan* p, uo_rx_state* s, const float* x, int n)
{
    s->cw_blocks_out = 0;
    for (int i = 0; i < n; i++)
    {
        if (s->cw_count < p->cw_blocksize)
        {
            const float g0 = p->cw_r * s->cw_g1 - s->cw_g2 + x[i];
            s->cw_g2 = s->cw_g1;
            s->cw_g1 = g0;
        }
        s->cw_count++;
    }
    if (s->cw_count >= p->cw_blocksize)
    {
        const float a = (s->cw_g1 - (s->cw_g2 * p->cw_cos));
        const float b = (s->cw_g2 * p->cw_sin);
        s->cw_g1 = s->cw_g2 = 0.0f;
        const float magnitude = sqrtf(a * a + b * b);
        float siglevel = magnitude;
        siglevel = siglevel * 0.1 + (1.0 - 0.1) * s->cw_old;       /* SIGNAL_TAU = 0.1 */
        s->cw_old = magnitude;
        const int newstate = (siglevel >= p->cw_thresh);
        if (p->cw_noisecancel)
        {
            if (s->cw_change) { s->cw_state = newstate; s->cw_change = 0; }
            else if (newstate != s->cw_state) s->cw_change = 1;
        }
        else s->cw_state = newstate;
        s->cw_energy_out = magnitude;
        s->cw_blocks_out = 1;
        s->cw_count = 0;
    }
    s->cw_signal_out = s->cw_state;
}

/* ---- CMSIS-DSP f32 kernels, restated (generic code paths; the CM7 unrolled versions
        accumulate in the same order) ---- */

/* arm_fir_f32.c:482-560: y[n] = sum_k c[k]*s[n+k], acc from 0.0f in tap order.
   hist holds the T-1 most recent inputs. */
static void fir(const float* c, int T, float* hist, const float* x, float* y, int n)
{
    float st[UHSDR_MAX_FIR_TAPS + BLK];
    memcpy(st, hist, sizeof(float) * (T - 1));
    memcpy(st + T - 1, x, sizeof(float) * n);
    for (int i = 0; i < n; i++)
    {
        float acc = 0.0f;
        for (int k = 0; k < T; k++) acc += st[i + k] * c[k];
        y[i] = acc;
    }
    memcpy(hist, st + n, sizeof(float) * (T - 1));
}

/* arm_fir_decimate_f32.c:440-518: one output per M inputs, same dot product. */
static void fir_decimate(const float* c, int T, int M, float* hist, const float* x, float* y, int n)
{
    float st[UHSDR_MAX_DEC_TAPS + BLK];
    memcpy(st, hist, sizeof(float) * (T - 1));
    memcpy(st + T - 1, x, sizeof(float) * n);
    for (int m = 0; m < n / M; m++)
    {
        float sum = 0.0f;
        for (int k = 0; k < T; k++) sum += st[m * M + k] * c[k];
        y[m] = sum;
    }
    memcpy(hist, st + n, sizeof(float) * (T - 1));
}

/* arm_fir_interpolate_f32.c:482-575: polyphase, output j of input m uses phase L-1-j. */
static void fir_interpolate(const float* c, int L, int P, float* hist, const float* x, float* y, int n)
{
    float st[UHSDR_MAX_INTERP + BLK];
    memcpy(st, hist, sizeof(float) * (P - 1));
    memcpy(st + P - 1, x, sizeof(float) * n);
    for (int m = 0; m < n; m++)
    {
        for (int i = L; i > 0; i--)
        {
            float sum = 0.0f;
            for (int t = 0; t < P; t++) sum += st[m + t] * c[(i - 1) + t * L];
            *y++ = sum;
        }
    }
    if (P > 1) memcpy(hist, st + n, sizeof(float) * (P - 1));
}

/* arm_iir_lattice_f32.c:348-447 (see the state hand-over: stage i of the next sample
   reads what stage i+1 wrote, the last one reads the final forward value). */
static void iir_lattice(const float* k, const float* v, int S, float* g, const float* x, float* y, int n)
{
    for (int m = 0; m < n; m++)
    {
        float fcurr = x[m], fnext = 0.0f, acc = 0.0f;
        float gn[UHSDR_MAX_LATTICE];
        for (int i = 0; i < S; i++)
        {
            const float gcurr = g[i];
            fnext = fcurr - (k[i] * gcurr);
            const float gnext = (fnext * k[i]) + gcurr;
            acc += (gnext * v[i]);
            gn[i] = gnext;
            fcurr = fnext;
        }
        acc += (fnext * v[S]);
        for (int i = 0; i < S - 1; i++) g[i] = gn[i + 1];
        g[S - 1] = fnext;
        y[m] = acc;
    }
}

/* arm_biquad_cascade_df1_f32.c:349-418, state per stage {x1, x2, y1, y2}. */
static void biquad_df1(const float* coeffs, int stages, float* st, float* x, int n)
{
    for (int s = 0; s < stages; s++)
    {
        const float b0 = coeffs[5 * s], b1 = coeffs[5 * s + 1], b2 = coeffs[5 * s + 2];
        const float a1 = coeffs[5 * s + 3], a2 = coeffs[5 * s + 4];
        float Xn1 = st[4 * s], Xn2 = st[4 * s + 1], Yn1 = st[4 * s + 2], Yn2 = st[4 * s + 3];
        for (int i = 0; i < n; i++)
        {
            const float Xn = x[i];
            const float acc = (b0 * Xn) + (b1 * Xn1) + (b2 * Xn2) + (a1 * Yn1) + (a2 * Yn2);
            x[i] = acc;
            Xn2 = Xn1; Xn1 = Xn; Yn2 = Yn1; Yn1 = acc;
        }
        st[4 * s] = Xn1; st[4 * s + 1] = Xn2; st[4 * s + 2] = Yn1; st[4 * s + 3] = Yn2;
    }
}

/* Math_log10f_fast, misc/uhsdr_math.c:26-39 */
static float log10f_fast(float X)
{
    float Y, F;
    int E;
    F = frexpf(fabsf(X), &E);
    Y = 1.23149591368684f;
    Y *= F;
    Y += -4.11852516267426f;
    Y *= F;
    Y += 6.02197014179219f;
    Y *= F;
    Y += -3.13396450166353f;
    Y += E;
    return (Y * 0.3010299956639812f);
}

static float sign_new(float x) { return (x < 0) ? -1.0 : ((x > 0) ? 1.0 : 0.0); }  /* uhsdr_math.c:84-87 */

/* AudioAgc_RunAgcWdsp, audio_agc.c:349-595; buf1 != NULL: use_stereo (second channel in the
   odd ring slots, abs_ring = the larger magnitude, one gain for both) */
static void agc_run(const uhsdr_agc_plan* a, uo_rx_state* s, float* buf, float* buf1, int n)
{
    if (a->mode == 5)
    {
        for (int i = 0; i < n; i++)
        {
            buf[i] = buf[i] * a->fixed_gain;
            if (buf1) buf1[i] = buf1[i] * a->fixed_gain;
        }
        return;
    }
    for (int i = 0; i < n; i++)
    {
        if (++s->out_index >= a->ring_buffsize) s->out_index -= a->ring_buffsize;
        if (++s->in_index >= a->ring_buffsize) s->in_index -= a->ring_buffsize;
        const float out_sample = s->ring[s->out_index];
        const float out_sample1 = s->ring1[s->out_index];
        const float abs_out_sample = s->abs_ring[s->out_index];
        s->ring[s->in_index] = buf[i];
        if (buf1) s->ring1[s->in_index] = buf1[i];
        s->abs_ring[s->in_index] = fabsf(buf[i]);
        if (buf1 && s->abs_ring[s->in_index] < fabsf(buf1[i])) s->abs_ring[s->in_index] = fabsf(buf1[i]);

        s->fast_backaverage = a->fast_backmult * abs_out_sample + a->onemfast_backmult * s->fast_backaverage;
        s->hang_backaverage = a->hang_backmult * abs_out_sample + a->onemhang_backmult * s->hang_backaverage;

        if ((abs_out_sample >= s->ring_max) && (abs_out_sample > 0.0))
        {
            s->ring_max = 0.0;
            int k = s->out_index;
            for (int j = 0; j < a->attack_buffsize; j++)
            {
                if (++k == a->ring_buffsize) k = 0;
                if (s->abs_ring[k] > s->ring_max) s->ring_max = s->abs_ring[k];
            }
        }
        if (s->abs_ring[s->in_index] > s->ring_max) s->ring_max = s->abs_ring[s->in_index];

        if (s->hang_counter > 0) --s->hang_counter;

        switch (s->state)
        {
        case 0:
            if (s->ring_max >= s->volts)
                s->volts += (s->ring_max - s->volts) * a->attack_mult;
            else if (s->volts > a->pop_ratio * s->fast_backaverage)
            {
                s->state = 1;
                s->volts += (s->ring_max - s->volts) * a->fast_decay_mult;
            }
            else if (a->hang_enable && (s->hang_backaverage > a->hang_level))
            {
                s->state = 2;
                s->hang_counter = a->hang_counter_init;
                s->decay_type = 1;
            }
            else
            {
                s->state = 3;
                s->volts += (s->ring_max - s->volts) * a->decay_mult;
                s->decay_type = 0;
            }
            break;
        case 1:
            if (s->ring_max >= s->volts)
            {
                s->state = 0;
                s->volts += (s->ring_max - s->volts) * a->attack_mult;
            }
            else if (s->volts > s->save_volts)
                s->volts += (s->ring_max - s->volts) * a->fast_decay_mult;
            else if (s->hang_counter > 0)
                s->state = 2;
            else if (s->decay_type == 0)
            {
                s->state = 3;
                s->volts += (s->ring_max - s->volts) * a->decay_mult;
            }
            else
            {
                s->state = 4;
                s->volts += (s->ring_max - s->volts) * a->hang_decay_mult;
            }
            break;
        case 2:
            if (s->ring_max >= s->volts)
            {
                s->state = 0;
                s->save_volts = s->volts;
                s->volts += (s->ring_max - s->volts) * a->attack_mult;
            }
            else if (s->hang_counter == 0)
            {
                s->state = 4;
                s->volts += (s->ring_max - s->volts) * a->hang_decay_mult;
            }
            break;
        case 3:
            if (s->ring_max >= s->volts)
            {
                s->state = 0;
                s->save_volts = s->volts;
                s->volts += (s->ring_max - s->volts) * a->attack_mult;
            }
            else
                s->volts += (s->ring_max - s->volts) * a->decay_mult;
            break;
        case 4:
            if (s->ring_max >= s->volts)
            {
                s->state = 0;
                s->save_volts = s->volts;
                s->volts += (s->ring_max - s->volts) * a->attack_mult;
            }
            else
                s->volts += (s->ring_max - s->volts) * a->hang_decay_mult;
            break;
        }
        if (s->volts < a->min_volts) s->volts = a->min_volts;

        float vo = log10f_fast(a->inv_max_input * s->volts);
        if (vo > 0.0) vo = 0.0;
        const float mult = (a->out_target - a->slope_constant * vo) / s->volts;
        buf[i] = out_sample * mult;
        if (buf1) buf1[i] = out_sample1 * mult;
    }
    if (a->remove_dc)
    {
        for (int i = 0; i < n; i++)
        {
            const float w = buf[i] + s->wold * 0.9999;
            buf[i] = w - s->wold;
            s->wold = w;
            if (buf1)
            {
                const float w1 = buf1[i] + s->wold1 * 0.9999;
                buf1[i] = w1 - s->wold1;
                s->wold1 = w1;
            }
        }
    }
}

/* AudioDriver_FadeLeveler, audio_driver.c:1911-1923 (channel 0) */
static float fade_leveler(const uhsdr_rx_plan* p, uo_rx_state* s, float audio, float corr)
{
    s->fade_dc27 = p->fade_mtauR * s->fade_dc27 + p->fade_onem_mtauR * audio;
    s->fade_dc_insert = p->fade_mtauI * s->fade_dc_insert + p->fade_onem_mtauI * corr;
    audio = audio + s->fade_dc_insert - s->fade_dc27;
    return audio;
}
/* channel 1 (only its output matters in stereo) */
static float fade_leveler1(const uhsdr_rx_plan* p, uo_rx_state* s, float audio, float corr)
{
    s->fade_dc27_1 = p->fade_mtauR * s->fade_dc27_1 + p->fade_onem_mtauR * audio;
    s->fade_dc_insert_1 = p->fade_mtauI * s->fade_dc_insert_1 + p->fade_onem_mtauI * corr;
    audio = audio + s->fade_dc_insert_1 - s->fade_dc27_1;
    return audio;
}

/* the 7-stage allpass pair of the SAM sideband selector, demod_sam_const (audio_driver.c:1931-1953) */
static const float sam_c0[7] = { -0.328201924180698, -0.744171491539427, -0.923022915444215, -0.978490468768238,
                                 -0.994128272402075, -0.998458978159551, -0.999790306259206 };
static const float sam_c1[7] = { -0.0991227952747244, -0.565619728761389, -0.857467122550052, -0.959123933111275,
                                 -0.988739372718090, -0.996959189310611, -0.999282492800792 };

/* AudioDriver_DemodSAM, audio_driver.c:1990-2166 (mono; the display-only carrier estimate
   at :2150-2162 does not touch the audio and is not restated) */
static void demod_sam(const uhsdr_rx_plan* p, uo_rx_state* s, const float* ib, const float* qb, float* a0, float* a1,
                      int n)
{
    if (p->dmod_mode == UHSDR_DEMOD_AM)
    {
        for (int i = 0; i < n; i++)
        {
            const float in = ib[i] * ib[i] + qb[i] * qb[i];
            float audio = (in >= 0.0f) ? sqrtf(in) : 0.0f;      /* arm_sqrt_f32, arm_math.h:5745-5771 */
            if (p->fade_leveler) audio = fade_leveler(p, s, audio, 0);
            a0[i] = audio;
        }
        return;
    }
    for (int i = 0; i < n; i++)
    {
        float Sin, Cos;
        sincosf(s->sam_phs, &Sin, &Cos);
        const float ai = Cos * ib[i];
        const float bi = Sin * ib[i];
        const float aq = Cos * qb[i];
        const float bq = Sin * qb[i];
        float audio, audio1 = 0;
        const float corr[2] = { ai + bq, -bi + aq };
        if (p->sam_sideband != UHSDR_SAM_SIDEBAND_BOTH)
        {
            s->sam_a[0] = s->sam_dsI;
            s->sam_b[0] = bi;
            s->sam_c[0] = s->sam_dsQ;
            s->sam_d[0] = aq;
            s->sam_dsI = ai;
            s->sam_dsQ = bq;
            for (int j = 0; j < 7; j++)
            {
                const int k = 3 * j;
                s->sam_a[k + 3] = sam_c0[j] * (s->sam_a[k] - s->sam_a[k + 5]) + s->sam_a[k + 2];
                s->sam_b[k + 3] = sam_c1[j] * (s->sam_b[k] - s->sam_b[k + 5]) + s->sam_b[k + 2];
                s->sam_c[k + 3] = sam_c0[j] * (s->sam_c[k] - s->sam_c[k + 5]) + s->sam_c[k + 2];
                s->sam_d[k + 3] = sam_c1[j] * (s->sam_d[k] - s->sam_d[k + 5]) + s->sam_d[k + 2];
            }
            const float ai_ps = s->sam_a[21], bi_ps = s->sam_b[21], bq_ps = s->sam_c[21], aq_ps = s->sam_d[21];
            for (int j = 23; j > 0; j--)
            {
                s->sam_a[j] = s->sam_a[j - 1];
                s->sam_b[j] = s->sam_b[j - 1];
                s->sam_c[j] = s->sam_c[j - 1];
                s->sam_d[j] = s->sam_d[j - 1];
            }
            if (p->sam_sideband == UHSDR_SAM_SIDEBAND_LSB) audio = (ai_ps + bi_ps) - (aq_ps - bq_ps);
            else if (p->sam_sideband == UHSDR_SAM_SIDEBAND_STEREO)
            {
                audio = (ai_ps + bi_ps) - (aq_ps - bq_ps);      /* audio_driver.c:2091-2094 */
                audio1 = (ai_ps - bi_ps) + (aq_ps + bq_ps);
            }
            else audio = (ai_ps - bi_ps) + (aq_ps + bq_ps);
        }
        else
        {
            audio = corr[0];
        }
        if (p->fade_leveler)
        {
            audio = fade_leveler(p, s, audio, corr[0]);
            audio1 = fade_leveler1(p, s, audio1, corr[0]);
        }
        a0[i] = audio;
        if (a1) a1[i] = audio1;
        const float phzerror = atan2f(corr[1], corr[0]);
        const float del_out = s->sam_fil_out;
        s->sam_omega2 = s->sam_omega2 + p->sam_g2 * phzerror;
        if (s->sam_omega2 < p->sam_omega_min) s->sam_omega2 = p->sam_omega_min;
        else if (s->sam_omega2 > p->sam_omega_max) s->sam_omega2 = p->sam_omega_max;
        s->sam_fil_out = p->sam_g1 * phzerror + s->sam_omega2;
        s->sam_phs = s->sam_phs + del_out;
        while (s->sam_phs >= 2.0 * CMSIS_PI) s->sam_phs -= (2.0 * CMSIS_PI);
        while (s->sam_phs < 0.0) s->sam_phs += (2.0 * CMSIS_PI);
    }
}

/* AudioFilter_GoertzelInput / _Energy, audio_filter.c:1290-1305 */
static void goertzel_in(float r, float* b, float in)
{
    const float b0 = r * b[0] - b[1] + in;
    b[1] = b[0];
    b[0] = b0;
}
static float goertzel_energy(float co, float si, float* b)
{
    const float a = (b[0] - (b[1] * co));
    const float bb = (b[1] * si);
    b[0] = 0;
    b[1] = 0;
    return sqrtf(a * a + bb * bb);
}

/* AudioDriver_DemodFM, audio_driver.c:1544-1737, with the subaudible tone detector (:1665-1734);
   returns signal_active = !squelched after this call's squelch update */
static int demod_fm(const uhsdr_rx_plan* p, uo_rx_state* s, const float* ib, const float* qb, float* a0, int n)
{
    float sq[BLK], gbuf[BLK];
    if (p->freq_shift_hz == 0) return !s->fm_squelched;      /* bails out without translation (:1548) */
    const int tone_en = p->tone_det_enabled;
    for (int i = 0; i < n; i++)
    {
        const float y = (s->fm_i_prev * qb[i]) - (ib[i] * s->fm_q_prev);
        const float x = (s->fm_i_prev * ib[i]) + (qb[i] * s->fm_q_prev);
        const float angle = atan2f(y, x);
        sq[i] = angle;
        const float a = s->fm_lpf_prev + (0.05 * (angle - s->fm_lpf_prev));     /* FM_RX_LPF_ALPHA */
        s->fm_lpf_prev = a;
        gbuf[i] = a;
        if ((!s->fm_squelched && !tone_en) || (s->fm_tone_detected && tone_en) || !p->fm_sql_threshold)
        {
            const float b = 0.96 * (s->fm_hpf_prev_b + a - s->fm_hpf_prev_a);  /* FM_RX_HPF_ALPHA */
            s->fm_hpf_prev_a = a;
            s->fm_hpf_prev_b = b;
            a0[i] = b;
        }
        else
        {
            a0[i] = 0;
        }
        s->fm_q_prev = qb[i];
        s->fm_i_prev = ib[i];
    }
    iir_lattice(p->sq_k, p->sq_v, p->sq_stages, s->fm_sq, sq, sq, n);
    s->fm_sql_avg = ((1 - 0.005) * s->fm_sql_avg) + (0.005 * sqrtf(fabsf(sq[0])));   /* FM_RX_SQL_SMOOTHING */
    s->fm_count = (s->fm_count + 1) % 200;                                            /* FM_SQUELCH_PROC_DECIMATION */
    if (s->fm_count == 0)
    {
        if (s->fm_sql_avg > 0.175) s->fm_sql_avg = 0.175;
        float scaled_sql_avg = s->fm_sql_avg * 172;
        if (scaled_sql_avg > 24) scaled_sql_avg = 24;
        scaled_sql_avg = 22 - scaled_sql_avg;
        const int thr = p->fm_sql_threshold;
        if (thr == 0) s->fm_squelched = 0;
        else if (s->fm_squelched)
        {
            if (scaled_sql_avg >= (float)(thr + 3)) s->fm_squelched = 0;           /* FM_SQUELCH_HYSTERESIS */
        }
        else if (thr > 3)
        {
            if (scaled_sql_avg < (float)(thr - 3)) s->fm_squelched = 1;
        }
        else if (scaled_sql_avg < (float)thr)
        {
            s->fm_squelched = 1;
        }
    }
    if (tone_en)
    {
        s->fm_gcount++;
        for (int i = 0; i < n; i++)
        {
            goertzel_in(p->tone_r[0], s->fm_g[0], gbuf[i]);     /* FM_HIGH */
            goertzel_in(p->tone_r[1], s->fm_g[1], gbuf[i]);     /* FM_LOW */
            goertzel_in(p->tone_r[2], s->fm_g[2], gbuf[i]);     /* FM_CTR */
        }
        if (s->fm_gcount >= 400)                                /* FM_SUBAUDIBLE_GOERTZEL_WINDOW */
        {
            const float so = goertzel_energy(p->tone_cos[0], p->tone_sin[0], s->fm_g[0])
                           + goertzel_energy(p->tone_cos[1], p->tone_sin[1], s->fm_g[1]);
            const float r = goertzel_energy(p->tone_cos[2], p->tone_sin[2], s->fm_g[2]);
            s->fm_subdet = ((1 - 0.9) * s->fm_subdet) + (r / (so / 2) * 0.9);    /* FM_TONE_DETECT_ALPHA */
            if (s->fm_subdet > 1.75)                            /* FM_SUBAUDIBLE_TONE_DET_THRESHOLD */
            {
                s->fm_tdet++;
                if (s->fm_tdet > 5) s->fm_tdet = 5;             /* FM_SUBAUDIBLE_DEBOUNCE_MAX */
            }
            else if (s->fm_tdet)
                s->fm_tdet--;
            s->fm_tone_detected = s->fm_tdet >= 2;              /* FM_SUBAUDIBLE_TONE_DEBOUNCE_THRESHOLD */
            s->fm_gcount = 0;
        }
    }
    return !s->fm_squelched;
}

/* AudioDriver_NotchFilter (audio_driver.c:1746-1763): delay line + arm_lms_norm_f32
   (CMSIS .../arm_lms_norm_f32.c, sequential tap order) in place on a0 */
static void notch_run(const uhsdr_rx_plan* p, uo_rx_state* s, float* a0, int n)
{
    const int T = p->notch_taps, D = p->notch_delay_len;
    memcpy(&s->notch_delay[s->notch_in], a0, sizeof(float) * n);
    const float* ref = &s->notch_delay[s->notch_out];
    float* st = s->notch_st;                  /* [0 .. T-2] carried, new samples appended */
    const float mu = p->notch_mu;
    for (int i = 0; i < n; i++)
    {
        const float in = a0[i];
        st[T - 1 + i] = in;
        s->notch_energy -= s->notch_x0 * s->notch_x0;
        s->notch_energy += in * in;
        float sum = 0.0f;
        for (int k = 0; k < T; k++) sum += st[i + k] * s->notch_w[k];
        const float e = ref[i] - sum;
        a0[i] = e;
        const float w = (e * mu) / (s->notch_energy + 0.000000119209289f);
        for (int k = 0; k < T; k++) s->notch_w[k] += w * st[i + k];
        s->notch_x0 = st[i];
    }
    memmove(st, st + n, sizeof(float) * (T - 1));
    s->notch_in += n;
    s->notch_out = s->notch_in + n;
    s->notch_in %= D;
    s->notch_out %= D;
}

void uo_rx_key_beep(uo_rx_state* states, int C, int calls)
{
    for (int c = 0; c < C; c++)
    {
        states[c].beep_acc = 0;               /* AudioManagement_KeyBeep, audio_management.c:372 */
        states[c].beep_left = calls;
    }
}

/* float -> int32 as x86 cvttss2si does it (out of range / NaN -> INT32_MIN), then the
   firmware's << AUDIO_BIT_SHIFT (audio_driver.c:2911-2923) in two's complement. */
static int32_t to_dma(float f)
{
    int32_t v = (f > -2147483904.0f && f < 2147483648.0f) ? (int32_t)f : INT32_MIN;
    return (int32_t)((uint32_t)v << 16);
}

/* key beep (audio_driver.c:2891-2898): is it on for this call (ts.beep_timing > 0)? */
static int beep_on(const uhsdr_rx_plan* p, uo_rx_state* s)
{
    if (s->beep_left <= 0 || p->beep_step == 0) return 0;
    s->beep_left--;
    return 1;
}
/* softdds_nextSample (softdds.h:48-66) x ads.beep_loudness_factor */
static float beep_next(const uhsdr_rx_plan* p, uo_rx_state* s)
{
    const uint32_t k = (s->beep_acc >> 22) % 1024;
    s->beep_acc += p->beep_step;
    return (float)p->dds_table[k] * p->beep_scale;
}

/* one AudioDriver_RxProcessor call on BLK frames, audio_driver.c:2603-2942 */
static void rx_call(const uhsdr_rx_plan* p, uo_rx_state* s, const int32_t* iq, float* out_a1, float* out_a0,
                    int32_t* dst)
{
    float ib[BLK], qb[BLK], a0[BLK], a1[BLK];
    const int n = BLK;
    for (int i = 0; i < n; i++)
    {
        /* ADC clip indicators on the I sample, |l| >> IQ_BIT_SHIFT against ADC_CLIP_WARN_THRESHOLD
           = 4096 and its quarter / half (audio_driver.c:2660-2676, audio_driver.h:81); the
           magnitude is taken unsigned, so a full-scale negative sample counts as a clip */
        const uint32_t v = (uint32_t)iq[2 * i];
        const uint32_t level = ((v & 0x80000000u) ? 0u - v : v) >> 16;
        if (level > 4096 / 4) s->clip |= UHSDR_ADC_QUARTER_CLIP;
        if (level > 4096 / 2) s->clip |= UHSDR_ADC_HALF_CLIP;
        if (level > 4096) s->clip |= UHSDR_ADC_CLIP;
        ib[i] = iq[2 * i];
        qb[i] = iq[2 * i + 1];
    }
    for (int i = 0; i < n; i++) ib[i] = ib[i] * IQ_BIT_SCALE_DOWN;
    for (int i = 0; i < n; i++) qb[i] = qb[i] * IQ_BIT_SCALE_DOWN;

    /* AudioDriver_RxHandleIqCorrection, audio_driver.c:2254-2316 */
    if (!p->iq_auto_correction)
    {
        for (int i = 0; i < n; i++) ib[i] = ib[i] * p->iq_gain_i;
        for (int i = 0; i < n; i++) qb[i] = qb[i] * p->iq_gain_q;
        const float ph = p->iq_phase_balance;       /* AudioDriver_IQPhaseAdjust :1776-1801 */
        if (ph < 0)
            for (int i = 0; i < n; i++) { const float e = ib[i] * ph; qb[i] = qb[i] + e; }
        else if (ph > 0)
            for (int i = 0; i < n; i++) { const float e = qb[i] * ph; ib[i] = ib[i] + e; }
    }
    else
    {
        float t1 = 0.0f, t2 = 0.0f, t3 = 0.0f;
        for (int i = 0; i < n; i++)
        {
            t1 += sign_new(ib[i]) * qb[i];
            t2 += sign_new(ib[i]) * ib[i];
            t3 += sign_new(qb[i]) * qb[i];
        }
        t1 = -0.003 * (t1 / n) + 0.997 * s->teta1_old;
        t2 = 0.003 * (t2 / n) + 0.997 * s->teta2_old;
        t3 = 0.003 * (t3 / n) + 0.997 * s->teta3_old;
        const float M_c1 = (t2 != 0.0) ? t1 / t2 : 0.0;
        float help = (t2 * t2);
        if (help > 0.0) help = (t3 * t3 - t1 * t1) / help;
        const float M_c2 = (help > 0.0) ? sqrtf(help) : 1.0;
        twinpeaks(s, t1, t3);
        s->teta1_old = t1;
        s->teta2_old = t2;
        s->teta3_old = t3;
        for (int i = 0; i < n; i++) qb[i] += M_c1 * ib[i];
        for (int i = 0; i < n; i++) ib[i] = ib[i] * M_c2;
    }

    /* FreqShift, freq_shift.c:275-334 */
    if (p->freq_shift_hz != 0)
    {
        float* ip = p->shift_up ? ib : qb;
        float* qp = p->shift_up ? qb : ib;
        if (p->shift_kind == 1)
        {
            for (int i = 0; i < n; i += 4)   /* FreqShift_QuarterFs :219-262 */
            {
                float h1 = qp[i + 1], h2 = -ip[i + 1];
                ip[i + 1] = h1; qp[i + 1] = h2;
                h1 = -ip[i + 2]; h2 = -qp[i + 2];
                ip[i + 2] = h1; qp[i + 2] = h2;
                h1 = -qp[i + 3]; h2 = ip[i + 3];
                ip[i + 3] = h1; qp[i + 3] = h2;
            }
        }
        else
        {
            for (int i = 0; i < n; i++)      /* FreqShift_Approx :57-101 */
            {
                const float oq = (s->osc_vq * p->osc_cos) - (s->osc_vi * p->osc_sin);
                const float oi = (s->osc_vi * p->osc_cos) + (s->osc_vq * p->osc_sin);
                const float qt = qp[i], it = ip[i];
                qp[i] = (qt * oq) - (it * oi);
                ip[i] = (it * oq) + (qt * oi);
                s->osc_vq = oq;
                s->osc_vi = oi;
            }
            const float g = (3 - ((s->osc_vq * s->osc_vq) + (s->osc_vi * s->osc_vi))) / 2;
            s->osc_vq = g * s->osc_vq;
            s->osc_vi = g * s->osc_vi;
        }
    }

    const int nd = n / p->decimation_rate;
    const int niq = p->use_decimated_iq ? nd : n;
    const int am = p->dmod_mode == UHSDR_DEMOD_AM || p->dmod_mode == UHSDR_DEMOD_SAM;
    if (p->use_decimated_iq)
    {
        fir_decimate(p->dec, p->dec_taps, p->decimation_rate, s->dec_i, ib, ib, n);
        fir_decimate(am ? p->dec_q : p->dec, p->dec_taps, p->decimation_rate, s->dec_q, qb, qb, n);
    }
    if (p->hilbert_taps)
    {
        fir(p->hilbert_i, p->hilbert_taps, s->hil_i, ib, ib, niq);
        fir(p->hilbert_q, p->hilbert_taps, s->hil_q, qb, qb, niq);
    }
    if (p->dmod_mode == UHSDR_DEMOD_FM)
    {
        /* FM: no decimation / post-processing; audio = demod x FM_RX_SCALING (audio_driver.c:2818-2828),
           the AGC run there only rewrites a_buffer[0], which the output stage overwrites */
        const int active = demod_fm(p, s, ib, qb, a0, n);
        for (int i = 0; i < n; i++) a1[i] = a0[i] * p->fm_scale;
        biquad_df1(p->biquad2, 1, s->bq2, a1, n);      /* audio_driver.c:2832 */
        const int beep = beep_on(p, s);
        for (int i = 0; i < n; i++)
        {
            /* mute when squelched (:2843-2850), else the board's line-out stage (:2856-2885) */
            float v1 = 0.0f, v0 = 0.0f;
            if (active && p->single_channel) { v0 = a1[i] * p->line_out0_scale; v1 = a1[i] * p->spkr_scale; }
            else if (active) v0 = v1 = a1[i] * p->line_out_scale;
            if (beep)
            {
                const float t = beep_next(p, s);
                v1 += t;
                if (!p->single_channel) v0 += t;             /* mcHF: the speaker channel only, :2896 */
            }
            out_a1[i] = v1;
            if (out_a0) out_a0[i] = v0;
            if (dst) { dst[2 * i] = active ? to_dma(v1) : 0; dst[2 * i + 1] = active ? to_dma(v0) : 0; }
        }
        return;
    }
    /* second channel a_buffer[1] while at the decimated rate (use_stereo) */
    const int st = p->stereo;
    float b1[BLK], a0o[BLK];
    if (am)
        demod_sam(p, s, ib, qb, a0, st ? b1 : NULL, niq);
    else if (p->dmod_mode == UHSDR_DEMOD_IQ)          /* audio_driver.c:2769-2772 */
    {
        for (int i = 0; i < niq; i++) a0[i] = ib[i];
        if (st) for (int i = 0; i < niq; i++) b1[i] = qb[i];
    }
    else if (p->dmod_mode == UHSDR_DEMOD_SSBSTEREO)   /* :2773-2776 */
    {
        for (int i = 0; i < niq; i++) a0[i] = ib[i] + qb[i];
        if (st) for (int i = 0; i < niq; i++) b1[i] = ib[i] - qb[i];
    }
    else if (p->lsb)
        for (int i = 0; i < niq; i++) a0[i] = ib[i] - qb[i];
    else
        for (int i = 0; i < niq; i++) a0[i] = ib[i] + qb[i];

    if (!p->use_decimated_iq)
    {
        fir_decimate(p->dec, p->dec_taps, p->decimation_rate, s->dec_i, a0, a0, niq);
        if (st) fir_decimate(p->dec, p->dec_taps, p->decimation_rate, s->dec_q, b1, b1, niq);   /* DECIMATE_RX_Q, :2797-2801 */
    }

    /* RxProcessor_DemodAudioPostprocessing, audio_driver.c:2436-2592 */
    if (p->notch_enabled) notch_run(p, s, a0, nd);
    if (p->pre_stages > 0)
    {
        iir_lattice(p->pre_k, p->pre_v, p->pre_stages, s->pre, a0, a0, nd);
        if (st) iir_lattice(p->pre_k, p->pre_v, p->pre_stages, s->pre1, b1, b1, nd);
    }
    agc_run(&p->agc, s, a0, st ? b1 : NULL, nd);
    for (int i = 0; i < nd; i++) a0[i] = a0[i] * p->post_agc_scale;
    biquad_df1(p->biquad1, 4, s->bq1, a0, nd);
    if (st)
    {
        for (int i = 0; i < nd; i++) b1[i] = b1[i] * p->post_agc_scale;
        biquad_df1(p->biquad1, 4, s->bq1_1, b1, nd);
    }
    if (p->cw_enabled) cw_front(p, s, a0, nd);         /* audio_driver.c:2550-2557 */
    /* interpolation: channel 1 into a temporary that becomes a_buffer[0], channel 0 into
       a_buffer[1] (:2560-2577) */
    if (p->interp_phase > 0)
    {
        if (st) fir_interpolate(p->interp, p->interp_L, p->interp_phase, s->interp1, b1, a0o, nd);
        fir_interpolate(p->interp, p->interp_L, p->interp_phase, s->interp, a0, a1, nd);
    }
    if (p->aa_stages > 0)
    {
        iir_lattice(p->aa_k, p->aa_v, p->aa_stages, s->aa, a1, a1, n);
        if (st) iir_lattice(p->aa_k, p->aa_v, p->aa_stages, s->aa1, a0o, a0o, n);
    }

    biquad_df1(p->biquad2, 1, s->bq2, a1, n);          /* audio_driver.c:2832 */
    if (st) biquad_df1(p->biquad2, 1, s->bq2_1, a0o, n);
    if (p->single_channel)
    {
        /* mcHF (no USE_TWO_CHANNEL_AUDIO, :2870-2885): line out into a_buffer[0], then the
           speaker's software gain on a_buffer[1] (1 at volume <= 16: exact) */
        for (int i = 0; i < n; i++) a0o[i] = a1[i] * p->line_out0_scale;
        for (int i = 0; i < n; i++) a1[i] = a1[i] * p->spkr_scale;
    }
    else
    {
        for (int i = 0; i < n; i++) a1[i] = a1[i] * p->line_out_scale;   /* :2860 (OVI40) */
        if (st) for (int i = 0; i < n; i++) a0o[i] = a0o[i] * p->line_out_scale;
        else for (int i = 0; i < n; i++) a0o[i] = a1[i];                  /* :2868 copy */
    }
    if (beep_on(p, s))
        for (int i = 0; i < n; i++)
        {
            const float t = beep_next(p, s);
            if (!p->single_channel) a0o[i] += t;     /* mcHF: softdds_addSingleTone on a_buffer[1], :2896 */
            a1[i] += t;
        }
    for (int i = 0; i < n; i++)
    {
        out_a1[i] = a1[i];
        if (out_a0) out_a0[i] = a0o[i];
        if (dst) { dst[2 * i] = to_dma(a1[i]); dst[2 * i + 1] = to_dma(a0o[i]); }
    }
}

int uo_rx_process(const uhsdr_rx_plan* p, uo_rx_state* s, const int32_t* iq, int n, float* a1, int32_t* dst)
{
    if (n % BLK) return UHSDR_LENGTH_ERROR;
    for (int off = 0; off < n; off += BLK)
        rx_call(p, s, iq + 2 * off, a1 + off, NULL, dst ? dst + 2 * off : NULL);
    return UHSDR_OK;
}

int uo_rx_process2(const uhsdr_rx_plan* p, uo_rx_state* s, const int32_t* iq, int n, float* a1, float* a0,
                   int32_t* dst)
{
    if (n % BLK) return UHSDR_LENGTH_ERROR;
    for (int off = 0; off < n; off += BLK)
        rx_call(p, s, iq + 2 * off, a1 + off, a0 ? a0 + off : NULL, dst ? dst + 2 * off : NULL);
    return UHSDR_OK;
}

typedef struct
{
    const uhsdr_rx_plan* p;
    uo_rx_state* states;
    const int32_t* iq;
    float* a1;
    float* a0;
    int32_t* dst;
    int c0, c1, n;
} uo_job;

static void* uo_worker(void* arg)
{
    uo_job* j = (uo_job*)arg;
    for (int c = j->c0; c < j->c1; c++)
        uo_rx_process2(j->p, &j->states[c], j->iq + (size_t)c * j->n * 2, j->n, j->a1 + (size_t)c * j->n,
                       j->a0 ? j->a0 + (size_t)c * j->n : NULL, j->dst ? j->dst + (size_t)c * j->n * 2 : NULL);
    return NULL;
}

typedef struct
{
    const uhsdr_rx_plan* p;
    uo_rx_state* states;
    const int32_t* iq;
    float* a1;
    int32_t* dst;
    uint8_t* sig;
    float* en;
    int c0, c1, n, bmax;
} uo_cw_job;

static void* uo_cw_worker(void* arg)
{
    uo_cw_job* j = (uo_cw_job*)arg;
    for (int c = j->c0; c < j->c1; c++)
    {
        uo_rx_state* s = &j->states[c];
        int nb = 0;
        for (int off = 0; off < j->n; off += BLK)
        {
            rx_call(j->p, s, j->iq + ((size_t)c * j->n + off) * 2, j->a1 + (size_t)c * j->n + off, NULL,
                    j->dst ? j->dst + ((size_t)c * j->n + off) * 2 : NULL);
            if (j->sig) j->sig[(size_t)c * (j->n / BLK) + off / BLK] = (uint8_t)s->cw_signal_out;
            if (j->p->cw_enabled && s->cw_blocks_out && j->en && nb < j->bmax) j->en[(size_t)c * j->bmax + nb] = s->cw_energy_out;
            if (j->p->cw_enabled && s->cw_blocks_out) nb++;
        }
    }
    return NULL;
}

int uo_rx_process_batch_cw(const uhsdr_rx_plan* p, uo_rx_state* states, int C, const int32_t* iq, int n,
                           float* a1, int32_t* dst, uint8_t* cw_signal, float* cw_energy, int bmax, int threads)
{
    if (n % BLK) return UHSDR_LENGTH_ERROR;
    if (threads < 1) threads = 1;
    if (threads > C) threads = C;
    if (threads > 256) threads = 256;
    pthread_t tid[256];
    uo_cw_job jobs[256];
    for (int t = 0; t < threads; t++)
    {
        jobs[t] = (uo_cw_job){ p, states, iq, a1, dst, cw_signal, cw_energy, (int)((long)C * t / threads),
                               (int)((long)C * (t + 1) / threads), n, bmax };
        if (threads == 1) uo_cw_worker(&jobs[t]);
        else pthread_create(&tid[t], NULL, uo_cw_worker, &jobs[t]);
    }
    if (threads > 1)
        for (int t = 0; t < threads; t++) pthread_join(tid[t], NULL);
    return UHSDR_OK;
}

int uo_rx_process_batch2(const uhsdr_rx_plan* p, uo_rx_state* states, int C, const int32_t* iq, int n,
                         float* a1, float* a0, int32_t* dst, int threads)
{
    if (n % BLK) return UHSDR_LENGTH_ERROR;
    if (threads < 1) threads = 1;
    if (threads > C) threads = C;
    pthread_t tid[256];
    uo_job jobs[256];
    if (threads > 256) threads = 256;
    for (int t = 0; t < threads; t++)
    {
        jobs[t] = (uo_job){ p, states, iq, a1, a0, dst, (int)((long)C * t / threads), (int)((long)C * (t + 1) / threads), n };
        if (threads == 1) uo_worker(&jobs[t]);
        else pthread_create(&tid[t], NULL, uo_worker, &jobs[t]);
    }
    if (threads > 1)
        for (int t = 0; t < threads; t++) pthread_join(tid[t], NULL);
    return UHSDR_OK;
}

int uo_rx_process_batch(const uhsdr_rx_plan* p, uo_rx_state* states, int C, const int32_t* iq, int n,
                        float* a1, int32_t* dst, int threads)
{
    return uo_rx_process_batch2(p, states, C, iq, n, a1, NULL, dst, threads);
}

/* CPU baseline for bench.py: `threads` persistent workers, worker t pinned
   to the t-th CPU of the process's affinity mask, each running its own contiguous channel slice
   (states and outputs private to the worker) call after call over a pool of `pool` input blocks
   [pool][C][n][2], until `budget_s` seconds have passed.  No thread is created or joined inside
   the timed loop.  Returns the total channel-calls done (sum over workers of channels x calls);
   *elapsed gets the slowest worker's wall time. */
typedef struct
{
    const uhsdr_rx_plan* p;
    uo_rx_state* states;
    const int32_t* iq;
    float* a1;
    int32_t* dst;
    int c0, c1, n, C, pool, cpu;
    double budget;
    pthread_barrier_t* bar;
    long long done;
    double el;
} uo_bench_job;

static double uo_now(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

static void* uo_bench_worker(void* arg)
{
    uo_bench_job* j = (uo_bench_job*)arg;
    if (j->cpu >= 0)
    {
        cpu_set_t set;
        CPU_ZERO(&set);
        CPU_SET(j->cpu, &set);
        pthread_setaffinity_np(pthread_self(), sizeof set, &set);
    }
    const int nc = j->c1 - j->c0;
    pthread_barrier_wait(j->bar);
    const double t0 = uo_now();
    long long calls = 0;
    double el = 0.0;
    do
    {
        const int32_t* blk = j->iq + (size_t)(calls % j->pool) * j->C * j->n * 2;
        for (int c = j->c0; c < j->c1; c++)
            uo_rx_process(j->p, &j->states[c], blk + (size_t)c * j->n * 2, j->n, j->a1 + (size_t)c * j->n,
                          j->dst ? j->dst + (size_t)c * j->n * 2 : NULL);
        ++calls;
        el = uo_now() - t0;
    } while (el < j->budget);
    j->done = calls * nc;
    j->el = el;
    return NULL;
}

long long uo_rx_bench(const uhsdr_rx_plan* p, uo_rx_state* states, int C, const int32_t* iq, int pool, int n,
                      float* a1, int32_t* dst, int threads, int pin, double budget_s, double* elapsed)
{
    if (n % BLK || C < 1 || pool < 1) return -1;
    cpu_set_t allowed;
    int cpus[1024], ncpu = 0;
    if (sched_getaffinity(0, sizeof allowed, &allowed) == 0)
        for (int i = 0; i < CPU_SETSIZE && ncpu < 1024; i++)
            if (CPU_ISSET(i, &allowed)) cpus[ncpu++] = i;
    if (threads < 1) threads = 1;
    if (threads > C) threads = C;
    if (threads > 1024) threads = 1024;
    pthread_t* tid = (pthread_t*)calloc(threads, sizeof(pthread_t));
    uo_bench_job* jobs = (uo_bench_job*)calloc(threads, sizeof(uo_bench_job));
    pthread_barrier_t bar;
    pthread_barrier_init(&bar, NULL, threads);
    for (int t = 0; t < threads; t++)
    {
        jobs[t] = (uo_bench_job){ p, states, iq, a1, dst, (int)((long)C * t / threads), (int)((long)C * (t + 1) / threads),
                                  n, C, pool, (pin && ncpu) ? cpus[t % ncpu] : -1, budget_s, &bar, 0, 0.0 };
        pthread_create(&tid[t], NULL, uo_bench_worker, &jobs[t]);
    }
    long long total = 0;
    double mx = 0.0;
    for (int t = 0; t < threads; t++)
    {
        pthread_join(tid[t], NULL);
        total += jobs[t].done;
        if (jobs[t].el > mx) mx = jobs[t].el;
    }
    pthread_barrier_destroy(&bar);
    free(tid);
    free(jobs);
    if (elapsed) *elapsed = mx;
    return total;
}

/* ================================ transmit ================================ */

size_t uo_tx_state_size(void) { return sizeof(uo_tx_state); }

void uo_tx_state_init(const uhsdr_tx_plan* p, uo_tx_state* s)
{
    (void)p;
    memset(s, 0, sizeof *s);
    s->alc_val = 1;             /* TxProcessor_Init, tx_processor.c:137 */
    s->osc_vi = 0.0f;           /* FreqShift_Approx_Prepare, freq_shift.c:48-49 */
    s->osc_vq = 1.0f;
}

static int32_t to_int32(float f)     /* float -> int32 as x86 cvttss2si (out of range -> INT32_MIN) */
{
    return (f > -2147483904.0f && f < 2147483648.0f) ? (int32_t)f : INT32_MIN;
}

void uo_tx_set_tune(uo_tx_state* states, int C, int tune)
{
    for (int c = 0; c < C; c++)     /* AudioManagement_SetSidetoneForDemodMode: configRunIQ, smooth 0 */
    {
        states[c].tune = tune;
        states[c].tune_acc[0] = states[c].tune_acc[1] = 0;
    }
}

void uo_tx_set_tone_burst(uo_tx_state* states, int C, int active)
{
    for (int c = 0; c < C; c++) states[c].burst = active;
}

/* softdds_nextSampleIndex (softdds.h:37-44) */
static uint32_t dds_next(uint32_t* acc, uint32_t step)
{
    const uint32_t k = (*acc >> 22) % 1024;
    *acc += step;
    return k;
}

/* TxProcessor_IqFinalProcessing (tx_processor.c:282-330) with final gains gi / gq */
static void tx_final(const uhsdr_tx_plan* p, float gi, float gq, float* ib, float* qb, int32_t* iq, int n)
{
    for (int i = 0; i < n; i++) ib[i] = ib[i] * gi;
    for (int i = 0; i < n; i++) qb[i] = qb[i] * gq;
    const float ph = p->phase_balance;                 /* AudioDriver_IQPhaseAdjust, audio_driver.c:1776-1801 */
    if (ph < 0)
        for (int i = 0; i < n; i++) { const float e = ib[i] * ph; qb[i] = qb[i] + e; }
    else if (ph > 0)
        for (int i = 0; i < n; i++) { const float e = qb[i] * ph; ib[i] = ib[i] + e; }
    for (int i = 0; i < n; i++)
    {
        iq[2 * i] = to_int32(ib[i]);
        iq[2 * i + 1] = to_int32(qb[i]);
    }
}

/* one TxProcessor_Run call (voice: SSB, AM, FM; or the USB I/Q source) on BLK frames */
static void tx_call(const uhsdr_tx_plan* p, uo_tx_state* s, const int32_t* audio, int32_t* iq, float* a0)
{
    const int n = BLK;
    float a[BLK], ib[BLK], qb[BLK], valbuf[BLK];
    if (p->digiq && !s->tune)
    {
        /* TX_AUDIO_DIGIQ (tx_processor.c:950-961): the USB frames are the I/Q; the voice chain
           does not run, a_buffer[0] keeps its contents (a0 left unwritten) */
        for (int i = 0; i < n; i++) { ib[i] = audio[2 * i]; qb[i] = audio[2 * i + 1]; }
        tx_final(p, p->digiq_i_gain, p->digiq_q_gain, ib, qb, iq, n);
        if (a0) memcpy(a0, s->a0, sizeof(float) * n);
        return;
    }
    if ((p->am || p->fm) && p->freq_shift_hz == 0)
    {
        /* USB I/Q source under TUNE in AM / FM without frequency translation (the plan admits it
           only with DIGIQ): the AM / FM branch is skipped (tx_processor.c:996-1016), signal_active
           stays false and zeroed I/Q goes through the final stage: zero DAC frames */
        for (int i = 0; i < n; i++) { ib[i] = 0.0f; qb[i] = 0.0f; }
        tx_final(p, p->final_i_gain, p->final_q_gain, ib, qb, iq, n);
        if (a0) memcpy(a0, s->a0, sizeof(float) * n);
        return;
    }
    /* TxProcessor_AudioBufferFill (tx_processor.c:339-405) */
    if (s->tune)
    {
        /* softdds_runIQ(a, a, n) (softdds.c:152-163): genIQSingleTone / genIQTwoTone write I then Q
           to the same sample, so the quadrature value remains */
        for (int i = 0; i < n; i++)
        {
            const uint32_t k0 = dds_next(&s->tune_acc[0], p->tune_step[0]);
            if (s->tune == 1)
                a[i] = p->dds_table[(k0 + 768) % 1024];
            else
            {
                const uint32_t k1 = dds_next(&s->tune_acc[1], p->tune_step[1]);
                a[i] = ((int32_t)p->dds_table[(k0 + 768) % 1024] + (int32_t)p->dds_table[(k1 + 768) % 1024]) / 2;
            }
        }
    }
    else
    {
        for (int i = 0; i < n; i++) a[i] = (p->audio_source == UHSDR_TX_AUDIO_LINEIN_R) ? audio[2 * i + 1] : audio[2 * i];
        if (p->apply_in_gain)
            for (int i = 0; i < n; i++) a[i] = a[i] * p->in_gain;
        /* TxProcessor_FilterAudio (:416-429), skipped in TUNE (:444) */
        if (p->run_lattice) iir_lattice(p->lat_k, p->lat_v, p->lat_stages, s->lat, a, a, n);
        if (p->run_biquad) biquad_df1(p->biquad, 3, s->bq, a, n);
    }
    /* TxProcessor_VoiceCompressor (:173-242) */
    if (p->comp_on)
    {
        if (!s->tune)
            for (int i = 0; i < n; i++) a[i] = a[i] * p->postfilt_gain;
        for (int i = 0; i < n; i++)
        {
            const float alc_var = fabsf(a[i] * s->alc_val) / 30000 - 1.0;        /* ALC_KNEE */
            if (alc_var < 0)
            {
                s->alc_val -= s->alc_val * p->alc_decay * alc_var;
            }
            else
            {
                s->alc_val -= s->alc_val * 0.1 * alc_var;                        /* ALC_ATTACK */
                if (s->alc_val < 0.001) s->alc_val = 0.001;                      /* ALC_VAL_MIN */
            }
            if (s->alc_val > 1) s->alc_val = 1;                                 /* ALC_VAL_MAX */
            valbuf[i] = (s->alc_val * p->alc_gain_scaling);
        }
        s->delay_in += n;
        int out = s->delay_in + n;
        s->delay_in %= UHSDR_TX_DELAY;
        out %= UHSDR_TX_DELAY;
        memcpy(&s->delay[s->delay_in], a, sizeof(float) * n);
        memcpy(a, &s->delay[out], sizeof(float) * n);
        for (int i = 0; i < n; i++) a[i] = a[i] * valbuf[i];
    }
    memcpy(s->a0, a, sizeof(float) * n);
    if (a0) memcpy(a0, a, sizeof(float) * n);
    if (p->fm)
    {
        /* TxProcessor_FM (:534-588): differentiating pre-emphasis, sub-audible tone, NCO */
        float a1[BLK];
        for (int i = 0; i < n; i++)
        {
            const float x = a[i];
            s->fm_hpf_b = 0.05 * (s->fm_hpf_b + x - s->fm_hpf_a);         /* FM_TX_HPF_ALPHA */
            s->fm_hpf_a = x;
            a1[i] = s->fm_hpf_b;
        }
        if (p->fm_sub_on && !s->burst)                                     /* softdds_addSingleTone */
            for (int i = 0; i < n; i++)
            {
                const uint32_t k = (s->fm_sub_acc >> 22) % 1024;
                s->fm_sub_acc += p->fm_sub_step;
                a1[i] += (float)p->dds_table[k] * p->fm_sub_scale;
            }
        if (s->burst)                                                      /* tone burst, :561-564 */
            for (int i = 0; i < n; i++)
                a1[i] += (float)p->dds_table[dds_next(&s->burst_acc, p->tone_burst_step)] * p->tone_burst_scale;
        float* ip = p->fm_swap ? qb : ib;
        float* qp = p->fm_swap ? ib : qb;
        for (int i = 0; i < n; i++)
        {
            /* uint32 += float: the sum in float, back through a 64-bit truncation as x86 does */
            const float sum = (float)s->fm_accum + (p->fm_word + (a1[i] * 16 * p->fm_mod_mult));
            s->fm_accum = (uint32_t)(int64_t)sum;
            s->fm_accum %= 65536;
            const uint32_t idx = s->fm_accum >> 6;
            ip[i] = p->dds_table[idx];
            qp[i] = p->dds_table[(idx + 768) % 1024];
        }
    }
    else
    {
    /* TxProcessor_SSB (:467-490) / TxProcessor_AM (:734-800): Hilbert pair, [both sidebands +
       carrier,] then FreqShift */
    fir(p->hilbert_i, UHSDR_TX_HILBERT_TAPS, s->hil_i, a, ib, n);
    fir(p->hilbert_q, UHSDR_TX_HILBERT_TAPS, s->hil_q, a, qb, n);
    if (p->am)
        for (int i = 0; i < n; i++)
        {
            const float i_am = (ib[i] - qb[i]) + (2 * 5100);          /* AM_CARRIER_LEVEL, audio_driver.h:429 */
            const float q_am = (qb[i] - ib[i]) - (2 * 5100);
            ib[i] = i_am;
            qb[i] = q_am;
        }
    if (p->freq_shift_hz != 0)
    {
        float* ip = p->shift_up ? ib : qb;
        float* qp = p->shift_up ? qb : ib;
        if (p->shift_kind == 1)
        {
            for (int i = 0; i < n; i += 4)
            {
                float h1 = qp[i + 1], h2 = -ip[i + 1];
                ip[i + 1] = h1; qp[i + 1] = h2;
                h1 = -ip[i + 2]; h2 = -qp[i + 2];
                ip[i + 2] = h1; qp[i + 2] = h2;
                h1 = -qp[i + 3]; h2 = ip[i + 3];
                ip[i + 3] = h1; qp[i + 3] = h2;
            }
        }
        else
        {
            for (int i = 0; i < n; i++)
            {
                const float oq = (s->osc_vq * p->osc_cos) - (s->osc_vi * p->osc_sin);
                const float oi = (s->osc_vi * p->osc_cos) + (s->osc_vq * p->osc_sin);
                const float qt = qp[i], it = ip[i];
                qp[i] = (qt * oq) - (it * oi);
                ip[i] = (it * oq) + (qt * oi);
                s->osc_vq = oq;
                s->osc_vi = oi;
            }
            const float g = (3 - ((s->osc_vq * s->osc_vq) + (s->osc_vi * s->osc_vi))) / 2;
            s->osc_vq = g * s->osc_vq;
            s->osc_vi = g * s->osc_vi;
        }
    }
    }
    tx_final(p, p->final_i_gain, p->final_q_gain, ib, qb, iq, n);
}

typedef struct
{
    const uhsdr_tx_plan* p;
    uo_tx_state* states;
    const int32_t* audio;
    int32_t* iq;
    float* a0;
    int c0, c1, n;
} uo_tx_job;

static void* uo_tx_worker(void* arg)
{
    uo_tx_job* j = (uo_tx_job*)arg;
    for (int c = j->c0; c < j->c1; c++)
        for (int off = 0; off < j->n; off += BLK)
            tx_call(j->p, &j->states[c], j->audio + ((size_t)c * j->n + off) * 2, j->iq + ((size_t)c * j->n + off) * 2,
                    j->a0 ? j->a0 + (size_t)c * j->n + off : NULL);
    return NULL;
}

int uo_tx_process_batch(const uhsdr_tx_plan* p, uo_tx_state* states, int C, const int32_t* audio, int n,
                        int32_t* iq, float* a0, int threads)
{
    if (n % BLK) return UHSDR_LENGTH_ERROR;
    if (threads < 1) threads = 1;
    if (threads > C) threads = C;
    if (threads > 256) threads = 256;
    pthread_t tid[256];
    uo_tx_job jobs[256];
    for (int t = 0; t < threads; t++)
    {
        jobs[t] = (uo_tx_job){ p, states, audio, iq, a0, (int)((long)C * t / threads), (int)((long)C * (t + 1) / threads), n };
        if (threads == 1) uo_tx_worker(&jobs[t]);
        else pthread_create(&tid[t], NULL, uo_tx_worker, &jobs[t]);
    }
    if (threads > 1)
        for (int t = 0; t < threads; t++) pthread_join(tid[t], NULL);
    return UHSDR_OK;
}

/* ============================= spectrum display ============================= */

size_t uo_spec_state_size(void) { return sizeof(uo_spec_state); }

void uo_spec_state_init(const uhsdr_spectrum_plan* p, uo_spec_state* s)
{
    (void)p;
    memset(s, 0, sizeof *s);
    s->osc_vq = 1.0f;          /* FreqShift_Approx oscillator starts at {I=0, Q=1} (freq_shift.c:48-49) */
}

/* FreqShift (freq_shift.c:275-334) on one 32-frame call, as rx_call */
static void spec_freq_shift(const uhsdr_spectrum_plan* p, uo_spec_state* s, float* ib, float* qb, int n)
{
    float* ip = p->shift_up ? ib : qb;
    float* qp = p->shift_up ? qb : ib;
    if (p->shift_kind == 1)
    {
        for (int i = 0; i < n; i += 4)   /* FreqShift_QuarterFs :219-262 */
        {
            float h1 = qp[i + 1], h2 = -ip[i + 1];
            ip[i + 1] = h1; qp[i + 1] = h2;
            h1 = -ip[i + 2]; h2 = -qp[i + 2];
            ip[i + 2] = h1; qp[i + 2] = h2;
            h1 = -qp[i + 3]; h2 = ip[i + 3];
            ip[i + 3] = h1; qp[i + 3] = h2;
        }
    }
    else
    {
        for (int i = 0; i < n; i++)      /* FreqShift_Approx :57-101 */
        {
            const float oq = (s->osc_vq * p->osc_cos) - (s->osc_vi * p->osc_sin);
            const float oi = (s->osc_vi * p->osc_cos) + (s->osc_vq * p->osc_sin);
            const float qt = qp[i], it = ip[i];
            qp[i] = (qt * oq) - (it * oi);
            ip[i] = (it * oq) + (qt * oi);
            s->osc_vq = oq;
            s->osc_vi = oi;
        }
        const float g = (3 - ((s->osc_vq * s->osc_vq) + (s->osc_vi * s->osc_vi))) / 2;
        s->osc_vq = g * s->osc_vq;
        s->osc_vi = g * s->osc_vi;
    }
}

/* 8-point DFT core of arm_radix8_butterfly_f32 (CMSIS TransformFunctions/arm_cfft_radix8_f32.c:
   130-383) on the complex values at x[2*(base + k*stride)], k = 0..7.  Both of the reference's
   loops (the twiddle-free first group :149-221 and the twiddled groups :228-372) form the same
   eight intermediate values X_k with the same operation sequence; the twiddled groups then
   rotate X_k (k >= 1) by twiddle[k * tstep] as (c*re + s*im, c*im - s*re).  tstep 0: no rotation. */
static void cfft_radix8(float* x, int base, int stride, const float* tw, int tstep)
{
    const float C81 = 0.70710678118f;
    float re[8], im[8];
    for (int k = 0; k < 8; k++)
    {
        re[k] = x[2 * (base + k * stride)];
        im[k] = x[2 * (base + k * stride) + 1];
    }
    float sr[4], dr[4], si[4], di[4];
    for (int k = 0; k < 4; k++)
    {
        sr[k] = re[k] + re[k + 4];
        dr[k] = re[k] - re[k + 4];
        si[k] = im[k] + im[k + 4];
        di[k] = im[k] - im[k + 4];
    }
    float Xr[8], Xi[8];
    /* even outputs */
    const float a = sr[0] - sr[2], b = sr[0] + sr[2], cc = sr[1] - sr[3], d = sr[1] + sr[3];
    const float ai = si[0] - si[2], bi = si[0] + si[2], ci = si[1] - si[3], dd = si[1] + si[3];
    Xr[0] = b + d;   Xi[0] = bi + dd;
    Xr[4] = b - d;   Xi[4] = bi - dd;
    Xr[2] = a + ci;  Xi[2] = ai - cc;
    Xr[6] = a - ci;  Xi[6] = ai + cc;
    /* odd outputs */
    const float u = (dr[1] - dr[3]) * C81, v = (dr[1] + dr[3]) * C81;
    const float ui = (di[1] - di[3]) * C81, vi = (di[1] + di[3]) * C81;
    const float e0 = dr[0] - u, e1 = dr[0] + u, f0 = dr[2] - v, f1 = dr[2] + v;
    const float g0 = di[0] - ui, g1 = di[0] + ui, h0 = di[2] - vi, h1 = di[2] + vi;
    Xr[1] = e1 + h1; Xi[1] = g1 - f1;
    Xr[7] = e1 - h1; Xi[7] = g1 + f1;
    Xr[5] = e0 + h0; Xi[5] = g0 - f0;
    Xr[3] = e0 - h0; Xi[3] = g0 + f0;
    for (int k = 0; k < 8; k++)
    {
        float yr = Xr[k], yi = Xi[k];
        if (tstep && k)
        {
            const float c = tw[2 * k * tstep], s = tw[2 * k * tstep + 1];
            const float p1 = c * Xr[k], p2 = s * Xi[k], p3 = c * Xi[k], p4 = s * Xr[k];
            yr = p1 + p2;
            yi = p3 - p4;
        }
        x[2 * (base + k * stride)] = yr;
        x[2 * (base + k * stride) + 1] = yi;
    }
}

/* arm_radix8_butterfly_f32 stage loop on n points at x (complex), twiddle modifier tm */
static void cfft_radix8_stages(float* x, int n, const float* tw, int tm)
{
    for (int span = n; span >= 8; span >>= 3, tm <<= 3)
    {
        const int stride = span >> 3;
        for (int j = 0; j < stride; j++)
            for (int g = j; g < n; g += span)
                cfft_radix8(x, g, stride, tw, j * tm);
    }
}

/* complex rotation forms of the first stages */
static void rot_fwd(float* y, float xr, float xi, float c, float s)   /* (m0 + m1, m2 - m3) */
{
    const float m0 = xr * c, m1 = xi * s, m2 = xi * c, m3 = xr * s;
    y[0] = m0 + m1;
    y[1] = m2 - m3;
}

/* arm_cfft_radix8by2_f32 (arm_cfft_f32.c:207-317): radix-2 split of n = 2H points */
static void cfft_by2(float* x, int n, const float* tw)
{
    const int H = n / 2, Q = n / 4;
    for (int a = 0; a < Q; a++)
    {
        float* p1 = x + 2 * a;
        float* p3 = x + 2 * (a + Q);
        float* p2 = x + 2 * (a + H);
        float* p4 = x + 2 * (a + H + Q);
        const float t2r = p1[0] - p2[0], t2i = p1[1] - p2[1];
        const float t4r = p4[0] - p3[0], t4i = p4[1] - p3[1];
        p1[0] = p1[0] + p2[0];
        p1[1] = p1[1] + p2[1];
        p3[0] = p3[0] + p4[0];
        p3[1] = p3[1] + p4[1];
        const float c = tw[2 * a], s = tw[2 * a + 1];
        rot_fwd(p2, t2r, t2i, c, s);
        /* the mirrored column (:283-290): (t4r*s - t4i*c, t4i*s + t4r*c) */
        const float m0 = t4r * s, m1 = t4i * c, m2 = t4i * s, m3 = t4r * c;
        p4[0] = m0 - m1;
        p4[1] = m2 + m3;
    }
    cfft_radix8_stages(x, H, tw, 2);
    cfft_radix8_stages(x + 2 * H, H, tw, 2);
}

/* arm_cfft_radix8by4_f32 (arm_cfft_f32.c:319-557): radix-4 split of n = 4Q points */
static void cfft_by4(float* x, int n, const float* tw)
{
    const int Q = n / 4;
    float* c1 = x;
    float* c2 = x + 2 * Q;
    float* c3 = x + 4 * Q;
    float* c4 = x + 6 * Q;
    /* top half (t = 0 .. Q/2; t = 0 untwiddled, t = Q/2 is the reference's MIDDLE block) */
    for (int t = 0; t <= Q / 2; t++)
    {
        float* p1 = c1 + 2 * t;
        float* p2 = c2 + 2 * t;
        float* p3 = c3 + 2 * t;
        float* p4 = c4 + 2 * t;
        const float s13r = p1[0] + p3[0], d13r = p1[0] - p3[0];
        const float s13i = p1[1] + p3[1], d13i = p1[1] - p3[1];
        const float t2r = d13r + p2[1] - p4[1], t2i = d13i - p2[0] + p4[0];
        const float t3r = s13r - p2[0] - p4[0], t3i = s13i - p2[1] - p4[1];
        const float t4r = d13r - p2[1] + p4[1], t4i = d13i + p2[0] - p4[0];
        p1[0] = s13r + p2[0] + p4[0];
        p1[1] = s13i + p2[1] + p4[1];
        if (t == 0)
        {
            p2[0] = t2r; p2[1] = t2i;
            p3[0] = t3r; p3[1] = t3i;
            p4[0] = t4r; p4[1] = t4i;
            continue;
        }
        rot_fwd(p2, t2r, t2i, tw[2 * t], tw[2 * t + 1]);
        rot_fwd(p3, t3r, t3i, tw[4 * t], tw[4 * t + 1]);
        rot_fwd(p4, t4r, t4i, tw[6 * t], tw[6 * t + 1]);
    }
    /* bottom half (b = Q - t, t = 1 .. Q/2 - 1) with the mirrored twiddles of t */
    for (int t = 1; t < Q / 2; t++)
    {
        const int b = Q - t;
        float* p1 = c1 + 2 * b;
        float* p2 = c2 + 2 * b;
        float* p3 = c3 + 2 * b;
        float* p4 = c4 + 2 * b;
        const float s13r = p1[0] + p3[0], d13r = p1[0] - p3[0];
        const float s13i = p1[1] + p3[1], d13i = p1[1] - p3[1];
        const float u2r = p2[1] - p4[1] + d13r;
        const float u2i = p1[1] - p3[1] - p2[0] + p4[0];
        const float u3r = s13r - p2[0] - p4[0];
        const float u3i = s13i - p2[1] - p4[1];
        const float u4r = p2[1] - p4[1] - d13r;
        const float u4i = p4[0] - p2[0] - d13i;
        p1[1] = s13i + p2[1] + p4[1];
        p1[0] = s13r + p2[0] + p4[0];
        {
            const float c = tw[2 * t], s = tw[2 * t + 1];
            const float m0 = u2i * s, m1 = u2r * c, m2 = u2r * s, m3 = u2i * c;
            p2[1] = m0 - m1;
            p2[0] = m2 + m3;
        }
        {
            const float c = tw[4 * t], s = tw[4 * t + 1];
            const float m0 = -u3i * c, m1 = u3r * s, m2 = u3r * c, m3 = u3i * s;
            p3[1] = m0 - m1;
            p3[0] = m3 - m2;
        }
        {
            const float c = tw[6 * t], s = tw[6 * t + 1];
            const float m0 = u4i * s, m1 = u4r * c, m2 = u4r * s, m3 = u4i * c;
            p4[1] = m0 - m1;
            p4[0] = m2 + m3;
        }
    }
    for (int k = 0; k < 4; k++) cfft_radix8_stages(x + 2 * k * Q, Q, tw, 4);
}

void uo_cfft(const uhsdr_spectrum_plan* p, float* x)
{
    const int n = p->fft_len;
    switch (n)             /* arm_cfft_f32.c:594-611 */
    {
    case 1024: cfft_by2(x, n, p->twiddle); break;
    case 256: cfft_by4(x, n, p->twiddle); break;
    case 512: cfft_radix8_stages(x, n, p->twiddle, 1); break;
    default: return;
    }
    /* arm_bitreversal_32 (arm_bitreversal2.S:136-180): swap the complex values at the byte
       offsets of each table pair */
    uint32_t* w = (uint32_t*)x;
    for (int k = 0; k + 1 < p->bitrev_len; k += 2)
    {
        const int a = p->bitrev[k] >> 2, b = p->bitrev[k + 1] >> 2;
        uint32_t t = w[a]; w[a] = w[b]; w[b] = t;
        t = w[a + 1]; w[a + 1] = w[b + 1]; w[b + 1] = t;
    }
}

/* one display frame from the full ring (ui_spectrum.c:1362-1446) */
static void spec_frame(const uhsdr_spectrum_plan* p, uo_spec_state* s, float* mag, float* avg)
{
    const int L = p->fft_len;
    float x[2 * UHSDR_SPECTRUM_MAX_LEN];
    for (int i = 0; i < 2 * L; i++)
        x[i] = p->window_formula ? 0.5f * (p->window[i] * s->frame[i]) : s->frame[i] * p->window[i];
    uo_cfft(p, x);
    const float f = p->filt_factor;
    for (int k = 0; k < L; k++)
    {
        const float re = x[2 * k], im = x[2 * k + 1];
        const float m = sqrtf((re * re) + (im * im));             /* arm_cmplx_mag_f32 */
        float a = s->avg[k];
        const float old = a * f;                                  /* arm_scale_f32 */
        a = a - old;                                              /* arm_sub_f32 */
        const float add = m * f;
        a = add + a;                                              /* arm_add_f32 */
        if (a < 1) a = 1;
        s->avg[k] = a;
        mag[k] = m;
        avg[k] = a;
    }
}

/* producer: convert + I/Q correction per 32-frame call (as rx_call), then into the ring
   (AudioDriver_SpectrumCopyIqBuffers, audio_driver.c:1811-1826: Q first, then I) */
static int spec_channel(const uhsdr_spectrum_plan* p, uo_spec_state* s, const int32_t* iq, int n,
                        float* mag, float* avg)
{
    const int L = p->fft_len;
    int frames = 0;
    for (int off = 0; off < n; off += BLK)
    {
        float ib[BLK], qb[BLK];
        for (int i = 0; i < BLK; i++) { ib[i] = iq[2 * (off + i)]; qb[i] = iq[2 * (off + i) + 1]; }
        for (int i = 0; i < BLK; i++) ib[i] = ib[i] * IQ_BIT_SCALE_DOWN;
        for (int i = 0; i < BLK; i++) qb[i] = qb[i] * IQ_BIT_SCALE_DOWN;
        if (!p->iq_auto_correction)
        {
            for (int i = 0; i < BLK; i++) ib[i] = ib[i] * p->iq_gain_i;
            for (int i = 0; i < BLK; i++) qb[i] = qb[i] * p->iq_gain_q;
            const float ph = p->iq_phase_balance;
            if (ph < 0)
                for (int i = 0; i < BLK; i++) { const float e = ib[i] * ph; qb[i] = qb[i] + e; }
            else if (ph > 0)
                for (int i = 0; i < BLK; i++) { const float e = qb[i] * ph; ib[i] = ib[i] + e; }
        }
        else
        {
            float t1 = 0.0f, t2 = 0.0f, t3 = 0.0f;
            for (int i = 0; i < BLK; i++)
            {
                t1 += sign_new(ib[i]) * qb[i];
                t2 += sign_new(ib[i]) * ib[i];
                t3 += sign_new(qb[i]) * qb[i];
            }
            t1 = -0.003 * (t1 / BLK) + 0.997 * s->teta1_old;
            t2 = 0.003 * (t2 / BLK) + 0.997 * s->teta2_old;
            t3 = 0.003 * (t3 / BLK) + 0.997 * s->teta3_old;
            const float M_c1 = (t2 != 0.0) ? t1 / t2 : 0.0;
            float help = (t2 * t2);
            if (help > 0.0) help = (t3 * t3 - t1 * t1) / help;
            const float M_c2 = (help > 0.0) ? sqrtf(help) : 1.0;
            s->teta1_old = t1;
            s->teta2_old = t2;
            s->teta3_old = t3;
            for (int i = 0; i < BLK; i++) qb[i] += M_c1 * ib[i];
            for (int i = 0; i < BLK; i++) ib[i] = ib[i] * M_c2;
        }
        int nout = BLK;
        if (p->magnify > 0)
        {
            /* AudioDriver_SpectrumZoomProcessSamples (audio_driver.c:1860-1909), after FreqShift
               (:2694-2705): biquad low-pass on I and Q, decimate by 2^magnify, BLK / 2^magnify
               samples into the ring */
            if (p->freq_shift_hz != 0) spec_freq_shift(p, s, ib, qb, BLK);
            biquad_df1(p->zoom_biquad, 4, s->zbq_i, ib, BLK);
            biquad_df1(p->zoom_biquad, 4, s->zbq_q, qb, BLK);
            const int M = p->zoom_decimation;
            fir_decimate(p->zoom_fir, p->zoom_taps, M, s->zdec_i, ib, ib, BLK);
            fir_decimate(p->zoom_fir, p->zoom_taps, M, s->zdec_q, qb, qb, BLK);
            nout = BLK / M;
        }
        for (int i = 0; i < nout; i++)
        {
            s->frame[2 * s->fill] = qb[i];
            s->frame[2 * s->fill + 1] = ib[i];
            if (++s->fill == L)
            {
                spec_frame(p, s, mag + (size_t)frames * L, avg + (size_t)frames * L);
                frames++;
                s->fill = 0;
            }
        }
    }
    return frames;
}

typedef struct
{
    const uhsdr_spectrum_plan* p;
    uo_spec_state* states;
    const int32_t* iq;
    float *mag, *avg;
    int c0, c1, n, fmax, frames;
} uo_spec_job;

static void* uo_spec_worker(void* arg)
{
    uo_spec_job* j = (uo_spec_job*)arg;
    const size_t L = j->p->fft_len;
    for (int c = j->c0; c < j->c1; c++)
        j->frames = spec_channel(j->p, &j->states[c], j->iq + (size_t)c * j->n * 2, j->n,
                                 j->mag + (size_t)c * j->fmax * L, j->avg + (size_t)c * j->fmax * L);
    return NULL;
}

int uo_spec_process_batch(const uhsdr_spectrum_plan* p, uo_spec_state* states, int C, const int32_t* iq, int n,
                          float* mag, float* avg, int threads)
{
    const int L = p->fft_len;
    const int nd = n / (p->magnify > 0 ? p->zoom_decimation : 1);     /* ring samples per call */
    if (n <= 0 || n % BLK || !(L == 256 || L == 512 || L == 1024) || (nd % L && L % nd)) return UHSDR_LENGTH_ERROR;
    const int fmax = nd >= L ? nd / L : 1;
    if (threads < 1) threads = 1;
    if (threads > C) threads = C;
    if (threads > 256) threads = 256;
    pthread_t tid[256];
    uo_spec_job jobs[256];
    for (int t = 0; t < threads; t++)
    {
        jobs[t] = (uo_spec_job){ p, states, iq, mag, avg, (int)((long)C * t / threads),
                                 (int)((long)C * (t + 1) / threads), n, fmax, 0 };
        if (threads == 1) uo_spec_worker(&jobs[t]);
        else pthread_create(&tid[t], NULL, uo_spec_worker, &jobs[t]);
    }
    if (threads > 1)
        for (int t = 0; t < threads; t++) pthread_join(tid[t], NULL);
    return jobs[0].frames;
}

/* ---- batched arm_fir_f32 (CMSIS FilteringFunctions/arm_fir_f32.c:482-560): per channel the
   window [T-1 carried samples | block], y[n] = sum_{k<T} c[k] * w[n + k] accumulated from +0.0f
   in tap order, separate multiply and add; the carried samples become the window's last T-1.
   The checker for uhsdr_fir_* (C5's synthetic long FIR). */
void uo_fir_batch(const float* c, int T, float* hist, int C, const float* x, int n, float* y)
{
    float* w = (float*)malloc(sizeof(float) * (size_t)(T - 1 + n));
    for (int ch = 0; ch < C; ++ch)
    {
        float* h = hist + (size_t)ch * (T - 1);
        memcpy(w, h, sizeof(float) * (size_t)(T - 1));
        memcpy(w + T - 1, x + (size_t)ch * n, sizeof(float) * (size_t)n);
        for (int i = 0; i < n; ++i)
        {
            float acc = 0.0f;
            for (int k = 0; k < T; ++k) acc += w[i + k] * c[k];
            y[(size_t)ch * n + i] = acc;
        }
        memcpy(h, w + n, sizeof(float) * (size_t)(T - 1));
    }
    free(w);
}
