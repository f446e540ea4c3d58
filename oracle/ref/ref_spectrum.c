/*
 * ORACLE TEST INFRASTRUCTURE -- the spectrum display consumer around the reference's own
 * CMSIS-DSP code, for the x86 reference build (oracle/ref/Makefile).
 *
 * Producer: the firmware itself.  AudioDriver_SpectrumNoZoomProcessSamples
 * (drivers/audio/audio_driver.c:1838-1851, via :2691) writes the I/Q-corrected samples into
 * sd.FFT_RingBuffer as interleaved [Q, I] while uhsdr_ref runs the RX chain; this file only
 * snapshots that ring the way UiSpectrum_RedrawSpectrum state 0 does (ui_spectrum.c:1362-1367).
 *
 * Consumer: ui_spectrum.c does not assemble on x86 (__DSB ARM asm), so its
 * few lines of glue are restated here around the reference's compiled functions:
 *   window      ui_spectrum.c:402-414 (Hann; tables extracted verbatim by extract_hann.py,
 *               formula branch with CMSIS arm_cos_f32 for 2048 floats, where no table exists)
 *   CFFT        arm_cfft_f32 (CMSIS TransformFunctions/arm_cfft_f32.c:574-632), forward: its
 *               length switch is restated and the reference's radix8by2 / radix8by4 /
 *               arm_radix8_butterfly_f32 are called directly.  The final bit reversal of
 *               arm_cfft_f32 is ARM assembly only (arm_bitreversal2.S:136-180); its semantics
 *               -- swap the 8-byte complex at byte offsets table[2k], table[2k+1] -- are
 *               restated in bitreverse() below from that listing.  arm_cfft_f32 itself is
 *               dropped from the link (-ffunction-sections / --gc-sections), so no stand-in
 *               for the assembly symbol exists in this build.
 *   magnitude   arm_cmplx_mag_f32 (reference)
 *   averaging   ui_spectrum.c:1432-1446 with the reference's arm_scale/sub/add_f32
 */
#include <stdio.h>
#include <string.h>
#include "arm_math.h"
#include "arm_const_structs.h"
#include "ui_spectrum.h"

extern SpectrumDisplay sd;
extern const float oracle_von_Hann_512[512];
extern const float oracle_von_Hann_1024[1024];

/* CMSIS arm_cfft_f32.c:207,319 and arm_cfft_radix8_f32.c:130 (exported, not in arm_math.h) */
void arm_cfft_radix8by2_f32(arm_cfft_instance_f32* S, float32_t* p1);
void arm_cfft_radix8by4_f32(arm_cfft_instance_f32* S, float32_t* p1);
void arm_radix8_butterfly_f32(float32_t* pSrc, uint16_t fftLen, const float32_t* pCoef, uint16_t twidCoefModifier);

static const arm_cfft_instance_f32* instance(int L)
{
    switch (L)          /* CMSIS arm_const_structs.c: every length arm_cfft_f32 dispatches */
    {
    case 16: return &arm_cfft_sR_f32_len16;
    case 32: return &arm_cfft_sR_f32_len32;
    case 64: return &arm_cfft_sR_f32_len64;
    case 128: return &arm_cfft_sR_f32_len128;
    case 256: return &arm_cfft_sR_f32_len256;
    case 512: return &arm_cfft_sR_f32_len512;
    case 1024: return &arm_cfft_sR_f32_len1024;
    case 2048: return &arm_cfft_sR_f32_len2048;
    case 4096: return &arm_cfft_sR_f32_len4096;
    default: return NULL;
    }
}
const arm_cfft_instance_f32* ref_cfft_instance(int L) { return instance(L); }

/* ring length in floats: the firmware's FFT_RingBuffer holds FFT_IQ_BUFF_LEN = 1024 floats
   (audio_driver.h:62-67 with USE_FFT_1024), so a 1024-point frame is assembled from two
   consecutive 512-point snapshots of the same producer */
int ref_spec_ring_len(int L) { return L >= 512 ? 1024 : 2 * L; }

void oracle_ref_spec_magnify(int m);
const float* oracle_ref_zoom_biquad(int m);
const arm_fir_decimate_instance_f32* oracle_ref_zoom_decim(void);

void ref_spec_setup(int L, int magnify)
{
    sd.fft_iq_len = (uint16_t)ref_spec_ring_len(L);
    sd.samp_ptr = 0;
    sd.reading_ringbuffer = false;
    oracle_ref_spec_magnify(magnify);       /* 0: no zoom (the no-zoom producer fills the ring) */
}

/* UiSpectrum_RedrawSpectrum state 0 copy (ui_spectrum.c:1362-1367) */
void ref_spec_snapshot(float* out)
{
    sd.reading_ringbuffer = true;
    arm_copy_f32(&sd.FFT_RingBuffer[sd.samp_ptr], &out[0], sd.fft_iq_len - sd.samp_ptr);
    arm_copy_f32(&sd.FFT_RingBuffer[0], &out[sd.fft_iq_len - sd.samp_ptr], sd.samp_ptr);
    sd.reading_ringbuffer = false;
}

/* arm_bitreversal_32 (arm_bitreversal2.S:136-180, CM7 branch): (bitRevLen + 1) >> 2
   iterations of two swaps each, table entries are byte offsets of 8-byte complex values */
static void bitreverse(float* p, uint16_t len, const uint16_t* tab)
{
    uint32_t* w = (uint32_t*)p;
    for (uint32_t it = 0; it < (uint32_t)((len + 1) >> 2); ++it)
        for (int s = 0; s < 2; ++s)
        {
            const uint32_t a = tab[4 * it + 2 * s] >> 2, b = tab[4 * it + 2 * s + 1] >> 2;
            uint32_t t = w[a]; w[a] = w[b]; w[b] = t;
            t = w[a + 1]; w[a + 1] = w[b + 1]; w[b + 1] = t;
        }
}

/* the length switch and optional bit reversal of arm_cfft_f32 (arm_cfft_f32.c:594-614) */
void ref_cfft_stages(int L, float* p, int bitrev)
{
    const arm_cfft_instance_f32* S = instance(L);
    switch (L)
    {
    case 16: case 128: case 1024: arm_cfft_radix8by2_f32((arm_cfft_instance_f32*)S, p); break;
    case 32: case 256: case 2048: arm_cfft_radix8by4_f32((arm_cfft_instance_f32*)S, p); break;
    case 64: case 512: case 4096: arm_radix8_butterfly_f32(p, L, (float32_t*)S->pTwiddle, 1); break;
    }
    if (bitrev) bitreverse(p, S->bitRevLength, S->pBitRevTable);
}

/* arm_cfft_f32(S, p1, 0, 1) for L in {256, 512, 1024} */
void ref_cfft(int L, float* p) { ref_cfft_stages(L, p, 1); }

/* UiSpectrum_FFTWindowFunction(FFT_WINDOW_HANN) on fft_iq_len = 2L floats */
void ref_spec_window(int L, float* x)
{
    const int n = 2 * L;
    if (n == 512 || n == 1024)
    {
        const float32_t* W = n == 512 ? oracle_von_Hann_512 : oracle_von_Hann_1024;
        for (int i = 0; i < n; i++) x[i] *= W[i];
    }
    else
    {
        const uint16_t fft_iq_len = (uint16_t)n;
        for (int i = 0; i < fft_iq_len; i++)
            x[i] = 0.5 * (float32_t)((1 - (arm_cos_f32(PI * 2 * (float32_t)i / (float32_t)(fft_iq_len - 1)))) * x[i]);
    }
}

/* one display frame: window -> CFFT -> magnitude -> IIR average (ui_spectrum.c:1362-1446) */
void ref_spec_frame(int L, int spectrum_filter, const float* ring, float* mag, float* avg)
{
    float buf[2048], tmp[1024];
    arm_copy_f32((float32_t*)ring, buf, 2 * L);
    ref_spec_window(L, buf);
    ref_cfft(L, buf);
    arm_cmplx_mag_f32(buf, mag, L);
    const float32_t filt_factor = 1 / (float)spectrum_filter;
    arm_scale_f32(avg, filt_factor, tmp, L);
    arm_sub_f32(avg, tmp, avg, L);
    arm_scale_f32(mag, filt_factor, tmp, L);
    arm_add_f32(tmp, avg, avg, L);
    for (int i = 0; i < L; i++)
        if (avg[i] < 1) avg[i] = 1;
}

static uint32_t fb(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

/* dump=spectrum: the tables the device needs, as raw bits (JSON) */
void ref_spec_dump(void)
{
    printf("{");
    const int lens[3] = { 256, 512, 1024 };
    for (int k = 0; k < 3; ++k)
    {
        const arm_cfft_instance_f32* S = instance(lens[k]);
        printf("\"twiddle_%d\": [", lens[k]);
        for (int i = 0; i < 2 * lens[k]; ++i) printf("%s%u", i ? "," : "", fb(S->pTwiddle[i]));
        printf("], \"bitrev_%d\": [", lens[k]);
        for (int i = 0; i < S->bitRevLength; ++i) printf("%s%u", i ? "," : "", S->pBitRevTable[i]);
        printf("], ");
    }
    printf("\"hann_512\": [");
    for (int i = 0; i < 512; ++i) printf("%s%u", i ? "," : "", fb(oracle_von_Hann_512[i]));
    printf("], \"hann_1024\": [");
    for (int i = 0; i < 1024; ++i) printf("%s%u", i ? "," : "", fb(oracle_von_Hann_1024[i]));
    /* formula branch for 2048 floats: 1 - arm_cos_f32(...) as the window code forms it */
    printf("], \"hann_formula_2048\": [");
    for (int i = 0; i < 2048; ++i)
    {
        const uint16_t fft_iq_len = 2048;
        const float32_t w = (1 - (arm_cos_f32(PI * 2 * (float32_t)i / (float32_t)(fft_iq_len - 1))));
        printf("%s%u", i ? "," : "", fb(w));
    }
    /* zoom producer tables per magnification 1..5 (2x .. 32x): the 4-stage lowpass biquad
       mag_coeffs[m] (audio_driver.c:204-363) and the decimator FirZoomFFTDecimate[m]
       (filters/fir_rx_decimate_4.c:108), read back from the instance Spectrum_Set configured */
    printf("]");
    for (int m = 1; m <= 5; ++m)
    {
        oracle_ref_spec_magnify(m);
        const float* bq = oracle_ref_zoom_biquad(m);
        const arm_fir_decimate_instance_f32* d = oracle_ref_zoom_decim();
        printf(", \"zoom_biquad_%d\": [", m);
        for (int i = 0; i < 20; ++i) printf("%s%u", i ? "," : "", fb(bq[i]));
        printf("], \"zoom_decim_%d\": {\"M\": %d, \"taps\": [", m, d->M);
        for (int i = 0; i < d->numTaps; ++i) printf("%s%u", i ? "," : "", fb(d->pCoeffs[i]));
        printf("]}");
    }
    oracle_ref_spec_magnify(0);
    printf("}\n");
}
