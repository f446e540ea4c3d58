/*
 * ORACLE TEST INFRASTRUCTURE -- golden vectors of the CMSIS-DSP f32 functions the firmware's
 * RX/TX path calls, from the reference's own CMSIS-DSP V1.4.5 build (oracle/ref/Makefile),
 * for the CMSIS-signature shims of libuhsdr_cmsis.so (include/uhsdr_cmsis.h).
 *
 *   uhsdr_ref dump=cmsis out=<dir>
 *
 * writes one raw little-endian float32 file per array, <dir>/<case>.<field>.f32, and prints a
 * JSON manifest {case: {"params": {...}, "fields": {field: count}}}.  Every stateful case runs
 * several consecutive calls on one instance, so the state carried in pState is exercised.
 * Inputs come from a fixed LCG; coefficients of the IIR cases are drawn stable.
 *
 * arm_cfft_f32 (TransformFunctions/arm_cfft_f32.c:574-628) is dropped from the link (its bit
 * reversal is ARM assembly, see ref_spectrum.c), so its wrapper -- input conjugation for the
 * inverse, length switch, bit reversal, conjugate-and-scale by 1/L -- is restated in
 * cfft_wrapper() around the reference's radix stages (ref_cfft_stages, ref_spectrum.c).
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>
#include "arm_math.h"

void ref_cfft_stages(int L, float* p, int bitrev);

static uint32_t lcg_state = 0x5EED1234u;
static float urand(void)   /* [-1, 1) */
{
    lcg_state = lcg_state * 1664525u + 1013904223u;
    return (float)((int32_t)lcg_state) * (1.0f / 2147483648.0f);
}

static const char* g_dir;
static int g_first_case = 1, g_first_field;

static void case_begin(const char* name, const char* params_json)
{
    printf("%s\"%s\": {\"params\": %s, \"fields\": {", g_first_case ? "" : ", ", name, params_json);
    g_first_case = 0;
    g_first_field = 1;
}

static void case_end(void) { printf("}}"); }

static void put(const char* cname, const char* field, const float* x, size_t n)
{
    char path[512];
    snprintf(path, sizeof path, "%s/%s.%s.f32", g_dir, cname, field);
    FILE* f = fopen(path, "wb");
    if (!f || fwrite(x, sizeof(float), n, f) != n) { fprintf(stderr, "write %s failed\n", path); exit(2); }
    fclose(f);
    printf("%s\"%s\": %zu", g_first_field ? "" : ", ", field, n);
    g_first_field = 0;
}

static float* frand(size_t n, float scale)
{
    float* x = malloc(sizeof(float) * (n ? n : 1));
    for (size_t i = 0; i < n; ++i) x[i] = urand() * scale;
    return x;
}

/* arm_fir_f32: numTaps T, blockSize B, K calls */
static void fir_case(const char* name, int T, int B, int K)
{
    char p[128];
    snprintf(p, sizeof p, "{\"numTaps\": %d, \"blockSize\": %d, \"calls\": %d}", T, B, K);
    case_begin(name, p);
    float* c = frand(T, 0.25f);
    float* x = frand((size_t)B * K, 1.0f);
    float* y = calloc((size_t)B * K, sizeof(float));
    float* st = calloc(T + B - 1, sizeof(float));
    arm_fir_instance_f32 S;
    arm_fir_init_f32(&S, T, c, st, B);
    for (int k = 0; k < K; ++k) arm_fir_f32(&S, x + (size_t)k * B, y + (size_t)k * B, B);
    put(name, "coeffs", c, T); put(name, "src", x, (size_t)B * K); put(name, "dst", y, (size_t)B * K);
    put(name, "state", st, T - 1);
    case_end();
    free(c); free(x); free(y); free(st);
}

/* arm_fir_decimate_f32: numTaps T, factor M, blockSize B (input samples), K calls */
static void decim_case(const char* name, int T, int M, int B, int K)
{
    char p[160];
    snprintf(p, sizeof p, "{\"numTaps\": %d, \"M\": %d, \"blockSize\": %d, \"calls\": %d}", T, M, B, K);
    case_begin(name, p);
    float* c = frand(T, 0.25f);
    float* x = frand((size_t)B * K, 1.0f);
    float* y = calloc((size_t)B / M * K, sizeof(float));
    float* st = calloc(T + B - 1, sizeof(float));
    arm_fir_decimate_instance_f32 S;
    if (arm_fir_decimate_init_f32(&S, T, M, c, st, B) != ARM_MATH_SUCCESS) exit(3);
    for (int k = 0; k < K; ++k) arm_fir_decimate_f32(&S, x + (size_t)k * B, y + (size_t)k * B / M, B);
    put(name, "coeffs", c, T); put(name, "src", x, (size_t)B * K); put(name, "dst", y, (size_t)B / M * K);
    put(name, "state", st, T - 1);
    case_end();
    free(c); free(x); free(y); free(st);
}

/* arm_fir_interpolate_f32: factor L, numTaps T (phaseLength T/L), blockSize B, K calls */
static void interp_case(const char* name, int L, int T, int B, int K)
{
    char p[160];
    snprintf(p, sizeof p, "{\"L\": %d, \"numTaps\": %d, \"blockSize\": %d, \"calls\": %d}", L, T, B, K);
    case_begin(name, p);
    const int ph = T / L;
    float* c = frand(T, 0.5f);
    float* x = frand((size_t)B * K, 1.0f);
    float* y = calloc((size_t)B * L * K, sizeof(float));
    float* st = calloc(ph + B - 1, sizeof(float));
    arm_fir_interpolate_instance_f32 S;
    if (arm_fir_interpolate_init_f32(&S, L, T, c, st, B) != ARM_MATH_SUCCESS) exit(3);
    for (int k = 0; k < K; ++k) arm_fir_interpolate_f32(&S, x + (size_t)k * B, y + (size_t)k * B * L, B);
    put(name, "coeffs", c, T); put(name, "src", x, (size_t)B * K); put(name, "dst", y, (size_t)B * L * K);
    put(name, "state", st, ph - 1 > 0 ? ph - 1 : 0);
    case_end();
    free(c); free(x); free(y); free(st);
}

/* arm_iir_lattice_f32: numStages S, blockSize B, K calls; reflection coefficients |k| < 0.8 */
static void lattice_case(const char* name, int NS, int B, int K)
{
    char p[128];
    snprintf(p, sizeof p, "{\"numStages\": %d, \"blockSize\": %d, \"calls\": %d}", NS, B, K);
    case_begin(name, p);
    float* kc = frand(NS, 0.8f);
    float* vc = frand(NS + 1, 0.5f);
    float* x = frand((size_t)B * K, 1.0f);
    float* y = calloc((size_t)B * K, sizeof(float));
    float* st = calloc(NS + B, sizeof(float));
    arm_iir_lattice_instance_f32 S;
    arm_iir_lattice_init_f32(&S, NS, kc, vc, st, B);
    for (int k = 0; k < K; ++k) arm_iir_lattice_f32(&S, x + (size_t)k * B, y + (size_t)k * B, B);
    put(name, "k", kc, NS); put(name, "v", vc, NS + 1); put(name, "src", x, (size_t)B * K);
    put(name, "dst", y, (size_t)B * K); put(name, "state", st, NS);
    case_end();
    free(kc); free(vc); free(x); free(y); free(st);
}

/* arm_biquad_cascade_df1_f32: numStages S, blockSize B, K calls; each stage a stable pair of
   poles (radius < 0.95) with CMSIS's sign convention (a1, a2 enter as + a1 y[n-1] + a2 y[n-2]) */
static void biquad_case(const char* name, int NS, int B, int K)
{
    char p[128];
    snprintf(p, sizeof p, "{\"numStages\": %d, \"blockSize\": %d, \"calls\": %d}", NS, B, K);
    case_begin(name, p);
    float* c = malloc(sizeof(float) * 5 * NS);
    for (int s = 0; s < NS; ++s)
    {
        const float r = 0.5f + 0.45f * (0.5f * urand() + 0.5f), th = 3.14159265f * (0.5f * urand() + 0.5f);
        c[5 * s + 0] = 0.5f * urand(); c[5 * s + 1] = 0.5f * urand(); c[5 * s + 2] = 0.5f * urand();
        c[5 * s + 3] = 2.0f * r * cosf(th);
        c[5 * s + 4] = -r * r;
    }
    float* x = frand((size_t)B * K, 1.0f);
    float* y = calloc((size_t)B * K, sizeof(float));
    float* st = calloc(4 * NS, sizeof(float));
    arm_biquad_casd_df1_inst_f32 S;
    arm_biquad_cascade_df1_init_f32(&S, NS, c, st);
    for (int k = 0; k < K; ++k) arm_biquad_cascade_df1_f32(&S, x + (size_t)k * B, y + (size_t)k * B, B);
    put(name, "coeffs", c, 5 * NS); put(name, "src", x, (size_t)B * K); put(name, "dst", y, (size_t)B * K);
    put(name, "state", st, 4 * NS);
    case_end();
    free(c); free(x); free(y); free(st);
}

/* arm_cfft_f32(S, p1, ifftFlag, bitReverseFlag), arm_cfft_f32.c:574-628 */
static void cfft_wrapper(int L, float* p1, int ifft, int bitrev)
{
    if (ifft == 1)
    {
        float* p = p1 + 1;
        for (int l = 0; l < L; ++l) { *p = -*p; p += 2; }
    }
    ref_cfft_stages(L, p1, bitrev);
    if (ifft == 1)
    {
        const float invL = 1.0f / (float32_t)L;
        float* p = p1;
        for (int l = 0; l < L; ++l)
        {
            *p++ *= invL;
            *p = -(*p) * invL;
            p++;
        }
    }
}

const arm_cfft_instance_f32* ref_cfft_instance(int L);

static void cfft_case(const char* name, int L, int ifft, int bitrev)
{
    char p[160];
    const arm_cfft_instance_f32* S = ref_cfft_instance(L);
    snprintf(p, sizeof p, "{\"fftLen\": %d, \"ifftFlag\": %d, \"bitReverseFlag\": %d, \"bitRevLength\": %d}", L, ifft,
             bitrev, S->bitRevLength);
    case_begin(name, p);
    {
        /* the instance's own tables (arm_const_structs.c / arm_common_tables.c): twiddleCoef_L
           (L complex values; the radix-8 stages index up to 7(L/8-1)) and the bit-reversal byte-offset table, stored as floats (exact) */
        float* tab = malloc(sizeof(float) * (S->bitRevLength + 1));
        for (int i = 0; i < S->bitRevLength; ++i) tab[i] = (float)S->pBitRevTable[i];
        put(name, "twiddle", S->pTwiddle, 2 * (size_t)L);
        put(name, "bitrev", tab, S->bitRevLength);
        free(tab);
    }
    float* x = frand(2 * (size_t)L, 1.0f);
    float* y = malloc(sizeof(float) * 2 * L);
    memcpy(y, x, sizeof(float) * 2 * L);
    cfft_wrapper(L, y, ifft, bitrev);
    put(name, "src", x, 2 * (size_t)L); put(name, "dst", y, 2 * (size_t)L);
    case_end();
    free(x); free(y);
}

/* arm_lms_norm_f32: numTaps T, blockSize B, K calls, step mu; the coefficients start from small
   random values (the firmware keeps them across re-inits unless reset_dsp_nr), the reference
   signal is a second LCG stream.  inplace: pErr == pSrc, as AudioDriver_NotchFilter calls it
   (audio_driver.c:1755). */
static void lms_case(const char* name, int T, int B, int K, float mu, int inplace)
{
    char p[192];
    snprintf(p, sizeof p, "{\"numTaps\": %d, \"blockSize\": %d, \"calls\": %d, \"mu\": %.9g, \"inplace\": %d}",
             T, B, K, mu, inplace);
    case_begin(name, p);
    float* c = frand(T, 0.05f);
    float* x = frand((size_t)B * K, 1.0f);
    float* d = frand((size_t)B * K, 1.0f);
    for (size_t i = 0; i < (size_t)B * K; ++i) d[i] = 0.5f * d[i] + 0.5f * x[i];   /* correlated reference */
    put(name, "coeffs0", c, T); put(name, "src", x, (size_t)B * K); put(name, "ref", d, (size_t)B * K);
    float* y = calloc((size_t)B * K, sizeof(float));
    float* e = calloc((size_t)B * K, sizeof(float));
    float* st = calloc(T + B - 1, sizeof(float));
    float* blk = malloc(sizeof(float) * B);
    arm_lms_norm_instance_f32 S;
    arm_lms_norm_init_f32(&S, T, c, st, mu, B);
    for (int k = 0; k < K; ++k)
    {
        if (inplace)
        {
            memcpy(blk, x + (size_t)k * B, sizeof(float) * B);
            arm_lms_norm_f32(&S, blk, d + (size_t)k * B, y + (size_t)k * B, blk, B);
            memcpy(e + (size_t)k * B, blk, sizeof(float) * B);
        }
        else
            arm_lms_norm_f32(&S, x + (size_t)k * B, d + (size_t)k * B, y + (size_t)k * B, e + (size_t)k * B, B);
    }
    const float ex[2] = { S.energy, S.x0 };
    put(name, "out", y, (size_t)B * K); put(name, "err", e, (size_t)B * K);
    put(name, "coeffs", c, T); put(name, "state", st, T - 1); put(name, "energy_x0", ex, 2);
    case_end();
    free(c); free(x); free(d); free(y); free(e); free(st); free(blk);
}

static void mag_case(const char* name, int n)
{
    char p[64];
    snprintf(p, sizeof p, "{\"numSamples\": %d}", n);
    case_begin(name, p);
    float* x = frand(2 * (size_t)n, 100.0f);
    float* y = malloc(sizeof(float) * n);
    arm_cmplx_mag_f32(x, y, n);
    put(name, "src", x, 2 * (size_t)n); put(name, "dst", y, n);
    case_end();
    free(x); free(y);
}

int ref_cmsis_dump(const char* dir)
{
    g_dir = dir;
    printf("{");
    fir_case("fir_89x32", 89, 32, 5);
    fir_case("fir_199x8", 199, 8, 40);
    fir_case("fir_7x13", 7, 13, 4);
    fir_case("fir_1x5", 1, 5, 3);
    fir_case("fir_513x256", 513, 256, 6);   /* C5's synthetic long FIR */
    decim_case("decim_43_m4", 43, 4, 32, 5);
    decim_case("decim_83_m4", 83, 4, 128, 3);
    decim_case("decim_5_m2", 5, 2, 10, 4);
    interp_case("interp_l4_t16", 4, 16, 8, 5);
    interp_case("interp_l4_t4", 4, 4, 8, 3);
    interp_case("interp_l2_t6", 2, 6, 7, 4);
    interp_case("interp_l3_t21", 3, 21, 9, 3);
    lattice_case("lattice_10x8", 10, 8, 6);
    lattice_case("lattice_6x32", 6, 32, 4);
    lattice_case("lattice_3x5", 3, 5, 3);
    biquad_case("biquad_4x8", 4, 8, 6);
    biquad_case("biquad_1x37", 1, 37, 3);
    biquad_case("biquad_3x1", 3, 1, 9);
    cfft_case("cfft_256", 256, 0, 1);
    cfft_case("cfft_512", 512, 0, 1);
    cfft_case("cfft_1024", 1024, 0, 1);
    cfft_case("cfft_512_nobitrev", 512, 0, 0);
    cfft_case("cfft_1024_nobitrev", 1024, 0, 0);
    cfft_case("icfft_256", 256, 1, 1);
    cfft_case("icfft_1024", 1024, 1, 1);
    cfft_case("cfft_16", 16, 0, 1);
    cfft_case("cfft_32", 32, 0, 1);
    cfft_case("cfft_64", 64, 0, 1);
    cfft_case("cfft_128", 128, 0, 1);
    cfft_case("cfft_2048", 2048, 0, 1);
    cfft_case("cfft_4096", 4096, 0, 1);
    cfft_case("icfft_16", 16, 1, 1);
    cfft_case("icfft_128", 128, 1, 1);
    cfft_case("icfft_2048", 2048, 1, 1);
    cfft_case("icfft_4096", 4096, 1, 1);
    cfft_case("cfft_64_nobitrev", 64, 0, 0);
    cfft_case("cfft_2048_nobitrev", 2048, 0, 0);
    mag_case("mag_1000", 1000);
    /* the auto notch's instance: 64 taps, IQ_BLOCK_SIZE 32, mu from notch_mu 5
       (audio_driver.c:1169-1173: log10f((5 + 1) / 1500 + 1)) */
    lms_case("lms_64x32", 64, 32, 12, log10f(((5 + 1.0) / 1500.0) + 1.0), 1);
    lms_case("lms_64x32_sep", 64, 32, 4, 0.1f, 0);
    lms_case("lms_13x7", 13, 7, 6, 0.05f, 0);
    lms_case("lms_1x5", 1, 5, 3, 0.2f, 1);
    lms_case("lms_200x3", 200, 3, 9, 0.01f, 0);
    printf("}\n");
    return 0;
}
