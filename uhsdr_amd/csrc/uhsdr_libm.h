/*
 * glibc-exact single-precision libm functions the demodulators call per sample.
 *
 * The reference runs AudioDriver_DemodSAM / AudioDriver_DemodFM (drivers/audio/audio_driver.c:
 * 2021-2147, 1544-1600) against the host's libm: glibc 2.35 here and on the GPU box host
 * (both x86-64 with FMA).  The SAM PLL feeds every rounding of sincosf / atan2f back into
 * its phase, so the device must reproduce those functions bit for bit, not merely within an
 * ulp.  This header restates glibc 2.35's published algorithms:
 *
 *   sincosf  sysdeps/ieee754/flt-32/s_sincosf.c + sincosf.h (Szabolcs Nagy, ARM
 *            optimized-routines, 2018): double-precision polynomials, fast pi/2 reduction;
 *            the x86-64 build dispatches (IFUNC) to s_sincosf-fma.c, compiled with -mfma,
 *            so every a + b*c below is one fused multiply-add.  Table values: the
 *            __sincosf_table of the published source.
 *   atan2f   sysdeps/ieee754/flt-32/e_atan2f.c + s_atanf.c (fdlibm, Sun 1993): pure binary32
 *            arithmetic, no IFUNC variant.
 *
 * Pinned against the host's libm by tests/test_libm.py (every float in [0, 2*pi] for
 * sincosf -- the PLL phase range -- plus random and special operands for atan2f).
 * Compiled by hipcc for the device and by gcc (-ffp-contract=off) for the host check;
 * the fused operations are explicit fma() calls, so no compiler contraction is involved.
 */
#ifndef UHSDR_LIBM_H
#define UHSDR_LIBM_H

#include <stdint.h>
#include <string.h>
#include <math.h>

#ifndef UHSDR_ATAN_SHORTDIV
#define UHSDR_ATAN_SHORTDIV 1
#endif
#ifdef __HIPCC__
#define UHSDR_LIBM_FN __host__ __device__ static inline
#else
#define UHSDR_LIBM_FN static inline
#endif

UHSDR_LIBM_FN uint32_t ul_asuint(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
UHSDR_LIBM_FN float ul_asfloat(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
/* top 12 bits of |x|: exponent and 3 mantissa bits (s_sincosf.c abstop12) */
UHSDR_LIBM_FN uint32_t ul_abstop12(float x) { return (ul_asuint(x) >> 20) & 0x7ff; }
UHSDR_LIBM_FN uint64_t ul_asuint64(double f) { uint64_t u; memcpy(&u, &f, 8); return u; }
UHSDR_LIBM_FN double ul_asdouble(uint64_t u) { double f; memcpy(&f, &u, 8); return f; }
/* c ? a : b on operands already evaluated.  clang emits a conditional operator whose arms
   compute something as a branch diamond, and the ones the optimizer does not fold back become
   exec-masked regions (separate basic blocks) on the GPU -- which keeps the scheduler from
   overlapping two PLL samples -- or, for a chain over an index, a table load.  As a function of
   its evaluated parameters the diamond is empty and folds into one v_cndmask. */
UHSDR_LIBM_FN float ul_sel(int c, float a, float b) { return c ? a : b; }

/* ---- sincosf, |y| < 120 (the PLL phase is in [0, 2*pi)) ---- */
typedef struct
{
    double hpi_inv;          /* 2/pi * 2^24 (no round-to-int intrinsics on x86-64) */
    double hpi;              /* pi/2 */
    double c0, c1, s1, c2, s2, c3, s3, c4;
} ul_sincos_t;

/* __sincosf_table[0]; table[1] (quadrants 2 and 3) holds the same sine coefficients and the
   cosine ones negated -- see ul_sincosf */
#ifdef __HIPCC__
__host__ __device__
#endif
static inline const ul_sincos_t* ul_sincosf_table(void)
{
#ifdef __HIPCC__
    static __constant__ const ul_sincos_t t = {
#else
    static const ul_sincos_t t = {
#endif
        0x1.45f306dc9c883p+23, 0x1.921fb54442d18p+0,
        0x1p+0, -0x1.ffffffd0c621cp-2, -0x1.555545995a603p-3, 0x1.55553e1068f19p-5,
        0x1.1107605230bc4p-7, -0x1.6c087e89a359dp-10, -0x1.994eb3774cf24p-13, 0x1.99343027bf8c3p-16,
    };
    return &t;
}

/* sincosf.h sincosf_poly (FMA build) before its quadrant swap */
UHSDR_LIBM_FN void ul_sincosf_poly(double x, double x2, const ul_sincos_t* p, float* rsp, float* rcp)
{
    const double x4 = x2 * x2;
    const double x3 = x2 * x;
    const double c2 = fma(x2, p->c4, p->c3);
    const double s1 = fma(x2, p->s3, p->s2);
    const double c1 = fma(x2, p->c1, p->c0);
    const double x5 = x3 * x2;
    const double x6 = x4 * x2;
    const double s = fma(x3, p->s1, x);
    const double c = fma(x4, p->c2, c1);
    *rsp = (float)fma(x5, s1, s);
    *rcp = (float)fma(x6, c2, c);
}

/* s_sincosf.c for |y| < 120 (callers guarantee the range; the Payne-Hanek branch for huge
   arguments is not needed by the PLL).  Branch-free: for |y| < pi/4 the reduction yields
   n = 0, x - 0*pi/2 = x (exact) and sign +1, i.e. exactly the small branch's polynomial call,
   so one path serves both and a wave's lanes never split between them; |y| < 2^-12 selects
   (y, 1) at the end.  Quadrants 2 and 3 evaluate the cosine polynomial with every coefficient
   negated (table[1]): round-to-nearest is symmetric and none of its partial sums is zero for
   |x| <= pi/4, so that is exactly table 0's result with the sign flipped. */
UHSDR_LIBM_FN void ul_sincosf(float y, float* sinp, float* cosp)
{
    double x = y;
    const ul_sincos_t* p = ul_sincosf_table();
    /* reduce_fast, !TOINT_INTRINSICS */
    const double r = x * p->hpi_inv;
    const int n = ((int32_t)r + 0x800000) >> 24;
    x = fma(-(double)n, p->hpi, x);
    /* x * sign[n & 3], sign = +1, -1, -1, +1: negative when bit 1 of n + 1 is set */
    const double xs = ul_asdouble(ul_asuint64(x) ^ ((uint64_t)((n + 1) & 2) << 62));
    float rs, rc;
    ul_sincosf_poly(xs, x * x, p, &rs, &rc);
    rc = ul_asfloat(ul_asuint(rc) ^ ((uint32_t)(n & 2) << 30));     /* table[1] */
    const float sv = ul_sel(n & 1, rc, rs), cv = ul_sel(n & 1, rs, rc);   /* quadrant swap */
    const int tiny = ul_abstop12(y) < ul_abstop12(0x1p-12f);
    *sinp = ul_sel(tiny, y, sv);
    *cosp = ul_sel(tiny, 1.0f, cv);
}

/* ---- atanf / atan2f (fdlibm binary32) ---- */
/* Both are written branch-free on the main path: in a wave, lanes whose arguments fall in
 * different reduction intervals would otherwise run every interval's division one after the
 * other.  Each interval of fdlibm's reduction is a quotient num / den of the same operations,
 * so the interval selects num, den and the atanhi / atanlo pair, one division runs, and the
 * special cases (tiny, huge, NaN) select their results at the end -- the same binary32
 * operations on the same operands as the branches (pinned against glibc, tests/test_libm.py). */
UHSDR_LIBM_FN float ul_atanf(float x)
{
    const float atanhi[4] = { 4.6364760399e-01f, 7.8539812565e-01f, 9.8279368877e-01f, 1.5707962513e+00f };
    const float atanlo[4] = { 5.0121582440e-09f, 3.7748947079e-08f, 3.4473217170e-08f, 7.5497894159e-08f };
    const float aT[11] = { 3.3333334327e-01f, -2.0000000298e-01f, 1.4285714924e-01f, -1.1111110449e-01f,
                           9.0908870101e-02f, -7.6918758452e-02f, 6.6610731184e-02f, -5.8335702866e-02f,
                           4.9768779427e-02f, -3.6531571299e-02f, 1.6285819933e-02f };
    const uint32_t hx = ul_asuint(x);
    const uint32_t ix = hx & 0x7fffffff;
    const float ax = fabsf(x);
    /* |x| < 7/16: no reduction; 7/16 <= |x| < 11/16: (2|x| - 1) / (2 + |x|); < 19/16:
       (|x| - 1) / (|x| + 1); < 2.4375: (|x| - 1.5) / (1 + 1.5|x|); above: -1 / |x| */
    const int small = ix < 0x3ee00000, lo2 = ix < 0x3f980000, i0 = ix < 0x3f300000, i2 = ix < 0x401c0000;
    const float n0 = 2.0f * ax - 1.0f, d0 = 2.0f + ax;
    const float n1 = ax - 1.0f, d1 = ax + 1.0f;
    const float n2 = ax - 1.5f, d2 = 1.0f + 1.5f * ax;
    const float num = ul_sel(lo2, ul_sel(i0, n0, n1), ul_sel(i2, n2, -1.0f));
    const float den = ul_sel(lo2, ul_sel(i0, d0, d1), ul_sel(i2, d2, ax));
    const float hi = ul_sel(lo2, ul_sel(i0, atanhi[0], atanhi[1]), ul_sel(i2, atanhi[2], atanhi[3]));
    const float lo = ul_sel(lo2, ul_sel(i0, atanlo[0], atanlo[1]), ul_sel(i2, atanlo[2], atanlo[3]));
    const float xr = ul_sel(small, x, num / den);
    const float z = xr * xr;
    const float w = z * z;
    const float s1 = z * (aT[0] + w * (aT[2] + w * (aT[4] + w * (aT[6] + w * (aT[8] + w * aT[10])))));
    const float s2 = w * (aT[1] + w * (aT[3] + w * (aT[5] + w * (aT[7] + w * aT[9]))));
    const float zz = hi - ((xr * (s1 + s2) - lo) - xr);
    float r = ul_sel(small, xr - xr * (s1 + s2), ul_sel(hx >> 31, -zz, zz));
    r = ul_sel(ix < 0x31000000, x, r);                                  /* |x| < 2^-29 */
    const float huge = ul_sel(hx >> 31, -atanhi[3] - atanlo[3], atanhi[3] + atanlo[3]);
    r = ul_sel(ix >= 0x4c000000, ul_sel(ix > 0x7f800000, x + x, huge), r);   /* |x| >= 2^25, NaN */
    return r;
}

/* ul_atanf for a >= +0 (atan2f's |y / x|), NaN operands left to the caller.  fdlibm's four
 * reductions are (ka a - kb) / (ka + kb a) with ka = 2, 1, 1, 0 and kb = 1, 1, 1.5, 1: ka a is
 * exact, so the numerator is one fused operation with fdlibm's rounding, and kb a + ka rounds
 * like fdlibm's denominators (1.5f * a, then the sum; the other products are exact). */
UHSDR_LIBM_FN float ul_atanf_pos(float a)
{
    const float atanhi[4] = { 4.6364760399e-01f, 7.8539812565e-01f, 9.8279368877e-01f, 1.5707962513e+00f };
    const float atanlo[4] = { 5.0121582440e-09f, 3.7748947079e-08f, 3.4473217170e-08f, 7.5497894159e-08f };
    const float aT[11] = { 3.3333334327e-01f, -2.0000000298e-01f, 1.4285714924e-01f, -1.1111110449e-01f,
                           9.0908870101e-02f, -7.6918758452e-02f, 6.6610731184e-02f, -5.8335702866e-02f,
                           4.9768779427e-02f, -3.6531571299e-02f, 1.6285819933e-02f };
    const uint32_t ia = ul_asuint(a);
    const int small = ia < 0x3ee00000, lo2 = ia < 0x3f980000, i0 = ia < 0x3f300000, i2 = ia < 0x401c0000;
    const float ka = ul_sel(i0, 2.0f, ul_sel(i2, 1.0f, 0.0f));
    const float kb = ul_sel(!lo2 && i2, 1.5f, 1.0f);
    const float num = fmaf(ka, a, -kb);
    const float den = kb * a + ka;
    const float hi = ul_sel(lo2, ul_sel(i0, atanhi[0], atanhi[1]), ul_sel(i2, atanhi[2], atanhi[3]));
    const float lo = ul_sel(lo2, ul_sel(i0, atanlo[0], atanlo[1]), ul_sel(i2, atanlo[2], atanlo[3]));
#if defined(__HIP_DEVICE_COMPILE__) && UHSDR_ATAN_SHORTDIV
    /* num / den by a reciprocal and one residual correction: equal to the IEEE quotient for every
       binary32 a that reaches it, checked exhaustively on the device (tools/micro/atan_div_check.hip,
       profiles/r05_atan_div_check.txt); 4 dependent operations instead of the scaled
       division's ~10 on the PLL's critical path */
    const float rr = __builtin_amdgcn_rcpf(den);
    const float q0 = num * rr;
    const float quo = fmaf(fmaf(-den, q0, num), rr, q0);
#else
    const float quo = num / den;
#endif
    const float xr = ul_sel(small, a, quo);
    const float z = xr * xr;
    const float w = z * z;
    const float s1 = z * (aT[0] + w * (aT[2] + w * (aT[4] + w * (aT[6] + w * (aT[8] + w * aT[10])))));
    const float s2 = w * (aT[1] + w * (aT[3] + w * (aT[5] + w * (aT[7] + w * aT[9]))));
    const float t = xr * (s1 + s2);
    float r = ul_sel(small, xr - t, hi - ((t - lo) - xr));
    r = ul_sel(ia < 0x31000000, a, r);                                  /* a < 2^-29 */
    return ul_sel(ia >= 0x4c000000, atanhi[3] + atanlo[3], r);         /* a >= 2^25 */
}

UHSDR_LIBM_FN float ul_atan2f(float y, float x)
{
    const float tiny = 1.0e-30f, pi_o_4 = 7.8539818525e-01f, pi_o_2 = 1.5707963705e+00f,
                pi = 3.1415927410e+00f, pi_lo = -8.7422776573e-08f;
    const int32_t hx = (int32_t)ul_asuint(x), hy = (int32_t)ul_asuint(y);
    const int32_t ix = hx & 0x7fffffff, iy = hy & 0x7fffffff;
    /* Branch-free: fdlibm's main path (e_atan2f.c, the k / atanf / quadrant tail) runs for
     * every operand pair and the operands it does not cover select their results after it,
     * lowest precedence first, so the SAM PLL's per-sample chain stays one basic block.
     * The main path already gives fdlibm's special results for y = +-0 with x != 0 (z = 0) and
     * for x = +-inf with y finite (y / x = +-0); x = 1.0 (fdlibm: atanf(y)) needs no case either:
     * y / 1 = y, atanf is odd and the |y/x| > 2^26 override is skipped for it.  Pinned for
     * every binary32 y at x = 1 (tools/libm_check.c "atan2x1") and on random and special pairs. */
    const int32_t k = (iy - ix) >> 23;
    float z = ul_atanf_pos(fabsf(y / x));
    z = ul_sel(hx < 0 && k < -26, 0.0f, z);                 /* |y|/x < -2^26 */
    z = ul_sel(k > 26 && hx != 0x3f800000, pi_o_2 + 0.5f * pi_lo, z);   /* |y/x| > 2^26 */
    /* fdlibm's quadrants: z, -z, pi - (z - pi_lo), (z - pi_lo) - pi; z and pi - (z - pi_lo) are
       positive and round-to-nearest is symmetric, so the sign of y goes on last */
    float r = copysignf(ul_sel(hx < 0, pi - (z - pi_lo), z), y);
    r = ul_sel(iy == 0x7f800000,                           /* y = +-inf */
               copysignf(ul_sel(ix == 0x7f800000, ul_sel(hx < 0, 3.0f * pi_o_4 + tiny, pi_o_4 + tiny),
                                pi_o_2 + tiny), y), r);
    r = ul_sel(ix == 0,                                     /* x = +-0 */
               ul_sel(iy == 0, ul_sel(hx < 0, copysignf(pi + tiny, y), y), copysignf(pi_o_2 + tiny, y)), r);
    r = ul_sel(ix > 0x7f800000 || iy > 0x7f800000, x + y, r);   /* NaN */
    return r;
}

/* ---- asinf (glibc sysdeps/ieee754/flt-32/e_asinf.c: fdlibm binary32 with a degree-4 minimax
 *      polynomial; the twin-peaks I/Q phase detector, audio_driver.c:2211) ---- */
UHSDR_LIBM_FN float ul_asinf(float x)
{
    const float one = 1.0f, pio2_hi = 1.57079637050628662109375f, pio2_lo = -4.37113900018624283e-8f,
                pio4_hi = 0.785398185253143310546875f,
                p0 = 1.666675248e-1f, p1 = 7.495297643e-2f, p2 = 4.547037598e-2f, p3 = 2.417951451e-2f,
                p4 = 4.216630880e-2f;
    const int32_t hx = (int32_t)ul_asuint(x);
    const int32_t ix = hx & 0x7fffffff;
    float t, w, p, q, c, r, s;
    if (ix == 0x3f800000) return x * pio2_hi + x * pio2_lo;       /* asin(+-1) = +-pi/2 */
    if (ix > 0x3f800000) return (x - x) / (x - x);                /* |x| > 1: NaN */
    if (ix < 0x3f000000)                                          /* |x| < 0.5 */
    {
        if (ix < 0x32000000) return x;                            /* |x| < 2^-27 */
        t = x * x;
        w = t * (p0 + t * (p1 + t * (p2 + t * (p3 + t * p4))));
        return x + x * w;
    }
    w = one - fabsf(x);                                           /* 1 > |x| >= 0.5 */
    t = w * 0.5f;
    p = t * (p0 + t * (p1 + t * (p2 + t * (p3 + t * p4))));
    s = sqrtf(t);
    if (ix >= 0x3F79999A)                                         /* |x| > 0.975 */
        t = pio2_hi - (2.0f * (s + s * p) - pio2_lo);
    else
    {
        w = ul_asfloat(ul_asuint(s) & 0xfffff000u);
        c = (t - w * w) / (s + w);
        r = p;
        p = 2.0f * s * r - (pio2_lo - 2.0f * c);
        q = pio4_hi - 2.0f * w;
        t = pio4_hi - (p - q);
    }
    return hx > 0 ? t : -t;
}

#endif /* UHSDR_LIBM_H */
