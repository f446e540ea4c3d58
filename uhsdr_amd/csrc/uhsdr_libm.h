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
/* c ? a : b as a bit-mask blend.  clang emits a conditional operator with non-constant arms as
   a branch diamond, and the ones the optimizer does not fold back become exec-masked regions
   (separate basic blocks) on the GPU -- which keeps the scheduler from overlapping two PLL
   samples -- or, for a chain over an index, a table load.  The blend is one v_cndmask. */
UHSDR_LIBM_FN float ul_sel(int c, float a, float b)
{
    const uint32_t m = 0u - (uint32_t)(c != 0);
    return ul_asfloat((ul_asuint(a) & m) | (ul_asuint(b) & ~m));
}
UHSDR_LIBM_FN double ul_seld(int c, double a, double b)
{
    const uint64_t m = 0ull - (uint64_t)(c != 0);
    return ul_asdouble((ul_asuint64(a) & m) | (ul_asuint64(b) & ~m));
}

/* ---- sincosf, |y| < 120 (the PLL phase is in [0, 2*pi)) ---- */
typedef struct
{
    double sign[4];          /* sign of sine in quadrants 0..3 */
    double hpi_inv;          /* 2/pi * 2^24 (no round-to-int intrinsics on x86-64) */
    double hpi;              /* pi/2 */
    double c0, c1, s1, c2, s2, c3, s3, c4;
} ul_sincos_t;

#ifdef __HIPCC__
__host__ __device__
#endif
static inline const ul_sincos_t* ul_sincosf_table(int k)
{
#ifdef __HIPCC__
    static __constant__ const ul_sincos_t t[2] = {
#else
    static const ul_sincos_t t[2] = {
#endif
        { { 1.0, -1.0, -1.0, 1.0 }, 0x1.45f306dc9c883p+23, 0x1.921fb54442d18p+0,
          0x1p+0, -0x1.ffffffd0c621cp-2, -0x1.555545995a603p-3, 0x1.55553e1068f19p-5,
          0x1.1107605230bc4p-7, -0x1.6c087e89a359dp-10, -0x1.994eb3774cf24p-13, 0x1.99343027bf8c3p-16 },
        { { 1.0, -1.0, -1.0, 1.0 }, 0x1.45f306dc9c883p+23, 0x1.921fb54442d18p+0,
          -0x1p+0, 0x1.ffffffd0c621cp-2, -0x1.555545995a603p-3, -0x1.55553e1068f19p-5,
          0x1.1107605230bc4p-7, 0x1.6c087e89a359dp-10, -0x1.994eb3774cf24p-13, -0x1.99343027bf8c3p-16 },
    };
    return &t[k];
}

/* sincosf.h sincosf_poly (FMA build); the quadrant swap as selects */
UHSDR_LIBM_FN void ul_sincosf_poly(double x, double x2, const ul_sincos_t* p, int n, float* sinp, float* cosp)
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
    const float rs = (float)fma(x5, s1, s);
    const float rc = (float)fma(x6, c2, c);
    *sinp = ul_sel(n & 1, rc, rs);                   /* quadrant swap */
    *cosp = ul_sel(n & 1, rs, rc);
}

/* s_sincosf.c for |y| < 120 (callers guarantee the range; the Payne-Hanek branch for huge
   arguments is not needed by the PLL).  Branch-free: for |y| < pi/4 the reduction yields
   n = 0, x - 0*pi/2 = x (exact) and sign +1, i.e. exactly the small branch's polynomial call,
   so one path serves both and a wave's lanes never split between them; |y| < 2^-12 selects
   (y, 1) at the end.  The quadrant's table is chosen by selects on its coefficients. */
UHSDR_LIBM_FN void ul_sincosf(float y, float* sinp, float* cosp)
{
    double x = y;
    const ul_sincos_t* p0 = ul_sincosf_table(0);
    const ul_sincos_t* p1 = ul_sincosf_table(1);
    /* reduce_fast, !TOINT_INTRINSICS */
    const double r = x * p0->hpi_inv;
    const int n = ((int32_t)r + 0x800000) >> 24;
    x = fma(-(double)n, p0->hpi, x);
    /* sign[n & 3] = +1, -1, -1, +1: negative when bit 1 of n + 1 is set */
    const double s = ul_asdouble(0x3ff0000000000000ull | ((uint64_t)((n + 1) & 2) << 62));
    ul_sincos_t q;
    const int h = (n & 2) != 0;
    q.c0 = ul_seld(h, p1->c0, p0->c0); q.c1 = ul_seld(h, p1->c1, p0->c1); q.s1 = ul_seld(h, p1->s1, p0->s1);
    q.c2 = ul_seld(h, p1->c2, p0->c2); q.s2 = ul_seld(h, p1->s2, p0->s2); q.c3 = ul_seld(h, p1->c3, p0->c3);
    q.s3 = ul_seld(h, p1->s3, p0->s3); q.c4 = ul_seld(h, p1->c4, p0->c4);
    float sv, cv;
    ul_sincosf_poly(x * s, x * x, &q, n, &sv, &cv);
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

UHSDR_LIBM_FN float ul_atan2f(float y, float x)
{
    const float tiny = 1.0e-30f, pi_o_4 = 7.8539818525e-01f, pi_o_2 = 1.5707963705e+00f,
                pi = 3.1415927410e+00f, pi_lo = -8.7422776573e-08f;
    const int32_t hx = (int32_t)ul_asuint(x), hy = (int32_t)ul_asuint(y);
    const int32_t ix = hx & 0x7fffffff, iy = hy & 0x7fffffff;
    const int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);      /* 2*sign(x) + sign(y) */
    /* Branch-free: fdlibm's main path (e_atan2f.c, the k / atanf / quadrant tail) runs for
     * every operand pair and the rare operands (NaN, zeros, infinities) select their results
     * after it, lowest precedence first, so the SAM PLL's per-sample chain stays one basic
     * block and consecutive samples' chains can interleave.  x = 1.0 (fdlibm: atanf(y)) needs
     * no case of its own: y / 1 = y, atanf is odd and the |y/x| > 2^26 override is skipped for
     * it -- pinned for every binary32 y by tools/libm_check.c "atan2x1". */
    const int32_t k = (iy - ix) >> 23;
    float z = ul_atanf(fabsf(y / x));
    z = ul_sel(hx < 0 && k < -26, 0.0f, z);                 /* |y|/x < -2^26 */
    z = ul_sel(k > 26 && hx != 0x3f800000, pi_o_2 + 0.5f * pi_lo, z);   /* |y/x| > 2^26 */
    const float zm = z - pi_lo;
    const float r2 = pi - zm, r3 = zm - pi;
    const float r1 = ul_asfloat(ul_asuint(z) ^ 0x80000000u);
    float r = ul_sel(m & 2, ul_sel(m & 1, r3, r2), ul_sel(m & 1, r1, z));
    const float pm_pi = ul_sel(m & 1, -pi - tiny, pi + tiny);   /* +-pi by sign(y) */
    const float pm_pi_o_2 = ul_sel(hy < 0, -pi_o_2 - tiny, pi_o_2 + tiny);
    r = ul_sel(iy == 0x7f800000, pm_pi_o_2, r);             /* y = +-inf, x finite */
    const float inf_inf = ul_sel(m & 2, ul_sel(m & 1, -3.0f * pi_o_4 - tiny, 3.0f * pi_o_4 + tiny),
                                 ul_sel(m & 1, -pi_o_4 - tiny, pi_o_4 + tiny));
    const float inf_fin = ul_sel(m & 2, pm_pi, ul_sel(m & 1, -0.0f, 0.0f));
    r = ul_sel(ix == 0x7f800000, ul_sel(iy == 0x7f800000, inf_inf, inf_fin), r);   /* x = +-inf */
    r = ul_sel(ix == 0, pm_pi_o_2, r);                      /* x = +-0 */
    r = ul_sel(iy == 0, ul_sel(m & 2, pm_pi, y), r);        /* y = +-0 */
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
