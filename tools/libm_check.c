/* Pins uhsdr_amd/csrc/uhsdr_libm.h against the host's libm (glibc).
 *   libm_check sincos <stride>   every stride-th float in [0, 2*pi] and (-2*pi, 0)
 *   libm_check atan2 <count>     random + structured operand pairs
 *   libm_check asin <stride>     every stride-th float in [-1, 1] (and NaN operands past it)
 *   libm_check atan2x1 <stride>  every stride-th binary32 y (all signs) against atan2f(y, 1.0f)
 *   libm_check atanpos <stride>  ul_atanf_pos (atan2f's reduction) on every stride-th float in [0, inf]
 * Prints mismatches (first 10) and a summary line; exit status 1 on any mismatch. */
#define _GNU_SOURCE
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>
#include "../uhsdr_amd/csrc/uhsdr_libm.h"

static uint64_t rng = 0x9E3779B97F4A7C15ull;
static uint32_t next32(void) { rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17; return (uint32_t)(rng >> 16); }

int main(int argc, char** argv)
{
    if (argc < 3) return 2;
    long bad = 0, n = 0;
    if (!strcmp(argv[1], "sincos"))
    {
        const long stride = atol(argv[2]);
        const uint32_t hi = ul_asuint(6.2831855f);      /* > 2*pi as float */
        for (int sgn = 0; sgn < 2; ++sgn)
            for (uint64_t u = 0; u <= hi; u += stride)
            {
                const float y = ul_asfloat((uint32_t)u | (sgn ? 0x80000000u : 0));
                float s0, c0, s1, c1;
                sincosf(y, &s0, &c0);
                ul_sincosf(y, &s1, &c1);
                ++n;
                if (ul_asuint(s0) != ul_asuint(s1) || ul_asuint(c0) != ul_asuint(c1))
                {
                    if (bad++ < 10) printf("sincosf(%a): glibc %a %a, ours %a %a\n", y, s0, c0, s1, c1);
                }
            }
        printf("sincosf: %ld of %ld arguments differ\n", bad, n);
    }
    else if (!strcmp(argv[1], "asin"))
    {
        const long stride = atol(argv[2]);
        const uint32_t hi = ul_asuint(1.0f) + 16;
        for (int sgn = 0; sgn < 2; ++sgn)
            for (uint64_t u = 0; u <= hi; u += (u + stride > hi && u < hi) ? 1 : stride)
            {
                const float y = ul_asfloat((uint32_t)u | (sgn ? 0x80000000u : 0));
                const float r0 = asinf(y), r1 = ul_asinf(y);
                ++n;
                if (ul_asuint(r0) != ul_asuint(r1) && !(isnan(r0) && isnan(r1)))
                {
                    if (bad++ < 10) printf("asinf(%a): glibc %a, ours %a\n", y, r0, r1);
                }
            }
        printf("asinf: %ld of %ld arguments differ\n", bad, n);
    }
    else if (!strcmp(argv[1], "atanpos"))
    {
        const long stride = atol(argv[2]);
        for (uint64_t u = 0; u <= 0x7f800000u; u += stride)
        {
            const float a = ul_asfloat((uint32_t)u);
            const float r0 = atanf(a), r1 = ul_atanf_pos(a);
            ++n;
            if (ul_asuint(r0) != ul_asuint(r1))
            {
                if (bad++ < 10) printf("atanf(%a): glibc %a, ours %a\n", a, r0, r1);
            }
        }
        printf("atanf(a >= 0): %ld of %ld arguments differ\n", bad, n);
    }
    else if (!strcmp(argv[1], "atan2x1"))
    {
        const long stride = atol(argv[2]);
        for (uint64_t u = 0; u <= 0xffffffffull; u += stride)
        {
            const float y = ul_asfloat((uint32_t)u);
            const float r0 = atan2f(y, 1.0f), r1 = ul_atan2f(y, 1.0f);
            ++n;
            if (ul_asuint(r0) != ul_asuint(r1) && !(isnan(r0) && isnan(r1)))
            {
                if (bad++ < 10) printf("atan2f(%a, 1): glibc %a, ours %a\n", y, r0, r1);
            }
        }
        printf("atan2f(y, 1): %ld of %ld arguments differ\n", bad, n);
    }
    else
    {
        const long count = atol(argv[2]);
        const float special[] = { 0.0f, -0.0f, 1.0f, -1.0f, INFINITY, -INFINITY, NAN, 1e-30f, -1e-30f, 3e38f, -3e38f,
                                  1e-45f, -1e-45f, 0.5f, 2.0f, 1.5f, 0.4375f, 1.1875f, 2.4375f, 0.6875f };
        const int ns = sizeof special / sizeof special[0];
        for (long i = 0; i < count + ns * ns; ++i)
        {
            float y, x;
            if (i < ns * ns) { y = special[i / ns]; x = special[i % ns]; }
            else if (i % 3 == 0) { y = ul_asfloat(next32()); x = ul_asfloat(next32()); }   /* any bits */
            else
            {   /* FM-like operands: products of audio-range samples, similar magnitudes */
                const float a = (float)((int32_t)next32()) * 0x1p-31f, b = (float)((int32_t)next32()) * 0x1p-31f;
                const int e = (int)(next32() % 40) - 20;
                y = ldexpf(a, e); x = ldexpf(b, e + (int)(next32() % 9) - 4);
            }
            const float r0 = atan2f(y, x), r1 = ul_atan2f(y, x);
            ++n;
            if (ul_asuint(r0) != ul_asuint(r1) && !(isnan(r0) && isnan(r1)))
            {
                if (bad++ < 10) printf("atan2f(%a, %a): glibc %a, ours %a\n", y, x, r0, r1);
            }
        }
        printf("atan2f: %ld of %ld operand pairs differ\n", bad, n);
    }
    return bad != 0;
}
