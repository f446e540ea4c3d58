/* Exhaustive check of two binary32 shortcuts in the TX ALC (tx_processor.c:202-212):
 *   (float)((double)q - 1.0) == q - 1.0f    for every non-negative binary32 q (q = |x| / ALC_KNEE)
 *   ((double)a < 0.001)       == (a < 0.001f) for every binary32 a
 * Build: gcc -O2 -ffp-contract=off tools/alc_check.c -o /tmp/alc_check && /tmp/alc_check */
#include <stdint.h>
#include <stdio.h>
#include <string.h>

static float f_of(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static uint32_t u_of(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

int main(void)
{
    unsigned long long bad1 = 0, bad2 = 0;
    for (uint64_t i = 0; i <= 0xFFFFFFFFull; ++i)
    {
        const float a = f_of((uint32_t)i);
        if (!(i >> 31))   /* non-negative q */
        {
            const float r0 = (float)((double)a - 1.0), r1 = a - 1.0f;
            if (u_of(r0) != u_of(r1) && !(r0 != r0 && r1 != r1)) ++bad1;
        }
        if (((double)a < 0.001) != (a < 0.001f)) ++bad2;
    }
    printf("q - 1: %llu mismatches; a < 0.001: %llu mismatches\n", bad1, bad2);
    return (bad1 || bad2) ? 1 : 0;
}
