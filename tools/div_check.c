/* Exhaustive check of uhsdr_tx.hip's alc_knee_div: for every non-negative finite binary32 x, the
 * FMA-corrected product q0 = x z, q = fma(fma(-q0, 30000, x), z, q0) against the IEEE quotient
 * x / 30000.  Mismatches are printed (the first five) and counted; all of them have quotients below
 * 2^-126 (subnormal), which the device code routes to the division itself.
 *   gcc -O2 -march=native -ffp-contract=off tools/div_check.c -o /tmp/div_check -lm && /tmp/div_check
 */
#include <stdio.h>
#include <stdint.h>
#include <string.h>
#include <math.h>
int main(void)
{
    const float y = 30000.0f, z = 1.0f / 30000.0f;
    unsigned long long bad = 0, n = 0;
    for (uint32_t u = 0; u < 0x7f800000u; ++u)
    {
        float a; memcpy(&a, &u, 4);
        const float q_ref = a / y;
        const float q0 = a * z;
        const float r = fmaf(-q0, y, a);
        const float q = fmaf(r, z, q0);
        uint32_t b1, b2; memcpy(&b1, &q_ref, 4); memcpy(&b2, &q, 4);
        if (b1 != b2) {
            if (q_ref >= 0x1p-126f) printf("NORMAL-RANGE mismatch a=%a\n", a); if (bad < 5) printf("mismatch a=%a ref=%a got=%a\n", a, q_ref, q); ++bad; }
        ++n;
    }
    printf("checked %llu, mismatches %llu\n", n, bad);
    return 0;
}
