"""One-off source transformation: move the CMSIS CFFT device primitives of uhsdr_spectrum.hip
into uhsdr_cfft.h and factor the transform out of spectrum_frame as cfft_core<L>."""
p = '/root/repo/uhsdr_amd/csrc/uhsdr_spectrum.hip'
s = open(p).read()

i0 = s.index('// complex index with one pad slot per 8:')
i1 = s.index('// Frame layout per wave (LDS):')
i2 = s.index('struct SpecParams\n')
prims = s[i0:i1]
geom = s[i1:i2]
s = s[:i0] + s[i2:]

old_core = s[s.index('    using G = SpecGeom<L>;\n    constexpr int K = G::K, NBF = G::NBF, R3 = G::R3;\n    const uhsdr_spectrum_plan* __restrict__ P = a.plan;\n    const float* __restrict__ twl = &P->tw_lane[0][0][0];'):
             s.index('    wave_sync();                                 // the frame is consumed: its LDS now stages the outputs')]
new_core = '''    using G = SpecGeom<L>;
    constexpr int NBF = G::NBF, R3 = G::R3;
    const uhsdr_spectrum_plan* __restrict__ P = a.plan;
    float2 y[R3][8];
    cfft_core<L>(z, X, tw, &P->tw_lane[0][0][0], lane, y);
'''
s = s.replace(old_core, new_core)
s = s.replace('#include "uhsdr_dsp.h"\n', '#include "uhsdr_dsp.h"\n#include "uhsdr_cfft.h"\n', 1)
open(p, 'w').write(s)

core_fn = '''
// arm_cfft_f32's transform (arm_cfft_f32.c:594-611) on the lane's positions z[k] = x[lane + 64k]:
// the first stages in registers, the middle radix-8 stage through the wave's LDS frame X
// (padded complex, SpecGeom<L>::FRAME floats), the last stage into registers.  y[r][k] is the
// in-place result at position 8q + k, q = lane + 64r (q < NBF); the reference's bit reversal
// maps position p to bin plan->iperm[p].  X is free again when this returns.
template <int L>
__device__ __forceinline__ void cfft_core(float2 (&z)[SpecGeom<L>::K], float2* X, const float* __restrict__ tw,
                                          const float* __restrict__ twl, int lane, float2 (&y)[SpecGeom<L>::R3][8])
{
    using G = SpecGeom<L>;
    constexpr int K = G::K, NBF = G::NBF, R3 = G::R3;
    if constexpr (L == 1024)
    {
        split_by2_regs(z, tw, lane);
        dft8_lane(z, twl, lane);                 // radix-8 stage span 512 of each half (j = lane)
        dft8_lane(z + 8, twl, lane);
    }
    else if constexpr (L == 512)
    {
        dft8_lane(z, twl, lane);
    }
    else
    {
        split_by4_regs(z, twl, lane);
    }
    wave_sync();                                 // earlier LDS readers (scratch / last frame) done
#pragma unroll
    for (int k = 0; k < K; ++k) X[padp(lane + 64 * k)] = z[k];
    wave_sync();
    for (int q = lane; q < NBF; q += 64)
    {
        constexpr int PER = G::SUBN / 8;
        const int sub = q / PER, rr = q % PER;
        const int j = rr & 7;
        const int base = sub * G::SUBN + j + 64 * (rr >> 3);
        float2 v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = X[padp(base + 8 * k)];
        dft8(v, tw, j * G::TMID);
#pragma unroll
        for (int k = 0; k < 8; ++k) X[padp(base + 8 * k)] = v[k];
    }
    wave_sync();
#pragma unroll
    for (int r = 0; r < R3; ++r)
    {
        const int q = lane + 64 * r;
        if (q < NBF)
        {
#pragma unroll
            for (int k = 0; k < 8; ++k) y[r][k] = X[padp(8 * q + k)];
            dft8(y[r], tw, 0);
        }
    }
}
'''

hdr = '''/*
 * CMSIS-DSP V1.4.5 arm_cfft_f32 on one 64-lane wave, bit-identical to the reference's radix-8
 * code for fft_len 256 / 512 / 1024 (CMSIS TransformFunctions/arm_cfft_f32.c:207-632,
 * arm_cfft_radix8_f32.c:130-383).  Shared by the spectrum display kernels (uhsdr_spectrum.hip)
 * and the arm_cfft_f32 shim (uhsdr_cmsis.hip).  Twiddles and the bit-reversal permutation come
 * from uhsdr_spectrum_plan (host setup, uhsdr_setup.c).
 */
#ifndef UHSDR_CFFT_H
#define UHSDR_CFFT_H

#include <hip/hip_runtime.h>
#include "uhsdr_dsp.h"

''' + prims + geom + core_fn + '''
#endif /* UHSDR_CFFT_H */
'''
open('/root/repo/uhsdr_amd/csrc/uhsdr_cfft.h', 'w').write(hdr)
print("ok")
