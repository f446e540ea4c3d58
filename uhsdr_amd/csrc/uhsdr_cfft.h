/*
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

// complex index with one pad slot per 8: the strided butterfly reads of every stage hit
// distinct LDS banks (at most the two passes a 64-lane ds_read_b64 needs anyway)
__device__ __forceinline__ int padp(int p) { return p + (p >> 3); }

// arm_radix8_butterfly_f32 butterfly (CMSIS arm_cfft_radix8_f32.c:130-383) on eight complex
// values in registers.  The reference's two loop bodies (twiddle-free first group :149-221,
// twiddled groups :228-372) form the same eight values X_k with the same sequence of adds; the
// twiddled groups then rotate X_k, k >= 1, by twiddle[k * tstep] as (c*re + s*im, c*im - s*re).
__device__ __forceinline__ void dft8(float2* z, const float* __restrict__ tw, int tstep)
{
    const float C81 = 0.70710678118f;
    float sr[4], dr[4], si[4], di[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
    {
        sr[k] = z[k].x + z[k + 4].x;
        dr[k] = z[k].x - z[k + 4].x;
        si[k] = z[k].y + z[k + 4].y;
        di[k] = z[k].y - z[k + 4].y;
    }
    const float a = sr[0] - sr[2], b = sr[0] + sr[2], cc = sr[1] - sr[3], d = sr[1] + sr[3];
    const float ai = si[0] - si[2], bi = si[0] + si[2], ci = si[1] - si[3], dd = si[1] + si[3];
    z[0] = make_float2(b + d, bi + dd);
    z[4] = make_float2(b - d, bi - dd);
    z[2] = make_float2(a + ci, ai - cc);
    z[6] = make_float2(a - ci, ai + cc);
    const float u = (dr[1] - dr[3]) * C81, v = (dr[1] + dr[3]) * C81;
    const float ui = (di[1] - di[3]) * C81, vi = (di[1] + di[3]) * C81;
    const float e0 = dr[0] - u, e1 = dr[0] + u, f0 = dr[2] - v, f1 = dr[2] + v;
    const float g0 = di[0] - ui, g1 = di[0] + ui, h0 = di[2] - vi, h1 = di[2] + vi;
    z[1] = make_float2(e1 + h1, g1 - f1);
    z[7] = make_float2(e1 - h1, g1 + f1);
    z[5] = make_float2(e0 + h0, g0 - f0);
    z[3] = make_float2(e0 - h0, g0 + f0);
    if (tstep)
    {
#pragma unroll
        for (int k = 1; k < 8; ++k)
        {
            const float2 t = *(const float2*)(tw + 2 * k * tstep);
            const float p1 = t.x * z[k].x, p2 = t.y * z[k].y, p3 = t.x * z[k].y, p4 = t.y * z[k].x;
            z[k] = make_float2(p1 + p2, p3 - p4);
        }
    }
}

// the same butterfly with per-lane twiddles (plan->tw_lane[k][lane], coalesced); lane 0 of a
// first stage is the reference's twiddle-free group j = 0
__device__ __forceinline__ void dft8_lane(float2* z, const float* __restrict__ twl, int lane)
{
    dft8(z, nullptr, 0);
    if (lane)
    {
#pragma unroll
        for (int k = 1; k < 8; ++k)
        {
            const float2 t = *(const float2*)(twl + k * 128 + 2 * lane);
            const float p1 = t.x * z[k].x, p2 = t.y * z[k].y, p3 = t.x * z[k].y, p4 = t.y * z[k].x;
            z[k] = make_float2(p1 + p2, p3 - p4);
        }
    }
}

__device__ __forceinline__ float2 rot_fwd(float2 x, float2 t)
{
    const float m0 = x.x * t.x, m1 = x.y * t.y, m2 = x.y * t.x, m3 = x.x * t.y;
    return make_float2(m0 + m1, m2 - m3);
}

// arm_cfft_radix8by2_f32 split (arm_cfft_f32.c:207-317), n = 1024, on the lane's 16 values
// z[k] = x[lane + 64k]: column a = lane + 64m pairs x[a], x[a+256] with x[a+512], x[a+768]
__device__ __forceinline__ void split_by2_regs(float2 (&z)[16], const float* __restrict__ tw, int lane)
{
#pragma unroll
    for (int m = 0; m < 4; ++m)
    {
        const float2 x1 = z[m], x3 = z[m + 4], x2 = z[m + 8], x4 = z[m + 12];
        const float2 t2 = make_float2(x1.x - x2.x, x1.y - x2.y);
        const float2 t4 = make_float2(x4.x - x3.x, x4.y - x3.y);
        z[m] = make_float2(x1.x + x2.x, x1.y + x2.y);
        z[m + 4] = make_float2(x3.x + x4.x, x3.y + x4.y);
        const float2 t = *(const float2*)(tw + 2 * (lane + 64 * m));
        z[m + 8] = rot_fwd(t2, t);
        const float m0 = t4.x * t.y, m1 = t4.y * t.x, m2 = t4.y * t.y, m3 = t4.x * t.x;
        z[m + 12] = make_float2(m0 - m1, m2 + m3);
    }
}

// arm_cfft_radix8by4_f32 split (arm_cfft_f32.c:319-557), n = 256, row r = lane of the four
// quarters (z[k] = x[r + 64k]): rows 0..32 are the reference's TOP rows t = r (t = 0
// untwiddled, t = 32 its MIDDLE block), rows 33..63 its BOTTOM rows 64 - t with the twiddles of t
__device__ __forceinline__ void split_by4_regs(float2 (&z)[4], const float* __restrict__ twl, int lane)
{
    constexpr int Q = 64;
    const bool top = lane <= Q / 2;
    const int t = top ? lane : Q - lane;
    const float2 x1 = z[0], x2 = z[1], x3 = z[2], x4 = z[3];
    const float s13r = x1.x + x3.x, d13r = x1.x - x3.x;
    const float s13i = x1.y + x3.y, d13i = x1.y - x3.y;
    // twiddles t, 2t, 3t of the row (plan->tw_lane[1..3][lane])
    const float2 w2 = *(const float2*)(twl + 128 + 2 * lane), w3 = *(const float2*)(twl + 256 + 2 * lane),
                 w4 = *(const float2*)(twl + 384 + 2 * lane);
    z[0] = make_float2(s13r + x2.x + x4.x, s13i + x2.y + x4.y);
    if (top)
    {
        const float2 t2 = make_float2(d13r + x2.y - x4.y, d13i - x2.x + x4.x);
        const float2 t3 = make_float2(s13r - x2.x - x4.x, s13i - x2.y - x4.y);
        const float2 t4 = make_float2(d13r - x2.y + x4.y, d13i + x2.x - x4.x);
        if (t == 0) { z[1] = t2; z[2] = t3; z[3] = t4; }
        else { z[1] = rot_fwd(t2, w2); z[2] = rot_fwd(t3, w3); z[3] = rot_fwd(t4, w4); }
    }
    else
    {
        const float u2r = x2.y - x4.y + d13r;
        const float u2i = x1.y - x3.y - x2.x + x4.x;
        const float u3r = s13r - x2.x - x4.x;
        const float u3i = s13i - x2.y - x4.y;
        const float u4r = x2.y - x4.y - d13r;
        const float u4i = x4.x - x2.x - d13i;
        {
            const float m0 = u2i * w2.y, m1 = u2r * w2.x, m2 = u2r * w2.y, m3 = u2i * w2.x;
            z[1] = make_float2(m2 + m3, m0 - m1);
        }
        {
            const float m0 = -u3i * w3.x, m1 = u3r * w3.y, m2 = u3r * w3.x, m3 = u3i * w3.y;
            z[2] = make_float2(m3 - m2, m0 - m1);
        }
        {
            const float m0 = u4i * w4.y, m1 = u4r * w4.x, m2 = u4r * w4.y, m3 = u4i * w4.x;
            z[3] = make_float2(m2 + m3, m0 - m1);
        }
    }
}

// Frame layout per wave (LDS): the frame as padded complex; before the frame is written there,
// the same words hold the auto-I/Q products of this segment ([3][32][33]: sample-in-call major,
// so the per-call sequential sums of 32 lanes read consecutive words), then T = [5][NCALL]
// sums / factors.
template <int L>
struct SpecGeom
{
    static constexpr int K = L / 64;                       // positions per lane before the LDS stages
    static constexpr int NCALL = L / BLK;
    static constexpr int NBF = L / 8;                      // butterflies per radix-8 stage
    static constexpr int R3 = (NBF + 63) / 64;             // final-stage butterflies per lane
    static constexpr int SUBN = L == 256 ? 64 : 512;       // sub-array of the middle radix-8 stage
    static constexpr int TMID = L == 1024 ? 16 : (L == 512 ? 8 : 4);   // its twiddle modifier
    static constexpr int FRAME = 2 * (L + L / 8);          // floats, padded complex
    static constexpr int PROD = 32 * 33;                   // one product array, [i][call], padded
    static constexpr int SCRATCH = 3 * PROD;
    static constexpr int REGION = FRAME > SCRATCH ? FRAME : SCRATCH;
    static constexpr int PITCH = REGION + 5 * NCALL + 4;   // floats per wave
};


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

#endif /* UHSDR_CFFT_H */
