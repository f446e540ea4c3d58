// MI355X (gfx950) spectrum display of the UHSDR firmware, batched over channels.
//
// Per channel and per fft_len input samples (one display frame), bit-identical to the firmware
// built for x86:
//   producer  convert x 2^-16, I/Q correction (manual / auto)   audio_driver.c:2660-2685, 2254-2316
//             into the interleaved [Q, I] ring                    audio_driver.c:1811-1851
//   consumer  Hann window per float of the ring                  ui_spectrum.c:402-414
//             arm_cfft_f32 forward + bit reversal                CMSIS arm_cfft_f32.c:574-632,
//                                                                arm_cfft_radix8_f32.c:130-383,
//                                                                arm_bitreversal2.S:136-180
//             arm_cmplx_mag_f32, IIR average clamped at 1        ui_spectrum.c:1405, 1432-1446
//
// One wave per channel (four per workgroup, no workgroup barrier): the frame lives in LDS
// (2 * fft_len floats), every FFT stage is one pass of independent butterflies over it, the
// running average sits in registers (fft_len / 64 bins per lane) for the whole launch.  Frames
// that straddle calls are carried in HBM.  HBM traffic per sample: 8 B I/Q in + 4 B per output
// array written; the state (average, carry) moves once per launch.

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>
#include <stdlib.h>
#include <math.h>
#include <type_traits>
#include "uhsdr_internal.h"
#include "uhsdr_dsp.h"
#include "uhsdr_cfft.h"

namespace {

constexpr int SPEC_WAVES = 4;   // waves (channels) per workgroup

struct SpecArgs
{
    const uhsdr_spectrum_plan* plan;
    const int2* iq;          // [C][ld] IqSample_t
    const float2* zq;        // zoom: [C][ld] {Q, I} from spectrum_zoom (corrected, translated, decimated)
    float* teta;             // [3][C] auto I/Q correction low-pass state
    float* avg_state;        // [C][L] sd.FFT_AVGData
    float* carry;            // [C][2L] windowed ring of an incomplete frame (positions < fill)
                             // avg_state is kept in butterfly-output order (bins via plan->iperm)
    float* mag;              // optional [C][F][L]
    float* avg;              // optional [C][F][L]
    int C, N, ld, F, fill0, lds_pitch;
};

__device__ __forceinline__ float sign_new(float x) { return (x < 0) ? -1.0f : ((x > 0) ? 1.0f : 0.0f); }

struct SpecParams
{
    const float* win;
    float gi, gq, ph;
};

// Producer side for the lane's positions p = lane + 64k of one segment [fill, end) of a frame:
// convert (audio_driver.c:2660-2685), I/Q correction (:2254-2316; the auto variant's per-call
// statistics summed in sample order through LDS), window (ui_spectrum.c:402-414).  PART: the
// segment does not start at 0 (positions below fill hold the carried, already windowed values)
// or does not reach L.  Positions outside [fill, end) are left alone.
template <int L, bool PART, bool AUTO, bool ZM = false, typename SrcT = typename std::conditional<ZM, float2, int2>::type>
__device__ __forceinline__ void produce(float2 (&z)[SpecGeom<L>::K], const SrcT* __restrict__ src, int fill, int end,
                                        const SpecParams& sp, float* S, float* T, float& o1, float& o2, float& o3,
                                        int lane)
{
    using G = SpecGeom<L>;
    constexpr int K = G::K, NCALL = G::NCALL;
    constexpr bool FORMULA = L == 1024;          // plan->window_formula (checked on the host)
    auto in_seg = [&](int p) { return !PART || (p >= fill && p < end); };
#pragma unroll
    for (int k = 0; k < K; ++k)
    {
        const int p = lane + 64 * k;
        if (in_seg(p))
        {
            if constexpr (ZM) z[k] = src[p - fill];          // zoom ring samples, ready to window
            else
            {
                const int2 v = src[p - fill];
                float I = (float)v.x, Q = (float)v.y;
                I = I * IQ_BIT_SCALE_DOWN;
                Q = Q * IQ_BIT_SCALE_DOWN;
                z[k] = make_float2(Q, I);
            }
        }
    }
    if constexpr (AUTO)
    {
        // per-call sums of sgn(I)Q, sgn(I)I, sgn(Q)Q in sample order (audio_driver.c:2274-2285):
        // the products are exact, so they are formed here and summed sequentially per call
#pragma unroll
        for (int k = 0; k < K; ++k)
        {
            const int p = lane + 64 * k;
            if (in_seg(p))
            {
                const int at = (p & 31) * 33 + (p >> 5);      // transposed, padded: [i][33]
                const float Q = z[k].x, I = z[k].y;
                S[at] = sign_new(I) * Q;
                S[G::PROD + at] = sign_new(I) * I;
                S[2 * G::PROD + at] = sign_new(Q) * Q;
            }
        }
        wave_sync();
        const int j = (fill >> 5) + lane;
        if (j < (end >> 5))
        {
            float t1 = 0.0f, t2 = 0.0f, t3 = 0.0f;
#pragma unroll 4
            for (int i = 0; i < BLK; ++i)
            {
                const int at = i * 33 + j;
                t1 += S[at];
                t2 += S[G::PROD + at];
                t3 += S[2 * G::PROD + at];
            }
            T[j] = t1; T[NCALL + j] = t2; T[2 * NCALL + j] = t3;
        }
        wave_sync();
        // the low-pass recursion (:2288-2290) is the only serial part: uniform in all lanes, each
        // lane keeping the state after its own call; the factors (:2292-2303) then in parallel
        float m1 = 0.0f, m2 = 0.0f, m3 = 0.0f;
#pragma unroll 1
        for (int jj = fill >> 5; jj < (end >> 5); ++jj)
        {
            o1 = (float)(-0.003 * (double)(T[jj] / (float)BLK) + 0.997 * (double)o1);
            o2 = (float)(0.003 * (double)(T[NCALL + jj] / (float)BLK) + 0.997 * (double)o2);
            o3 = (float)(0.003 * (double)(T[2 * NCALL + jj] / (float)BLK) + 0.997 * (double)o3);
            if (jj == j) { m1 = o1; m2 = o2; m3 = o3; }
        }
        if (j < (end >> 5))
        {
            const float t1 = m1, t2 = m2, t3 = m3;
            const float M_c1 = (t2 != 0.0f) ? t1 / t2 : 0.0f;
            float help = (t2 * t2);
            if (help > 0.0f) help = (t3 * t3 - t1 * t1) / help;
            const float M_c2 = (help > 0.0f) ? sqrtf(help) : 1.0f;
            T[3 * NCALL + j] = M_c1;
            T[4 * NCALL + j] = M_c2;
        }
        wave_sync();
        __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int k = 0; k < K; ++k)
    {
        const int p = lane + 64 * k;
        if (in_seg(p))
        {
            float Q = z[k].x, I = z[k].y;
            if constexpr (ZM) {}
            else if constexpr (!AUTO)
            {
                I = I * sp.gi;
                Q = Q * sp.gq;
                // AudioDriver_IQPhaseAdjust (:1776-1801) as selects on the uniform sign of ph
                const float qa = Q + I * sp.ph, ia = I + Q * sp.ph;
                Q = sp.ph < 0 ? qa : Q;
                I = sp.ph > 0 ? ia : I;
            }
            else
            {
                Q += T[3 * NCALL + (p >> 5)] * I;
                I = I * T[4 * NCALL + (p >> 5)];
            }
            const float2 wv = *(const float2*)(sp.win + 2 * p);
            if constexpr (FORMULA) z[k] = make_float2(0.5f * (wv.x * Q), 0.5f * (wv.y * I));
            else z[k] = make_float2(Q * wv.x, I * wv.y);
        }
        if constexpr (AUTO)
            if (k % 4 == 3) __builtin_amdgcn_sched_barrier(0);   // bound the loads in flight
    }
}

template <int L>
__device__ __forceinline__ SpecParams spec_params(const uhsdr_spectrum_plan* __restrict__ P)
{
    SpecParams sp;
    sp.win = P->window;
    sp.gi = P->iq_gain_i; sp.gq = P->iq_gain_q; sp.ph = P->iq_phase_balance;
    return sp;
}

// One display frame from the produced positions z[k] = x[lane + 64k]: arm_cfft_f32's first
// stages in registers, the middle radix-8 stage through LDS, the last stage into registers,
// the bit reversal as the output bin of each butterfly result, then magnitude and average
// (ui_spectrum.c:1405, 1432-1446).
template <int L>
__device__ __forceinline__ void spectrum_frame(float2 (&z)[SpecGeom<L>::K], float2* X, const float* __restrict__ tw,
                                               float (&av)[SpecGeom<L>::R3][8], float f, const SpecArgs& a, int c,
                                               int frame, int lane)
{
    using G = SpecGeom<L>;
    constexpr int NBF = G::NBF, R3 = G::R3;
    const uhsdr_spectrum_plan* __restrict__ P = a.plan;
    float2 y[R3][8];
    cfft_core<L>(z, X, tw, &P->tw_lane[0][0][0], lane, y);
    wave_sync();                                 // the frame is consumed: its LDS now stages the outputs
    float* O = (float*)X;                        // [2][L] in bin order
#pragma unroll
    for (int r = 0; r < R3; ++r)
    {
        const int q = lane + 64 * r;
        if (q < NBF)
        {
            const uint4 bins = *(const uint4*)(P->iperm + 8 * q);   // 8 x u16
            const uint32_t bw[4] = { bins.x, bins.y, bins.z, bins.w };
#pragma unroll
            for (int k = 0; k < 8; ++k)
            {
                const float mg = sqrtf((y[r][k].x * y[r][k].x) + (y[r][k].y * y[r][k].y));
                float s = av[r][k];
                const float old = s * f;
                s = s - old;
                const float add = mg * f;
                s = add + s;
                if (s < 1) s = 1;
                av[r][k] = s;
                const int bin = (bw[k >> 1] >> (16 * (k & 1))) & 0xffff;
                O[bin] = mg;
                O[L + bin] = s;
            }
        }
    }
    wave_sync();
    float* __restrict__ mo = a.mag ? a.mag + ((size_t)c * a.F + frame) * L : nullptr;
    float* __restrict__ ao = a.avg ? a.avg + ((size_t)c * a.F + frame) * L : nullptr;
#pragma unroll
    for (int m = 0; m < L / 256; ++m)
    {
        const int i = 4 * (lane + 64 * m);
        if (mo) *(float4*)(mo + i) = *(const float4*)(O + i);
        if (ao) *(float4*)(ao + i) = *(const float4*)(O + L + i);
    }
    wave_sync();                                 // staged outputs read before the next frame lands
}

// A call that completes no frame (frames_per_call < fft_len): produce into the carried ring.
template <int L, bool AUTO, bool ZM>
__global__ void __launch_bounds__(64 * SPEC_WAVES) spectrum_accumulate(SpecArgs a)
{
    extern __shared__ __attribute__((aligned(16))) float smem[];
    using G = SpecGeom<L>;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int c = blockIdx.x * SPEC_WAVES + w;
    if (c >= a.C) return;
    float* S = smem + w * a.lds_pitch;
    const SpecParams sp = spec_params<L>(a.plan);
    float o1 = 0.0f, o2 = 0.0f, o3 = 0.0f;
    if (AUTO) { o1 = a.teta[c]; o2 = a.teta[a.C + c]; o3 = a.teta[2 * a.C + c]; }
    const int fill = a.fill0, end = a.fill0 + a.N;
    float2 z[G::K];
    if constexpr (ZM) produce<L, true, false, true>(z, a.zq + (size_t)c * a.ld, fill, end, sp, S, S + G::REGION, o1, o2, o3, lane);
    else produce<L, true, AUTO>(z, a.iq + (size_t)c * a.ld, fill, end, sp, S, S + G::REGION, o1, o2, o3, lane);
    float2* __restrict__ carry = (float2*)a.carry + (size_t)c * L;
#pragma unroll
    for (int k = 0; k < G::K; ++k)
    {
        const int p = lane + 64 * k;
        if (p >= fill && p < end) carry[p] = z[k];
    }
    if (AUTO && lane == 0) { a.teta[c] = o1; a.teta[a.C + c] = o2; a.teta[2 * a.C + c] = o3; }
}

// Calls that complete frames: every segment ends a frame; the first may start from the carry.
template <int L, bool AUTO, bool ZM>
__global__ void __launch_bounds__(64 * SPEC_WAVES) spectrum_frames(SpecArgs a)
{
    extern __shared__ __attribute__((aligned(16))) float smem[];
    using G = SpecGeom<L>;
    constexpr int K = G::K, NBF = G::NBF, R3 = G::R3;
    const uhsdr_spectrum_plan* __restrict__ P = a.plan;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int c = blockIdx.x * SPEC_WAVES + w;
    if (c >= a.C) return;                        // whole wave; no workgroup barrier below
    float* S = smem + w * a.lds_pitch;           // auto-I/Q products, then the frame
    float2* X = (float2*)S;
    float* T = S + G::REGION;                    // used only with auto I/Q correction
    const float* __restrict__ tw = P->twiddle;
    const SpecParams sp = spec_params<L>(P);
    const float f = P->filt_factor;
    const int C = a.C, N = a.N;
    const size_t row = (size_t)c * L;

    // the final-stage outputs this lane owns: positions 8q + k, q = lane + 64r; their running
    // averages stay in registers (state kept in position order, bins via plan->iperm)
    float av[R3][8];
#pragma unroll
    for (int r = 0; r < R3; ++r)
    {
        const int q = lane + 64 * r;
#pragma unroll
        for (int k = 0; k < 8; ++k) av[r][k] = q < NBF ? a.avg_state[row + 8 * q + k] : 0.0f;
    }
    float o1 = 0.0f, o2 = 0.0f, o3 = 0.0f;
    if (AUTO) { o1 = a.teta[c]; o2 = a.teta[C + c]; o3 = a.teta[2 * C + c]; }
    using SrcT = typename std::conditional<ZM, float2, int2>::type;
    const SrcT* __restrict__ src;
    if constexpr (ZM) src = a.zq + (size_t)c * a.ld;
    else src = a.iq + (size_t)c * a.ld;

    int n0 = 0, frame = 0;
    if (a.fill0)
    {
        // ---- the frame begun in earlier calls ----
        const float2* __restrict__ carry = (const float2*)a.carry + (size_t)c * L;
        float2 z[K];
#pragma unroll
        for (int k = 0; k < K; ++k)
        {
            const int p = lane + 64 * k;
            z[k] = carry[p < a.fill0 ? p : 0];
        }
        produce<L, true, AUTO && !ZM, ZM>(z, src, a.fill0, L, sp, S, T, o1, o2, o3, lane);
        spectrum_frame<L>(z, X, tw, av, f, a, c, frame, lane);
        n0 = L - a.fill0;
        ++frame;
    }
    for (; n0 < N; n0 += L, ++frame)
    {
        // per-frame reloads (L1-resident) instead of loop-invariant registers: keeps the window
        // and the twiddles from being hoisted out of the frame loop into VGPRs
        SpecParams spf = sp;
        const float* __restrict__ twf = tw;
        asm volatile("" : "+s"(spf.win), "+s"(twf));
        float2 z[K];
        produce<L, false, AUTO && !ZM, ZM>(z, src + n0, 0, L, spf, S, T, o1, o2, o3, lane);
        spectrum_frame<L>(z, X, twf, av, f, a, c, frame, lane);
    }
#pragma unroll
    for (int r = 0; r < R3; ++r)
    {
        const int q = lane + 64 * r;
        if (q < NBF)
#pragma unroll
            for (int k = 0; k < 8; ++k) a.avg_state[row + 8 * q + k] = av[r][k];
    }
    if (AUTO && lane == 0) { a.teta[c] = o1; a.teta[C + c] = o2; a.teta[2 * C + c] = o3; }
}


// ---- zoom producer (AudioDriver_SpectrumZoomProcessSamples, audio_driver.c:1860-1909) ----
// One lane per channel walks the launch's 32-frame calls in order, each exactly as the ISR:
// convert, I/Q correction (:2254-2316), FreqShift (freq_shift.c:275-334; the ring sees the
// translated I/Q, :2694-2705), IIR_biquad_Zoom_FFT_I/_Q (arm_biquad_cascade_df1_f32, 4 stages)
// and DECIMATE_ZOOM_FFT_I/_Q (arm_fir_decimate_f32 by 2^magnify), writing the BLK / 2^magnify
// ring samples {Q, I} of every call to zq[c][*].  All recursions are per channel and sequential
// (a lane pair per channel: I and Q); state is field-major [field][C], so loads and stores
// coalesce.
struct ZoomState
{
    float* bq_i;     // [16][C]  x1 x2 y1 y2 per stage (IIR_biquad_Zoom_FFT_I pState)
    float* bq_q;     // [16][C]
    float* dec_i;    // [3][C]   decimator history (numTaps - 1)
    float* dec_q;    // [3][C]
    float* osc;      // [2][C]   FreqShift_Approx oscillator {vi, vq}
};

struct ZoomArgs
{
    const uhsdr_spectrum_plan* plan;
    const int2* iq;  // [C][N]
    float2* zq;      // [C][N / D]
    float* teta;     // [3][C]
    ZoomState s;
    int C, N;
};

constexpr int ZOOM_TAPS = 4;        // every FirZoomFFTDecimate entry (checked on the host)

template <int D>
__global__ void __launch_bounds__(64) spectrum_zoom(ZoomArgs a)
{
    const uhsdr_spectrum_plan* __restrict__ P = a.plan;
    // two lanes per channel: both run the correction / translation (they mix I and Q), then
    // lane q = 0 filters and decimates I, lane q = 1 Q -- twice the waves of lane == channel,
    // half the recursive work per lane
    const int t = blockIdx.x * 64 + threadIdx.x;
    const int c = t >> 1, q = t & 1;
    if (c >= a.C) return;
    const int C = a.C;
    constexpr int T = ZOOM_TAPS;
    const bool auto_iq = P->iq_auto_correction != 0;
    const int shift = P->freq_shift_hz != 0 ? P->shift_kind : 0;
    float* __restrict__ bq_g = q ? a.s.bq_q : a.s.bq_i;
    float* __restrict__ dec_g = q ? a.s.dec_q : a.s.dec_i;
    float bq[16], h[T - 1];
#pragma unroll
    for (int k = 0; k < 16; ++k) bq[k] = bq_g[k * C + c];
#pragma unroll
    for (int k = 0; k < T - 1; ++k) h[k] = dec_g[k * C + c];
    float vi = a.s.osc[c], vq = a.s.osc[C + c];
    float o1 = a.teta[c], o2 = a.teta[C + c], o3 = a.teta[2 * C + c];
    const int4* __restrict__ src = (const int4*)(a.iq + (size_t)c * a.N);
    float* __restrict__ dst = (float*)(a.zq + (size_t)c * (a.N / D)) + (q ? 0 : 1);   // {Q, I} pairs
    for (int n0 = 0; n0 < a.N; n0 += BLK)
    {
        float ib[BLK], qb[BLK];
#pragma unroll
        for (int j = 0; j < BLK / 2; ++j)
        {
            const int4 v = src[n0 / 2 + j];
            ib[2 * j] = ((float)v.x) * IQ_BIT_SCALE_DOWN; qb[2 * j] = ((float)v.y) * IQ_BIT_SCALE_DOWN;
            ib[2 * j + 1] = ((float)v.z) * IQ_BIT_SCALE_DOWN; qb[2 * j + 1] = ((float)v.w) * IQ_BIT_SCALE_DOWN;
        }
        if (!auto_iq)
        {
            const float gi = P->iq_gain_i, gq = P->iq_gain_q, ph = P->iq_phase_balance;
#pragma unroll
            for (int i = 0; i < BLK; ++i) { ib[i] = ib[i] * gi; qb[i] = qb[i] * gq; }
            if (ph < 0)
            {
#pragma unroll
                for (int i = 0; i < BLK; ++i) { const float e = ib[i] * ph; qb[i] = qb[i] + e; }
            }
            else if (ph > 0)
            {
#pragma unroll
                for (int i = 0; i < BLK; ++i) { const float e = qb[i] * ph; ib[i] = ib[i] + e; }
            }
        }
        else
        {
            float t1 = 0.0f, t2 = 0.0f, t3 = 0.0f;
#pragma unroll
            for (int i = 0; i < BLK; ++i)
            {
                t1 += sign_new(ib[i]) * qb[i];
                t2 += sign_new(ib[i]) * ib[i];
                t3 += sign_new(qb[i]) * qb[i];
            }
            t1 = (float)(-0.003 * (double)(t1 / (float)BLK) + 0.997 * (double)o1);
            t2 = (float)(0.003 * (double)(t2 / (float)BLK) + 0.997 * (double)o2);
            t3 = (float)(0.003 * (double)(t3 / (float)BLK) + 0.997 * (double)o3);
            const float M_c1 = (t2 != 0.0f) ? t1 / t2 : 0.0f;
            float help = (t2 * t2);
            if (help > 0.0f) help = (t3 * t3 - t1 * t1) / help;
            const float M_c2 = (help > 0.0f) ? sqrtf(help) : 1.0f;
            o1 = t1; o2 = t2; o3 = t3;
#pragma unroll
            for (int i = 0; i < BLK; ++i) { qb[i] += M_c1 * ib[i]; ib[i] = ib[i] * M_c2; }
        }
        if (shift)
        {
            float* ip = P->shift_up ? ib : qb;
            float* qp = P->shift_up ? qb : ib;
            if (shift == 1)
            {
#pragma unroll
                for (int i = 0; i < BLK; i += 4)   // FreqShift_QuarterFs, freq_shift.c:219-262
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
                const float oc = P->osc_cos, os = P->osc_sin;
#pragma unroll
                for (int i = 0; i < BLK; ++i)      // FreqShift_Approx, freq_shift.c:57-101
                {
                    const float oq = (vq * oc) - (vi * os);
                    const float oi = (vi * oc) + (vq * os);
                    const float qt = qp[i], it = ip[i];
                    qp[i] = (qt * oq) - (it * oi);
                    ip[i] = (it * oq) + (qt * oi);
                    vq = oq; vi = oi;
                }
                const float g = (3 - ((vq * vq) + (vi * vi))) / 2;
                vq = g * vq; vi = g * vi;
            }
        }
        // IIR_biquad_Zoom_FFT_I / _Q: stage by stage over the call (arm_biquad_cascade_df1_f32)
        float x[BLK];
#pragma unroll
        for (int i = 0; i < BLK; ++i) x[i] = q ? qb[i] : ib[i];
#pragma unroll
        for (int st = 0; st < 4; ++st)
        {
            const float* cf = P->zoom_biquad + 5 * st;
#pragma unroll
            for (int i = 0; i < BLK; ++i)
                x[i] = biquad_step(x[i], bq[4 * st], bq[4 * st + 1], bq[4 * st + 2], bq[4 * st + 3], cf);
        }
        // DECIMATE_ZOOM_FFT_I / _Q: y[m] = sum_k c[k] * w[m D + k], w = [T-1 history | call]
#pragma unroll
        for (int m = 0; m < BLK / D; ++m)
        {
            float sum = 0.0f;
#pragma unroll
            for (int k = 0; k < T; ++k)
            {
                const int j = m * D + k - (T - 1);      // < 0: history
                sum += (j < 0 ? h[j + T - 1] : x[j]) * P->zoom_fir[k];
            }
            dst[2 * (n0 / D + m)] = sum;
        }
#pragma unroll
        for (int k = 0; k < T - 1; ++k) h[k] = x[BLK - (T - 1) + k];
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) bq_g[k * C + c] = bq[k];
#pragma unroll
    for (int k = 0; k < T - 1; ++k) dec_g[k * C + c] = h[k];
    if (q == 0)
    {
        a.s.osc[c] = vi; a.s.osc[C + c] = vq;
        a.teta[c] = o1; a.teta[C + c] = o2; a.teta[2 * C + c] = o3;
    }
}

} // namespace

struct uhsdr_spectrum_s
{
    uhsdr_spectrum_plan plan;
    uhsdr_spectrum_plan* d_plan;
    int C, N, L, F, fill;
    int D, Nd;               // zoom decimation (1: no zoom), ring samples per call N / D
    hipStream_t stream;
    float *teta, *avg, *carry;
    float2* zq;              // zoom ring samples of the current call [C][Nd]
    ZoomState zs;
    void* arena;
    size_t arena_bytes;
};

#define HIPCHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { uhsdr_set_error("%s: %s", #x, hipGetErrorString(e_)); return UHSDR_DEVICE_ERROR; } } while (0)

// LDS floats per wave: the padded frame; with auto I/Q correction also the product scratch and
// the per-call sums / factors behind it
template <int L>
static int spec_pitch_t(bool iq_auto) { return iq_auto ? SpecGeom<L>::PITCH : SpecGeom<L>::FRAME + 4; }
static int spec_pitch(int L, bool iq_auto)
{
    return L == 256 ? spec_pitch_t<256>(iq_auto) : (L == 512 ? spec_pitch_t<512>(iq_auto) : spec_pitch_t<1024>(iq_auto));
}

extern "C" uhsdr_status uhsdr_spectrum_reset(uhsdr_spectrum_handle h)
{
    if (!h) return UHSDR_ARGUMENT_ERROR;
    HIPCHK(hipMemsetAsync(h->arena, 0, h->arena_bytes, h->stream));   // sd.FFT_AVGData / iq_corr start zeroed
    if (h->D > 1)
    {
        // FreqShift_Approx oscillator starts at {I=0, Q=1} (freq_shift.c:48-49)
        float* ones = (float*)malloc(sizeof(float) * h->C);
        for (int i = 0; i < h->C; ++i) ones[i] = 1.0f;
        const hipError_t e = hipMemcpyAsync(h->zs.osc + h->C, ones, sizeof(float) * h->C, hipMemcpyHostToDevice, h->stream);
        if (e == hipSuccess) (void)hipStreamSynchronize(h->stream);
        free(ones);
        HIPCHK(e);
    }
    HIPCHK(hipStreamSynchronize(h->stream));
    h->fill = 0;
    return UHSDR_OK;
}

extern "C" uhsdr_status uhsdr_spectrum_create(const uhsdr_spectrum_config* cfg, int32_t C, int32_t N, void* stream,
                                              uhsdr_spectrum_handle* out)
{
    if (!cfg || !out || C <= 0 || N <= 0) { uhsdr_set_error("bad argument"); return UHSDR_ARGUMENT_ERROR; }
    *out = nullptr;
    uhsdr_spectrum_s* h = (uhsdr_spectrum_s*)calloc(1, sizeof(uhsdr_spectrum_s));
    uhsdr_status st = uhsdr_spectrum_plan_build(cfg, &h->plan);
    if (st != UHSDR_OK) { free(h); return st; }
    const int L = h->plan.fft_len;
    if ((L == 1024) != (h->plan.window_formula != 0))
    {
        free(h);
        uhsdr_set_error("window kind does not match fft_len %d", L);
        return UHSDR_UNSUPPORTED;
    }
    const int D = h->plan.magnify > 0 ? h->plan.zoom_decimation : 1, Nd = N / D;
    if (h->plan.magnify > 0 && h->plan.zoom_taps != ZOOM_TAPS)
    {
        free(h);
        uhsdr_set_error("zoom decimator with %d taps (kernel built for %d)", h->plan.zoom_taps, ZOOM_TAPS);
        return UHSDR_UNSUPPORTED;
    }
    if (N % BLK || (Nd % L && L % Nd))
    {
        free(h);
        uhsdr_set_error("frames_per_call %d: need a multiple of %d whose ring samples (frames / %d) are a multiple "
                        "or a divisor of fft_len %d", N, BLK, D, L);
        return UHSDR_LENGTH_ERROR;
    }
    h->C = C; h->N = N; h->L = L;
    h->D = D; h->Nd = Nd;
    h->F = Nd >= L ? Nd / L : 1;
    h->stream = (hipStream_t)stream;
    size_t fl = 0;
    auto take = [&](size_t n) { size_t o = fl; fl += (n + 63) & ~(size_t)63; return o; };
    const size_t o_teta = take((size_t)3 * C), o_avg = take((size_t)C * L), o_carry = take(Nd < L ? (size_t)C * 2 * L : 0);
    const bool zoom = D > 1;
    const size_t o_zq = take(zoom ? (size_t)C * 2 * Nd : 0), o_bqi = take(zoom ? (size_t)16 * C : 0),
                 o_bqq = take(zoom ? (size_t)16 * C : 0), o_di = take(zoom ? (size_t)(ZOOM_TAPS - 1) * C : 0),
                 o_dq = take(zoom ? (size_t)(ZOOM_TAPS - 1) * C : 0), o_osc = take(zoom ? (size_t)2 * C : 0);
    h->arena_bytes = fl * sizeof(float);
    if (hipMalloc(&h->arena, h->arena_bytes) != hipSuccess ||
        hipMalloc((void**)&h->d_plan, sizeof(uhsdr_spectrum_plan)) != hipSuccess)
    {
        uhsdr_set_error("hipMalloc failed (%zu bytes state)", h->arena_bytes);
        (void)uhsdr_spectrum_destroy(h);
        return UHSDR_DEVICE_ERROR;
    }
    float* A = (float*)h->arena;
    h->teta = A + o_teta; h->avg = A + o_avg; h->carry = A + o_carry;
    h->zq = (float2*)(A + o_zq);
    h->zs.bq_i = A + o_bqi; h->zs.bq_q = A + o_bqq; h->zs.dec_i = A + o_di; h->zs.dec_q = A + o_dq; h->zs.osc = A + o_osc;
    if (hipMemcpy(h->d_plan, &h->plan, sizeof(uhsdr_spectrum_plan), hipMemcpyHostToDevice) != hipSuccess)
    {
        uhsdr_set_error("plan upload failed");
        (void)uhsdr_spectrum_destroy(h);
        return UHSDR_DEVICE_ERROR;
    }
    const uhsdr_status rs = uhsdr_spectrum_reset(h);
    if (rs != UHSDR_OK) { (void)uhsdr_spectrum_destroy(h); return rs; }
    *out = h;
    return UHSDR_OK;
}

extern "C" uhsdr_status uhsdr_spectrum_process(uhsdr_spectrum_handle h, const int32_t* iq, float* mag, float* avg,
                                               int32_t* frames)
{
    if (!h || !iq) { uhsdr_set_error("null argument"); return UHSDR_ARGUMENT_ERROR; }
    const bool zoom = h->D > 1;
    if (zoom)
    {
        ZoomArgs za;
        za.plan = h->d_plan; za.iq = (const int2*)iq; za.zq = h->zq; za.teta = h->teta; za.s = h->zs;
        za.C = h->C; za.N = h->N;
        const dim3 zg((2 * h->C + 63) / 64), zb(64);      // two lanes per channel
        switch (h->D)
        {
        case 2: hipLaunchKernelGGL(spectrum_zoom<2>, zg, zb, 0, h->stream, za); break;
        case 4: hipLaunchKernelGGL(spectrum_zoom<4>, zg, zb, 0, h->stream, za); break;
        case 8: hipLaunchKernelGGL(spectrum_zoom<8>, zg, zb, 0, h->stream, za); break;
        case 16: hipLaunchKernelGGL(spectrum_zoom<16>, zg, zb, 0, h->stream, za); break;
        default: hipLaunchKernelGGL(spectrum_zoom<32>, zg, zb, 0, h->stream, za); break;
        }
        HIPCHK(hipGetLastError());
    }
    SpecArgs sa;
    sa.plan = h->d_plan; sa.iq = (const int2*)iq; sa.zq = h->zq;
    sa.teta = h->teta; sa.avg_state = h->avg; sa.carry = h->carry;
    sa.mag = mag; sa.avg = avg;
    sa.C = h->C; sa.N = h->Nd; sa.ld = h->Nd; sa.F = h->F; sa.fill0 = h->fill;
    const bool au = h->plan.iq_auto_correction != 0 && !zoom;   // zoom: corrected by spectrum_zoom
    sa.lds_pitch = spec_pitch(h->L, au);
    const size_t lds = sizeof(float) * (size_t)SPEC_WAVES * sa.lds_pitch;
    const dim3 grid((h->C + SPEC_WAVES - 1) / SPEC_WAVES), block(64 * SPEC_WAVES);
    const bool completes = h->fill + h->Nd >= h->L;
#define SPEC_LAUNCH3(LEN, AU, ZM) do { if (completes) hipLaunchKernelGGL((spectrum_frames<LEN, AU, ZM>), grid, block, lds, h->stream, sa); \
                                       else hipLaunchKernelGGL((spectrum_accumulate<LEN, AU, ZM>), grid, block, lds, h->stream, sa); } while (0)
#define SPEC_LAUNCH(LEN) do { if (zoom) SPEC_LAUNCH3(LEN, false, true); else if (au) SPEC_LAUNCH3(LEN, true, false); \
                              else SPEC_LAUNCH3(LEN, false, false); } while (0)
    switch (h->L)
    {
    case 256: SPEC_LAUNCH(256); break;
    case 512: SPEC_LAUNCH(512); break;
    default: SPEC_LAUNCH(1024); break;
    }
#undef SPEC_LAUNCH
#undef SPEC_LAUNCH3
    HIPCHK(hipGetLastError());
    const int done = (h->fill + h->Nd) / h->L;
    h->fill = (h->fill + h->Nd) % h->L;
    if (frames) *frames = done;
    return UHSDR_OK;
}

extern "C" uhsdr_status uhsdr_spectrum_get_plan(uhsdr_spectrum_handle h, uhsdr_spectrum_plan* plan)
{
    if (!h || !plan) return UHSDR_ARGUMENT_ERROR;
    memcpy(plan, &h->plan, sizeof *plan);
    return UHSDR_OK;
}

extern "C" uhsdr_status uhsdr_spectrum_destroy(uhsdr_spectrum_handle h)
{
    if (!h) return UHSDR_ARGUMENT_ERROR;
    (void)hipStreamSynchronize(h->stream);
    if (h->arena) (void)hipFree(h->arena);
    if (h->d_plan) (void)hipFree(h->d_plan);
    free(h);
    return UHSDR_OK;
}
